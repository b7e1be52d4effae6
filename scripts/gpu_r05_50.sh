# r05 GPU session 50: every row on the round's last tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_rows.py > gpurun_out/r05_rows4.jsonl 2> gpurun_out/r05_rows4.err || { tail -5 gpurun_out/r05_rows4.err; exit 1; }
cut -c1-120 gpurun_out/r05_rows4.jsonl
