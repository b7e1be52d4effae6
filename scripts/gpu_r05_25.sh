# r05 GPU session 25: config-4 decode ablation — the staged-chunk _sequence_number classification skipped
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/ab_rows.py abl/base.so abl/noclass.so --work var,mixed --rounds 5 > gpurun_out/r05_25_ab.log 2>&1 || { tail -20 gpurun_out/r05_25_ab.log; exit 1; }
tail -12 gpurun_out/r05_25_ab.log
