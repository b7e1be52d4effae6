# r05 GPU session 33: every row (bench_rows) on the current tree + the Order JSON profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_rows.py > gpurun_out/r05_rows2.jsonl 2> gpurun_out/r05_rows2.err || { tail -5 gpurun_out/r05_rows2.err; exit 1; }
cut -c1-250 gpurun_out/r05_rows2.jsonl
TAG=r05_orderjson3 CMD="scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1" KREGEX="order_json" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_orderjson3.txt 2>&1 || { tail -20 gpurun_out/prof_r05_orderjson3.txt; exit 1; }
