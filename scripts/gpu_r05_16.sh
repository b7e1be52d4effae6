# r05 GPU session 16: Order JSON row profile (kernel trace + PMC)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05_orderjson CMD="scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1" KREGEX="order_json" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_orderjson.txt 2>&1 || { tail -20 gpurun_out/prof_r05_orderjson.txt; exit 1; }
cat gpurun_out/prof_r05_orderjson.txt | tail -60
