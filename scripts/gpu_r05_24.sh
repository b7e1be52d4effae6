# r05 GPU session 24: Order JSON row profile after the LDS-staged sizing / block-sum offsets / no-scratch selects
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r05_orderjson2 CMD="scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1" KREGEX="order_json" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_orderjson2.txt 2>&1 || { tail -20 gpurun_out/prof_r05_orderjson2.txt; exit 1; }
cat gpurun_out/prof_r05_orderjson2.txt | tail -45
