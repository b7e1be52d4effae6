# r06 GPU session 23: MATERIALIZE launches under the kernel trace, and their PMC (wave-staged copy)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r06_materialize CMD="scripts/bench_rows.py --no-cpu --rows materialize --steps 5 --warmup 1" KREGEX="mat_" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_materialize.txt 2>&1 || { tail -20 gpurun_out/prof_r06_materialize.txt; exit 1; }
cat gpurun_out/prof_r06_materialize.txt
