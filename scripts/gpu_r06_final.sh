# r06 final evidence on the round's tree: GPU suite, smoke, the default bench (rotated inputs),
# the bench under rocprofv3 --kernel-trace --stats (one process), PMC of the rotated headline,
# every row (rotated where the row fits the MALL), PMC of configs 3 and 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail -20 gpurun_out/r06_smoke.log; exit 1; }
tail -1 gpurun_out/r06_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r06_bench.log 2> gpurun_out/r06_bench.err || { tail -5 gpurun_out/r06_bench.err; exit 1; }
cut -c1-300 gpurun_out/r06_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06_benchtrace -o run --output-format csv -- python3 bench.py --no-config5 --no-cpu-baseline > gpurun_out/r06_bench_traced.log 2> gpurun_out/r06_bench_traced.err || { tail -5 gpurun_out/r06_bench_traced.err; exit 1; }
TAG=r06_fixed256 bash scripts/gpu_profile.sh > gpurun_out/prof_r06_fixed256.txt 2>&1 || { tail -20 gpurun_out/prof_r06_fixed256.txt; exit 1; }
timeout -k 10 900 python -u scripts/bench_rows.py > gpurun_out/r06_rows.jsonl 2> gpurun_out/r06_rows.err || { tail -5 gpurun_out/r06_rows.err; exit 1; }
cut -c1-150 gpurun_out/r06_rows.jsonl
TAG=r06_config3 CMD="scripts/bench_rows.py --no-cpu --rows mixed --steps 5 --warmup 1" KREGEX="sbe_decode_kernel" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_config3.txt 2>&1 || { tail -20 gpurun_out/prof_r06_config3.txt; exit 1; }
TAG=r06_config4 CMD="scripts/bench_rows.py --no-cpu --rows var --steps 3 --warmup 1" KREGEX="sbe_enc_pack|sbe_decode_kernel|sbe_enc_sums" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_config4.txt 2>&1 || { tail -20 gpurun_out/prof_r06_config4.txt; exit 1; }
echo done
