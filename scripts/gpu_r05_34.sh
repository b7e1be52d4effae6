# r05 GPU session 34: final evidence on the round's tree: the GPU suite, smoke, the default bench,
# rocprofv3 kernel trace + PMC of the headline, config 3, config 4 and reassembly
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_gpu_tests_final.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/r05_gpu_tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_final.log 2>&1 || { tail -20 gpurun_out/r05_smoke_final.log; exit 1; }
tail -1 gpurun_out/r05_smoke_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_final.log 2> gpurun_out/r05_bench_final.err || { tail -5 gpurun_out/r05_bench_final.err; exit 1; }
TAG=r05_fixed256f bash scripts/gpu_profile.sh > gpurun_out/prof_r05_fixed256f.txt 2>&1 || { tail -20 gpurun_out/prof_r05_fixed256f.txt; exit 1; }
TAG=r05_config3f CMD="scripts/bench_rows.py --no-cpu --rows mixed --steps 5 --warmup 1" KREGEX="sbe_decode_kernel" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_config3f.txt 2>&1 || { tail -20 gpurun_out/prof_r05_config3f.txt; exit 1; }
TAG=r05_config4f CMD="scripts/bench_rows.py --no-cpu --rows var --steps 3 --warmup 1" KREGEX="sbe_enc_pack|sbe_decode_kernel|sbe_enc_sums" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_config4f.txt 2>&1 || { tail -20 gpurun_out/prof_r05_config4f.txt; exit 1; }
TAG=r05_reasmf CMD="scripts/bench_rows.py --no-cpu --rows reassemble --steps 5 --warmup 1" KREGEX="frag_" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_reasmf.txt 2>&1 || { tail -20 gpurun_out/prof_r05_reasmf.txt; exit 1; }
cut -c1-700 gpurun_out/r05_bench_final.log
