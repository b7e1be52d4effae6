# r05 GPU session 48: final evidence on the round's last tree (default-policy pack loads): GPU suite, smoke, bench, headline profile
# rocprofv3 kernel trace + PMC of the headline, config 3, config 4 and reassembly
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_gpu_tests_final3.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/r05_gpu_tests_final3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_final3.log 2>&1 || { tail -20 gpurun_out/r05_smoke_final.log; exit 1; }
tail -1 gpurun_out/r05_smoke_final3.log
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_final3.log 2> gpurun_out/r05_bench_final3.err || { tail -5 gpurun_out/r05_bench_final3.err; exit 1; }
TAG=r05_fixed256h bash scripts/gpu_profile.sh > gpurun_out/prof_r05_fixed256h.txt 2>&1 || { tail -20 gpurun_out/prof_r05_fixed256h.txt; exit 1; }
cut -c1-700 gpurun_out/r05_bench_final3.log
