# r05 GPU session 26: full GPU suite, smoke and the default bench on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_gpu_tests_3.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_3.log; exit 1; }
tail -2 gpurun_out/r05_gpu_tests_3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_3.log 2>&1 || { tail -20 gpurun_out/r05_smoke_3.log; exit 1; }
tail -2 gpurun_out/r05_smoke_3.log
timeout -k 10 300 python bench.py > gpurun_out/r05_bench_3.log 2>&1 || { tail -20 gpurun_out/r05_bench_3.log; exit 1; }
tail -1 gpurun_out/r05_bench_3.log | cut -c1-600
