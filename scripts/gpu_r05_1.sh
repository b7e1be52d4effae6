# r05 GPU session 1: the whole GPU suite (gather-mock harness rebuilt: bounded waits, main-thread
# allocation, sized gather), then the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r05_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r05_gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r05_bench.log 2> gpurun_out/r05_bench.err || { tail -5 gpurun_out/r05_bench.err; exit 1; }
cat gpurun_out/r05_bench.log
