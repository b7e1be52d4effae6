# r05 GPU session 46: the GPU suite and smoke on the round's last tree (after the include clean-up)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_gpu_tests_last.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_last.log; exit 1; }
tail -1 gpurun_out/r05_gpu_tests_last.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_last.log 2>&1 || { tail -20 gpurun_out/r05_smoke_last.log; exit 1; }
tail -1 gpurun_out/r05_smoke_last.log
timeout -k 10 400 python -u bench.py --steps 50 > gpurun_out/r05_bench_last.log 2> gpurun_out/r05_bench_last.err || { tail -5 gpurun_out/r05_bench_last.err; exit 1; }
cut -c1-300 gpurun_out/r05_bench_last.log
