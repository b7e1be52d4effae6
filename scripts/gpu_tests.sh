# The GPU test suite (parity at small sizes, full-size configs, host mirror), then a bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60
echo "pytest rc=$rc"
[ $rc -eq 0 ] && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
