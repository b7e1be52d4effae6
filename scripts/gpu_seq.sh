# seqnum parity tests first (new code), then the whole GPU suite, then a bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_seqnum.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_seq.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/pytest_seq.log | tail -30
echo "seq rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
[ $rc -eq 0 ] && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
