# r06 GPU session 16: 32-record session-frame tiles in the product build: session, serve, host
# pipeline / API and parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_serve.py tests/test_gpu_parity.py tests/test_gpu_host_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_16_tests.log 2>&1 || { tail -30 gpurun_out/r06_16_tests.log; exit 1; }
tail -1 gpurun_out/r06_16_tests.log
