# r04 GPU session 20: the host mirror with the new worker pool: its GPU tests, then the per-call
# latency table (serve kernel on; spinning helpers on and off), then the phase trace of 1 K-record calls
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_host_api.py tests/test_gpu_serve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_host_tests_pool.log 2>&1 &&
timeout -k 10 240 scripts/host_latency > gpurun_out/r04_host_latency_pool.log 2>&1 &&
AERON_AMD_SPIN_US=0 timeout -k 10 240 scripts/host_latency > gpurun_out/r04_host_latency_pool_nospin.log 2>&1 &&
AERON_AMD_TRACE=1 timeout -k 10 120 scripts/host_latency 1024 > gpurun_out/r04_trace_1024_pool.log 2> gpurun_out/r04_trace_1024_pool.err
