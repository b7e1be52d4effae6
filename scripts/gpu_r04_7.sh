# r04 GPU session 7: the small-batch serve kernel: parity (C ABI + host mirror with and without
# it), then host-mirror latency with it (default: batches up to 256 records), up to 4096, and off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_serve.py tests/test_gpu_host_api.py "tests/test_gpu_parity.py::test_encode_input_offsets_past_2gib" -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_serve_tests.log 2>&1 &&
timeout -k 10 240 scripts/host_latency > gpurun_out/r04_host_latency_serve.log 2>&1 &&
AERON_AMD_SERVE_RECORDS=4096 timeout -k 10 120 scripts/host_latency 1024 > gpurun_out/r04_host_latency_serve4096.log 2>&1 &&
AERON_AMD_SERVE_RECORDS=4096 timeout -k 10 120 scripts/host_latency 4096 >> gpurun_out/r04_host_latency_serve4096.log 2>&1 &&
AERON_AMD_SERVE_RECORDS=0 AERON_AMD_SERVE_WIDE_RECORDS=0 timeout -k 10 240 scripts/host_latency > gpurun_out/r04_host_latency_noserve.log 2>&1 &&
timeout -k 10 240 python -u scripts/bench_host_inclusive.py > gpurun_out/r04_host_inclusive.log 2>&1
