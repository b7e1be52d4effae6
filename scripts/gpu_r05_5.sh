# r05 GPU session 5: BatchingParser with results built at delivery (host-API test + bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_api.py -x -v --timeout 280 -k host_api_binary > gpurun_out/r05_host_api_2.log 2>&1 &&
tail -3 gpurun_out/r05_host_api_2.log &&
timeout -k 10 300 scripts/batching_parser_bench > gpurun_out/r05_batching_parser_3.log 2>&1 && cat gpurun_out/r05_batching_parser_3.log &&
AERON_AMD_TRACE=1 timeout -k 10 120 scripts/batching_parser_bench 8192 > gpurun_out/r05_bp_trace2.log 2> gpurun_out/r05_bp_trace2.err && tail -4 gpurun_out/r05_bp_trace2.err
