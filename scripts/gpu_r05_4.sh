# r05 GPU session 4: the GPU suite on the tree with the 13 KiB large-record decode window, unaligned
# frag_copy loads and the BatchingParser; then the BatchingParser bench (pool-backed batches), and
# one setting traced (AERON_AMD_TRACE=1: the decode thread's per-batch phases)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gpu_tests_2.log 2>&1 || { tail -40 gpurun_out/r05_gpu_tests_2.log; exit 1; }
tail -3 gpurun_out/r05_gpu_tests_2.log
timeout -k 10 300 scripts/batching_parser_bench > gpurun_out/r05_batching_parser_2.log 2>&1 && cat gpurun_out/r05_batching_parser_2.log &&
AERON_AMD_TRACE=1 timeout -k 10 120 scripts/batching_parser_bench 8192 > gpurun_out/r05_bp_trace.log 2> gpurun_out/r05_bp_trace.err && tail -5 gpurun_out/r05_bp_trace.err
