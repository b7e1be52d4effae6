# r05 GPU session 6: BatchingParser bench, steady state (one parser per setting, warm-up pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 scripts/batching_parser_bench > gpurun_out/r05_batching_parser_4.log 2>&1 && cat gpurun_out/r05_batching_parser_4.log
