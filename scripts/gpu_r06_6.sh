# r06 GPU session 6: BatchingParser with a batch queue, spinning waits and resumable delivery
# (host-API binary test, the reference-granularity bench); reassembly with the out-of-line
# singles lookup (tests + row A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_host_api.py tests/test_reassembly.py > gpurun_out/r06_6_tests.log 2>&1 || { tail -30 gpurun_out/r06_6_tests.log; exit 1; }
tail -1 gpurun_out/r06_6_tests.log
timeout -k 10 300 scripts/batching_parser_bench > gpurun_out/r06_host_latency.log 2>&1 || { tail -20 gpurun_out/r06_host_latency.log; exit 1; }
cut -c1-330 gpurun_out/r06_host_latency.log
timeout -k 10 300 python -u scripts/ab_reasm.py abl/ntl0.so abl/sel.so abl/sel2.so --rounds 7 > gpurun_out/r06_ab_reasm_sel2.log 2>&1 || { tail -20 gpurun_out/r06_ab_reasm_sel2.log; exit 1; }
tail -3 gpurun_out/r06_ab_reasm_sel2.log
