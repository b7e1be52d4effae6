# r05 GPU session 3: frag_copy knobs (unaligned loads, metadata prefetch) on the reassembly row;
# the wide decode window at 12 / 13 / 14 KiB (config 4, session frames); the host-API binary with
# the BatchingParser test; the BatchingParser bench at 100-fragment polls
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/base.so abl/fcua.so abl/fcpf.so abl/fcboth.so --rounds 7 > gpurun_out/r05_ab_fragcopy.log 2>&1 &&
tail -5 gpurun_out/r05_ab_fragcopy.log &&
timeout -k 10 500 python -u scripts/ab_rows.py abl/base.so abl/w13.so abl/w14.so --work var,session --rounds 5 > gpurun_out/r05_ab_decwide.log 2>&1 &&
tail -8 gpurun_out/r05_ab_decwide.log &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_api.py -x -v --timeout 280 -k host_api_binary > gpurun_out/r05_host_api.log 2>&1 &&
tail -3 gpurun_out/r05_host_api.log &&
timeout -k 10 300 scripts/batching_parser_bench > gpurun_out/r05_batching_parser.log 2>&1 &&
cat gpurun_out/r05_batching_parser.log
