# r05 GPU session 10: frag_copy's flat stream copy (in-order batches) against the per-group copy,
# on the row's stream and on a stream without messages inside groups; the reassembly GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/base.so abl/noflat.so --rounds 7 > gpurun_out/r05_ab_fragflat.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_reasm.py abl/base.so abl/noflat.so --rounds 7 --clean >> gpurun_out/r05_ab_fragflat.log 2>&1 &&
grep reassemble gpurun_out/r05_ab_fragflat.log &&
timeout -k 10 300 python -u -m pytest tests/test_reassembly.py -x -q --timeout 120 -m gpu > gpurun_out/r05_reasm_tests.log 2>&1 ; tail -3 gpurun_out/r05_reasm_tests.log
