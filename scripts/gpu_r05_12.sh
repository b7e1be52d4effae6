# r05 GPU session 12: frag_copy's gapped messages (a single inside the group) as runs of fragments
# loaded 64 at a time, against the per-fragment loop; the reassembly GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/prev.so abl/gapruns.so --rounds 7 > gpurun_out/r05_ab_gapruns.log 2>&1 &&
grep reassemble gpurun_out/r05_ab_gapruns.log &&
timeout -k 10 300 python -u -m pytest tests/test_reassembly.py -x -q --timeout 120 -m gpu > gpurun_out/r05_reasm_tests2.log 2>&1 ; tail -3 gpurun_out/r05_reasm_tests2.log
