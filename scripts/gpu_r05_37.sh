# r05 GPU session 37: reassembly scan + message table in one launch (frag_scan_msgs) — parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reassembly.py > gpurun_out/r05_37_tests.log 2>&1 || { tail -30 gpurun_out/r05_37_tests.log; exit 1; }
tail -1 gpurun_out/r05_37_tests.log
timeout -k 10 300 python -u scripts/ab_reasm.py abl/fr_unfused.so abl/fr_fused.so --rounds 7 > gpurun_out/r05_37_ab.log 2>&1 || { tail -20 gpurun_out/r05_37_ab.log; exit 1; }
grep reassemble gpurun_out/r05_37_ab.log
