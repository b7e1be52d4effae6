# r06 GPU session 4: reassembly with the nearer-boundary singles count (tests + row A/B against r05),
# then the virtual-tile pack loop (contiguous ranges / 4-tile chunks) against the tile loop on
# rotated inputs, every layout and record sizes 256 / 389 / 513 B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_reassembly.py > gpurun_out/r06_4_tests.log 2>&1 || { tail -30 gpurun_out/r06_4_tests.log; exit 1; }
grep -h "reassembly 1 M\|passed\|failed" gpurun_out/r06_4_tests.log | tail -3
timeout -k 10 300 python -u scripts/ab_reasm.py abl/ntl0.so abl/big2.so --rounds 7 > gpurun_out/r06_ab_reasm_big2.log 2>&1 || { tail -20 gpurun_out/r06_ab_reasm_big2.log; exit 1; }
tail -2 gpurun_out/r06_ab_reasm_big2.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/big2.so abl/vt0.so abl/vt4.so --work fixed,var,session,lite301,lite201,fixedp389,fixedp513 --rotate 3 --rounds 5 > gpurun_out/r06_ab_vt.log 2>&1 || { tail -20 gpurun_out/r06_ab_vt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_vt.log
