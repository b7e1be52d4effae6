# r06 GPU session 5: the pack loop chosen per launch (virtual tiles when a tile's last window is
# under 60 % full): GPU suite, A/B against the tile-loop build on rotated inputs; reassembly row with
# and without the big-message list
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_5_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06_5_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06_5_gpu_tests.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/big2.so abl/sel.so abl/vt0.so --work fixed,var,session,lite301,lite201 --rotate 3 --rounds 5 > gpurun_out/r06_ab_sel.log 2>&1 || { tail -20 gpurun_out/r06_ab_sel.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_sel.log
timeout -k 10 300 python -u scripts/ab_reasm.py abl/ntl0.so abl/nobig.so abl/sel.so --rounds 7 > gpurun_out/r06_ab_reasm_nobig.log 2>&1 || { tail -20 gpurun_out/r06_ab_reasm_nobig.log; exit 1; }
tail -3 gpurun_out/r06_ab_reasm_nobig.log
