# r04 GPU session 9: lane_u64 sign-extension fix; the guarded VT build on config 5, the whole GPU
# suite (virtual-tile pack, serve kernel, host mirror), then A/B of the tile and VT pack loops
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/vt_debug.py abl/vtguard.so 134217728 > gpurun_out/vt_debug2.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_rows.py abl/tile.so abl/vt.so --work fixed,var,session,lite301,lite201 --rounds 5 > gpurun_out/ab_r04_vt.log 2>&1
