# r04 GPU session 10: virtual tiles in round-robin chunks of CT tiles: guarded build on config 5,
# the whole GPU suite (CT = 4), then A/B of the tile loop against CT = contiguous, 1, 2, 4, 8
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/vt_debug.py abl/vtguard.so 134217728 > gpurun_out/vt_debug3.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python -u scripts/ab_rows.py abl/tile.so abl/vtc0.so abl/vtc1.so abl/vtc2.so abl/vtc4.so abl/vtc8.so --work fixed,var,session,lite301,lite201 --rounds 5 > gpurun_out/ab_r04_vtc.log 2>&1
