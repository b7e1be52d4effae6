# r04 GPU session 6: virtual-tile pack (every window full): parity tests, then A/B against the
# tile-aligned loop on every encode row
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python scripts/ab_rows.py abl/tile.so abl/vt.so --work fixed,var,session,lite301,lite201 --rounds 5 > gpurun_out/ab_r04_vt.log 2>&1 || exit 1
cat gpurun_out/ab_r04_vt.log
