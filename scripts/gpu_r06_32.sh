# r06 GPU session 32: the over-320 B decode shape's window (config 4's 387-B average), 13 KiB
# (product: two windows a tile) against 25 / 27 KiB (most tiles in one window); session frames on
# the 20 KiB wide window again
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_rows.py abl/dw12.so abl/dl25.so abl/dl27.so abl/dw20.so --work var,session --rotate 1 --rounds 5 > gpurun_out/r06_ab_declarge.log 2>&1 || { tail -20 gpurun_out/r06_ab_declarge.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_declarge.log
