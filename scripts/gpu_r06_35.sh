# r06 GPU session 35: OrderRequestLite pack on the virtual-tile loop with 32- and 64-record tiles
# against the product (tile loop, 64-record tiles); rotated inputs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_rows.py abl/p_base.so abl/p_l3vt32.so abl/p_l3vt64.so --work lite201 --rotate 3 --rounds 7 > gpurun_out/r06_ab_l3vt.log 2>&1 || { tail -20 gpurun_out/r06_ab_l3vt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_l3vt.log
