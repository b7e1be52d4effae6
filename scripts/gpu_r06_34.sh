# r06 GPU session 34: decode windows on rotated inputs: the 113-204 B shape (config 3) at 15 KiB
# (product) / 16 / 17 / 18 KiB, and the over-320 B shape (OrderRequestLite 333 B, config 4 387 B)
# at 13 KiB (product) / 22 KiB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_rows.py abl/d_base.so abl/d_mid16.so abl/d_mid17.so abl/d_mid18.so --work mixed --rotate 3 --rounds 7 > gpurun_out/r06_ab_decmid6.log 2>&1 || { tail -20 gpurun_out/r06_ab_decmid6.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_decmid6.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/d_base.so abl/d_lg22.so --work lite201,var --rotate 1 --rounds 5 > gpurun_out/r06_ab_declg22.log 2>&1 || { tail -20 gpurun_out/r06_ab_declg22.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_declg22.log
