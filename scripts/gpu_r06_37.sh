# r06 GPU session 37: decode staging loads nontemporal (product) against the default cache policy,
# rotated inputs (verdict r5 item 1: the load policy decided on cache-cold data) and warm (one set)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_rows.py abl/d_ntl1.so abl/d_ntl0.so --work fixed,mixed,session,lite201 --rotate 3 --rounds 7 > gpurun_out/r06_ab_decntl_rot.log 2>&1 || { tail -20 gpurun_out/r06_ab_decntl_rot.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_decntl_rot.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/d_ntl1.so abl/d_ntl0.so --work fixed,var --rotate 1 --rounds 5 > gpurun_out/r06_ab_decntl_warm.log 2>&1 || { tail -20 gpurun_out/r06_ab_decntl_warm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_decntl_warm.log
