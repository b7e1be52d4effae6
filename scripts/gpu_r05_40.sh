# r05 GPU session 40: pack staged-input loads nontemporal (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python scripts/ab_rows.py abl/pk_base.so abl/pk_ntl.so --work fixed,var,session,lite301,lite201 --rounds 5 > gpurun_out/r05_40_ab.log 2>&1 || { tail -20 gpurun_out/r05_40_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05_40_ab.log | tail -10
