# r05 GPU session 42: pack lengths / timestamps loaded nontemporal (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python scripts/ab_rows.py abl/pk_cur.so abl/pk_ntl2.so --work fixed,var,lite201 --rounds 5 > gpurun_out/r05_42_ab.log 2>&1 || { tail -20 gpurun_out/r05_42_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05_42_ab.log | tail -6
