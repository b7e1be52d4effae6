# r05 GPU session 43: decode staging loads with the default policy instead of nontemporal (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python scripts/ab_rows.py abl/dec_cur.so abl/dec_plain.so --work fixed,mixed,var --rounds 5 > gpurun_out/r05_43_ab.log 2>&1 || { tail -20 gpurun_out/r05_43_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05_43_ab.log | tail -6
