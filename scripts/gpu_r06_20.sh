# r06 GPU session 20: pack loop phase shares on the final tree (-DSBE_PACK_PHASES build) for every
# layout, rotated inputs: where a wave's time goes per window for the weak pack rows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab_rows.py abl/ph.so --work fixed,var,session,lite301,lite201 --rounds 1 --rotate 3 --phases > gpurun_out/r06_pack_phases.log 2>&1 || { tail -20 gpurun_out/r06_pack_phases.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_pack_phases.log
