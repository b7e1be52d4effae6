# r06 GPU session 15: 32-record tiles (two lanes a record) for the session-frame and
# OrderRequestLite layouts against 64, now that the pack loop is chosen per launch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_rows.py abl/rpt64.so abl/rpt32.so --work session,lite201 --rotate 3 --rounds 7 > gpurun_out/r06_ab_rpt.log 2>&1 || { tail -20 gpurun_out/r06_ab_rpt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_rpt.log
