# r06 GPU session 30: session-frame decode window (the 257-320 B shape): 12 KiB (product) against
# 18 KiB (a 64-frame tile whole in one window), 9 and 10 KiB (two windows, more workgroups per CU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/ab_rows.py abl/dw12.so abl/dw18.so abl/dw9.so abl/dw10.so --work session --rotate 3 --rounds 7 > gpurun_out/r06_ab_decsess.log 2>&1 || { tail -20 gpurun_out/r06_ab_decsess.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_decsess.log
