# r06 GPU session 31: the 257-320 B decode shape's window, 12 (product) / 18 / 20 KiB, on session
# frames (280 B) and fixed-size TopicMessages of 300 and 320 B (payloads 187 / 207 B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_rows.py abl/dw12.so abl/dw18.so abl/dw20.so --work session,fixedp187,fixedp207 --rotate 3 --rounds 7 > gpurun_out/r06_ab_decsess2.log 2>&1 || { tail -20 gpurun_out/r06_ab_decsess2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_decsess2.log
