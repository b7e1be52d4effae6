# r04 GPU session 24: the wide decode kernel (12 KiB windows: config 4, session frames, OrderRequestLite)
# compiled for 4 waves per SIMD (<= 128 VGPRs, so the LDS's 13 workgroups per CU fit) against 3 (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/ab_rows.py abl/base.so abl/mw4.so --work var,session,lite201 --rounds 5 > gpurun_out/r04_ab_decwide_w4.log 2>&1
