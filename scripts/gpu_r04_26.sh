# r04 GPU session 26: confirm the mid decode window at 14 / 15 / 16 KiB (config 3), and the wide
# window at 10 / 12 / 14 / 16 KiB (config 4, session frames) (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab_rows.py abl/base.so abl/m15.so abl/m16.so --work mixed,fixed --rounds 9 > gpurun_out/r04_ab_decmid2.log 2>&1 &&
timeout -k 10 500 python -u scripts/ab_rows.py abl/base.so abl/w10.so abl/w14.so abl/w16.so --work var,session --rounds 5 > gpurun_out/r04_ab_decwide.log 2>&1
