# r04 GPU session 25: the mid decode window (batches of 112-204 B records on average: config 3) at
# 13 / 14 / 15 KiB (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab_rows.py abl/base.so abl/m13.so abl/m15.so --work mixed --rounds 7 > gpurun_out/r04_ab_decmid.log 2>&1
