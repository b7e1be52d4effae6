# r05 GPU session 2: the 15 KiB mid decode window (config 3) against the 14 KiB default, A/B in one process
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/ab_rows.py abl/base.so abl/m15.so --work mixed,fixed --rounds 9 > gpurun_out/r05_ab_decmid.log 2>&1
tail -8 gpurun_out/r05_ab_decmid.log
