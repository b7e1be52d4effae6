# r05 GPU session 9: pack windows of two-lane records capped at 8 chunks a lane; rebalance T by
# loop iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python -u scripts/ab_rows.py abl/base.so abl/tp.so abl/lc.so abl/tplc.so --work fixed,fixedp276,fixedp400,var,session --rounds 5 > gpurun_out/r05_ab_packwin.log 2>&1 &&
tail -20 gpurun_out/r05_ab_packwin.log
