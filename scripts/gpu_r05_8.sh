# r05 GPU session 8: pack knobs for records over 256 B: store rows 6-8 behind a uniform branch,
# no rebalance up to 13 chunks a lane, 64-record tiles, both
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/ab_rows.py abl/base.so abl/r5.so abl/nr.so abl/tm64.so abl/tm64r5.so --work fixed,fixedp276,var --rounds 5 > gpurun_out/r05_ab_packknobs.log 2>&1 &&
tail -15 gpurun_out/r05_ab_packknobs.log
