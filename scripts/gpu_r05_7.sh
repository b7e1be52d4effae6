# r05 GPU session 7: pack cost per byte by record size (fixed payloads 143 / 276 / 400 B against
# config 4's variable records), the phase profile, 64-record tiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_rows.py abl/base.so abl/tm64.so --work fixed,fixedp143,fixedp276,fixedp400,var --rounds 5 > gpurun_out/r05_ab_packsize.log 2>&1 &&
tail -12 gpurun_out/r05_ab_packsize.log &&
timeout -k 10 300 python -u scripts/ab_rows.py abl/ph.so --work fixedp143,fixedp276,var --rounds 1 --phases --no-check > gpurun_out/r05_pack_phases.log 2>&1 &&
grep phases gpurun_out/r05_pack_phases.log
