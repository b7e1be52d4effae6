# r05 GPU session 15: frag_copy chunks a lane per step (4 / 8 / 16) with one unaligned load a chunk
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/base.so abl/u8.so abl/u16.so --rounds 7 > gpurun_out/r05_ab_fcu.log 2>&1 &&
grep reassemble gpurun_out/r05_ab_fcu.log
