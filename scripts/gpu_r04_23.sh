# r04 GPU session 23: frag_copy with one load a chunk (the second block from the next lane, DPP) at 4 / 6 / 8
# chunks a lane per step, against two loads a chunk at 4 and 8 (A/B, reassembly row)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/base.so abl/d4.so abl/d6.so abl/d8.so abl/u8.so > gpurun_out/r04_ab_fragdpp.log 2>&1
