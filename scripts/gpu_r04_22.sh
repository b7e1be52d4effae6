# r04 GPU session 22: frag_copy grid cap (blocks of 4 waves looping over the message groups) and
# chunks per lane per step (A/B, reassembly row)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/base.so abl/b512.so abl/b1024.so abl/b2048.so abl/u2.so abl/u2b1024.so > gpurun_out/r04_ab_fraggrid.log 2>&1
