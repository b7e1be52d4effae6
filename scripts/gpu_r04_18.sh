# r04 GPU session 18: frag_copy with non-temporal copies and / or one load a chunk (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/base.so abl/fcnt.so abl/fcsh.so abl/fcntsh.so > gpurun_out/r04_ab_fragcopy.log 2>&1
