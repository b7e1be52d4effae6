# r05 GPU session 39: frag_copy with nt stores: nontemporal source loads, 2 / 8 chunks a lane per step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/fc_base.so abl/fc_ntl.so abl/fc_u2.so abl/fc_u8.so --rounds 7 > gpurun_out/r05_39_ab.log 2>&1 || { tail -20 gpurun_out/r05_39_ab.log; exit 1; }
grep reassemble gpurun_out/r05_39_ab.log
