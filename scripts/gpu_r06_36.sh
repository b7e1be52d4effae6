# r06 GPU session 36: virtual-tile loop work split on rotated inputs: one contiguous record range
# per workgroup (product) against chunks of 4 / 16 / 64 tiles dealt round robin (config 4, session)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/ab_rows.py abl/p_base.so abl/p_vc4.so abl/p_vc16.so abl/p_vc64.so --work var,session --rotate 1 --rounds 5 > gpurun_out/r06_ab_vtchunk.log 2>&1 || { tail -20 gpurun_out/r06_ab_vtchunk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_vtchunk.log
