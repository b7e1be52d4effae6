# r05 GPU session 13: frag_copy with the next group's metadata prefetched and fewer copy waves,
# each looping over several groups (grid cap 512 / 1024 / 2048 blocks of four waves)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/gapruns.so abl/pf512.so abl/pf1k.so abl/pf2k.so --rounds 7 > gpurun_out/r05_ab_fcpf.log 2>&1 &&
grep reassemble gpurun_out/r05_ab_fcpf.log &&
timeout -k 10 400 python -u scripts/ab_rows.py abl/prev.so abl/dot4.so --work mixed,fixed --rounds 9 > gpurun_out/r05_ab_dot4.log 2>&1 &&
tail -4 gpurun_out/r05_ab_dot4.log
