# r05 GPU session 11: reassembly row, previous commit's build against the flat-copy build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/prev.so abl/base.so abl/noflat.so --rounds 7 > gpurun_out/r05_ab_fragflat2.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_reasm.py abl/prev.so abl/base.so abl/noflat.so --rounds 7 --clean >> gpurun_out/r05_ab_fragflat2.log 2>&1 &&
grep reassemble gpurun_out/r05_ab_fragflat2.log
