# r06 GPU session 14: PMC of the session-frame and CommitOffsetLite packs (rotated rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r06_session CMD="scripts/bench_rows.py --no-cpu --rows session --steps 5 --warmup 1" KREGEX="sbe_enc_pack|sbe_decode_kernel" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_session.txt 2>&1 || { tail -20 gpurun_out/prof_r06_session.txt; exit 1; }
tail -12 gpurun_out/prof_r06_session.txt
TAG=r06_lite301 CMD="scripts/bench_rows.py --no-cpu --rows lite301 --steps 5 --warmup 1" KREGEX="sbe_enc_pack|sbe_decode_kernel" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_lite301.txt 2>&1 || { tail -20 gpurun_out/prof_r06_lite301.txt; exit 1; }
tail -12 gpurun_out/prof_r06_lite301.txt
