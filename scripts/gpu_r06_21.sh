# r06 GPU session 21: PMC of the session-frame pack in its final form (32-record tiles, virtual
# tiles) and of the CommitOffsetLite pack, rotated rows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r06_session32 CMD="scripts/bench_rows.py --no-cpu --rows session --steps 3 --warmup 1" KREGEX="sbe_enc_pack" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_session32.txt 2>&1 || { tail -20 gpurun_out/prof_r06_session32.txt; exit 1; }
TAG=r06_lite301f CMD="scripts/bench_rows.py --no-cpu --rows lite301 --steps 3 --warmup 1" KREGEX="sbe_enc_pack" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_lite301f.txt 2>&1 || { tail -20 gpurun_out/prof_r06_lite301f.txt; exit 1; }
cat gpurun_out/prof_r06_session32.txt gpurun_out/prof_r06_lite301f.txt
