# r06 GPU session 9: PMC of the group decode kernel (g4) and the one-wave mid kernel (g0) on config 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in g0 g4; do
  TAG=r06_grp_$L CMD="scripts/ab_rows.py abl/$L.so --work mixed --rounds 1 --steps 5 --no-check" KREGEX="sbe_decode" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_grp_$L.txt 2>&1 || { tail -20 gpurun_out/prof_r06_grp_$L.txt; exit 1; }
  cat gpurun_out/prof_r06_grp_$L.txt
done
