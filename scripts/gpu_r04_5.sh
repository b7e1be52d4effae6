# r04 GPU session 5: pack ablations (timing only, wrong bytes) on fixed / var, then the PMC
# profiles of the headline and configs 3 / 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_rows.py abl/ackfast.so abl/nocompose.so abl/nofix.so abl/nolit.so abl/nostage.so abl/nogroups.so --work fixed,var --rounds 3 --no-check > gpurun_out/ab_r04_abl.log 2>&1 || exit 1
cat gpurun_out/ab_r04_abl.log
bash scripts/gpu_r04_3.sh
