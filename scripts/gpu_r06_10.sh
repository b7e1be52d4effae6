# r06 GPU session 10: group decode without the in-kernel one-wave fallback (records outside the
# shared window parsed from HBM): decode tests, A/B on config 3, PMC of g4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_seqnum.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_10_tests.log 2>&1 || { tail -30 gpurun_out/r06_10_tests.log; exit 1; }
tail -1 gpurun_out/r06_10_tests.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/g0.so abl/g2.so abl/g3.so abl/g4.so --work mixed --rotate 3 --rounds 7 > gpurun_out/r06_ab_group3.log 2>&1 || { tail -20 gpurun_out/r06_ab_group3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_group3.log
TAG=r06_grp3_g4 CMD="scripts/ab_rows.py abl/g4.so --work mixed --rounds 1 --steps 5 --no-check" KREGEX="sbe_decode" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_grp3_g4.txt 2>&1 || { tail -20 gpurun_out/prof_r06_grp3_g4.txt; exit 1; }
tail -6 gpurun_out/prof_r06_grp3_g4.txt
