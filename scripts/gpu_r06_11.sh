# r06 GPU session 11: persistent group decode (next group's bytes in registers during the parse),
# 2 / 3 / 4 tiles a workgroup, against the one-wave mid kernel; decode tests; PMC of the default (g3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_seqnum.py tests/test_gpu_materialize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_11_tests.log 2>&1 || { tail -30 gpurun_out/r06_11_tests.log; exit 1; }
tail -1 gpurun_out/r06_11_tests.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/g0.so abl/g2.so abl/g3.so abl/g4.so --work mixed --rotate 3 --rounds 7 > gpurun_out/r06_ab_group4.log 2>&1 || { tail -20 gpurun_out/r06_ab_group4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_group4.log
TAG=r06_grp4_g3 CMD="scripts/ab_rows.py abl/g3.so --work mixed --rounds 1 --steps 5 --no-check" KREGEX="sbe_decode" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_grp4_g3.txt 2>&1 || { tail -20 gpurun_out/prof_r06_grp4_g3.txt; exit 1; }
tail -6 gpurun_out/prof_r06_grp4_g3.txt
