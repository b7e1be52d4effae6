# r06 GPU session 7: mixed-batch decode with waves specialised by record kind (group kernel,
# 2 / 3 / 4 tiles a workgroup) against the one-wave-per-tile mid kernel; GPU suite on the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_7_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06_7_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06_7_gpu_tests.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/g0.so abl/g2.so abl/g3.so abl/g4.so --work mixed --rotate 3 --rounds 7 > gpurun_out/r06_ab_group.log 2>&1 || { tail -20 gpurun_out/r06_ab_group.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_group.log
