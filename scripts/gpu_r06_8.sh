# r06 GPU session 8: group decode with the descriptors staged back into record order (LDS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_seqnum.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_8_tests.log 2>&1 || { tail -30 gpurun_out/r06_8_tests.log; exit 1; }
tail -1 gpurun_out/r06_8_tests.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/g0.so abl/g2.so abl/g3.so abl/g4.so --work mixed --rotate 3 --rounds 7 > gpurun_out/r06_ab_group2.log 2>&1 || { tail -20 gpurun_out/r06_ab_group2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_group2.log
