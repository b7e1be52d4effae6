# r06 GPU session 18: pack chunks as one unaligned ds_read_b128 (ua1) against five dword reads +
# four v_alignbyte (ua0), every layout, rotated inputs; encode parity tests on ua1 (in-tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_18_tests.log 2>&1 || { tail -30 gpurun_out/r06_18_tests.log; exit 1; }
tail -1 gpurun_out/r06_18_tests.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/ua0.so abl/ua1.so --work fixed,var,session,lite301,lite201 --rotate 3 --rounds 7 > gpurun_out/r06_ab_ua.log 2>&1 || { tail -20 gpurun_out/r06_ab_ua.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_ua.log
