# r05 GPU session 41: per-layout nontemporal staged-input loads — encode parity + A/B against plain loads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_scale.py > gpurun_out/r05_41_tests.log 2>&1 || { tail -30 gpurun_out/r05_41_tests.log; exit 1; }
tail -1 gpurun_out/r05_41_tests.log
timeout -k 10 500 python scripts/ab_rows.py abl/pk_base.so aeron-cluster-client-cpp_amd/libsbecodec.so --work fixed,var,session,lite301,lite201 --rounds 5 > gpurun_out/r05_41_ab.log 2>&1 || { tail -20 gpurun_out/r05_41_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05_41_ab.log | tail -10
