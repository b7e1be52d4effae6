# r06 GPU session 12: _sequence_number chunk classification with the key-slice compares as wave
# masks (v_cmp + s_or) against the per-lane xor/min form: seqnum + decode tests, A/B on config 4
# (the only wide-tile workload) and fixed-256 / session (unaffected: per-lane scans)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seqnum.py tests/test_gpu_parity.py tests/test_gpu_serve.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_12_tests.log 2>&1 || { tail -30 gpurun_out/r06_12_tests.log; exit 1; }
tail -1 gpurun_out/r06_12_tests.log
timeout -k 10 600 python -u scripts/ab_rows.py abl/cmp0.so abl/cmp1.so --work var,fixed --rotate 3 --rounds 7 > gpurun_out/r06_ab_cmp.log 2>&1 || { tail -20 gpurun_out/r06_ab_cmp.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ab_cmp.log
