# r05 GPU session 27: persistent decode (next tile's window in flight during the parse) — parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py > gpurun_out/r05_27_tests.log 2>&1 || { tail -30 gpurun_out/r05_27_tests.log; exit 1; }
tail -1 gpurun_out/r05_27_tests.log
timeout -k 10 400 python scripts/ab_rows.py abl/nopersist.so abl/persist.so --work fixed,mixed --rounds 7 > gpurun_out/r05_27_ab.log 2>&1 || { tail -20 gpurun_out/r05_27_ab.log; exit 1; }
tail -6 gpurun_out/r05_27_ab.log
