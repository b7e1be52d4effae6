# r06 GPU session 22: MATERIALIZE copy staged per wave through an LDS window (mat_wave, in-tree)
# against one thread a record straight to the arena (mat_lane); parity tests on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_materialize.py tests/test_integration_snippets.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_22_tests.log 2>&1 || { tail -30 gpurun_out/r06_22_tests.log; exit 1; }
tail -1 gpurun_out/r06_22_tests.log
for r in 1 2; do
for lib in abl/mat_lane.so abl/mat_wave.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows materialize --steps 20 --warmup 3 --lib $lib 2>&1 | tail -1 | cut -c1-260 || exit 1
done
done > gpurun_out/r06_ab_mat.log
cat gpurun_out/r06_ab_mat.log
