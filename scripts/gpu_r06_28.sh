# r06 GPU session 28: MATERIALIZE copy on a persistent grid, next tile descriptors in flight
# (mat_p1, in-tree) against a workgroup per tile (mat_p0); parity on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_materialize.py tests/test_integration_snippets.py tests/test_gpu_parity.py -k "materializ or snippet" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_28_tests.log 2>&1 || { tail -30 gpurun_out/r06_28_tests.log; exit 1; }
tail -1 gpurun_out/r06_28_tests.log
for r in 1 2; do
for lib in abl/mat_p0.so abl/mat_p1.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows materialize --steps 20 --warmup 3 --lib $lib 2>&1 | tail -1 | cut -c1-200 || exit 1
done
done > gpurun_out/r06_ab_mat6.log
cat gpurun_out/r06_ab_mat6.log
