# r06 GPU session 13: Order JSON writer with 64 orders a wave (all lanes writing) in a 28 / 36 KiB
# window against 32 in 18 KiB (base); Order JSON tests on the product build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_orderjson.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_13_tests.log 2>&1 || { tail -30 gpurun_out/r06_13_tests.log; exit 1; }
tail -1 gpurun_out/r06_13_tests.log
for r in 1 2 3; do
for lib in abl/ojbase.so abl/oj64w28.so abl/oj64w36.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 | cut -c1-200 || exit 1
done
done > gpurun_out/r06_ab_ojwin.log
cat gpurun_out/r06_ab_ojwin.log
