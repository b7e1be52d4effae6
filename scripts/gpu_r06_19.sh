# r06 GPU session 19: Order JSON writer touching its wave's strings up front (oj_pf) against the
# dependent block walk alone (oj_base); Order JSON parity tests on the in-tree build (prefetch on)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_orderjson.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_19_tests.log 2>&1 || { tail -30 gpurun_out/r06_19_tests.log; exit 1; }
tail -1 gpurun_out/r06_19_tests.log
for r in 1 2 3; do
for lib in abl/oj_base.so abl/oj_pf.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 | cut -c1-130 || exit 1
done
done > gpurun_out/r06_ab_ojpf.log
cat gpurun_out/r06_ab_ojpf.log
