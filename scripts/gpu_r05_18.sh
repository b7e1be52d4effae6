# r05 GPU session 18: Order JSON single-pass (look-back) launch — parity + A/B against the three-launch form
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orderjson.py > gpurun_out/r05_18_tests.log 2>&1 || { tail -30 gpurun_out/r05_18_tests.log; exit 1; }
tail -3 gpurun_out/r05_18_tests.log
for lib in abl/oj_nofuse.so aeron-cluster-client-cpp_amd/libsbecodec.so abl/oj_lbw1.so abl/oj_nofuse.so aeron-cluster-client-cpp_amd/libsbecodec.so abl/oj_lbw1.so; do
  echo "== $lib"
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 || exit 1
done
