# r05 GPU session 36: Order JSON headers: the UPDATED / CANCELLED test on two 64-bit words — parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orderjson.py > gpurun_out/r05_36_tests.log 2>&1 || { tail -30 gpurun_out/r05_36_tests.log; exit 1; }
tail -1 gpurun_out/r05_36_tests.log
for lib in abl/oj_prev.so aeron-cluster-client-cpp_amd/libsbecodec.so abl/oj_prev.so aeron-cluster-client-cpp_amd/libsbecodec.so; do
  echo "== $lib"
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 | cut -c1-120 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_36 -o run --output-format csv -- python3 scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1 > gpurun_out/r05_36_prof.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_r05_36/run_kernel_stats.csv')): print('  ', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1000,1))"
