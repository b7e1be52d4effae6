# r05 GPU session 19: Order JSON single-pass tile shapes (A/B) + per-kernel trace of the three-launch form
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SBECODEC_LIB=$PWD/abl/oj_f64.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orderjson.py > gpurun_out/r05_19_tests.log 2>&1 || { tail -30 gpurun_out/r05_19_tests.log; exit 1; }
tail -1 gpurun_out/r05_19_tests.log
for lib in abl/oj_nofuse.so abl/oj_f64.so abl/oj_f64w18.so aeron-cluster-client-cpp_amd/libsbecodec.so abl/oj_nofuse.so abl/oj_f64.so abl/oj_f64w18.so; do
  echo "== $lib"
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_oj_nofuse -o run --output-format csv -- python3 scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1 --lib abl/oj_nofuse.so > gpurun_out/prof_r05_oj_nofuse.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_oj_f64 -o run --output-format csv -- python3 scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1 --lib abl/oj_f64.so > gpurun_out/prof_r05_oj_f64.log 2>&1 || exit 1
for d in gpurun_out/prof_r05_oj_nofuse gpurun_out/prof_r05_oj_f64; do echo "== $d"; f=$(ls $d/*/run_kernel_stats.csv 2>/dev/null || ls $d/run_kernel_stats.csv); cut -d, -f1-4 $f | head -12; done
