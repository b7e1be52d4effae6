# r05 GPU session 32: Order JSON ablations: literals not written, window not stored, everything
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in abl/ojbase.so abl/ojlit.so abl/ojwin.so abl/ojall.so; do
  echo "== $lib"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_32_$(basename $lib .so) -o run --output-format csv -- python3 scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1 --lib $lib > gpurun_out/r05_32_$(basename $lib .so).log 2>&1 || exit 1
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/prof_r05_32_$(basename $lib .so)/run_kernel_stats.csv')): print('  ', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1000,1))"
done
