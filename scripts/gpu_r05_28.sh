# r05 GPU session 28: Order JSON ablations (wrong bytes by design): numbers / quoted strings as constants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in abl/ojbase.so abl/ojnum.so abl/ojstr.so abl/ojboth.so; do
  echo "== $lib"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_28_$(basename $lib .so) -o run --output-format csv -- python3 scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1 --lib $lib > gpurun_out/r05_28_$(basename $lib .so).log 2>&1 || exit 1
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/prof_r05_28_$(basename $lib .so)/run_kernel_stats.csv')): print('  ', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1000,1))"
done
