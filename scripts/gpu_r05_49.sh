# r05 GPU session 49: the headline bench under rocprofv3 --kernel-trace --stats on the last tree (line and trace from one process)
# trace's kernel averages from the same process)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_benchtrace2 -o run --output-format csv -- python3 bench.py --no-config5 --no-cpu-baseline > gpurun_out/r05_bench_traced2.log 2> gpurun_out/r05_bench_traced2.err || { tail -5 gpurun_out/r05_bench_traced2.err; exit 1; }
cut -c1-400 gpurun_out/r05_bench_traced2.log
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/prof_r05_benchtrace2/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sbe_' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000,2), r.get('MinNs'), r.get('MaxNs'))"
