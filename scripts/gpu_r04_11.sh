# r04 GPU session 11 (final evidence): the default bench run, then rocprofv3 kernel trace + PMC
# passes of the headline (fixed-256 round trip), config 3 (mixed decode) and config 4
# (variable-length round trip), then every row
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_final.log 2> gpurun_out/r04_bench_final.err || { tail -5 gpurun_out/r04_bench_final.err; exit 1; }
cat gpurun_out/r04_bench_final.log
bash scripts/gpu_r04_3.sh
