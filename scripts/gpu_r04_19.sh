# r04 GPU session 19: the round's closing evidence on the final tree: the default bench, rocprofv3
# kernel trace + PMC passes of the headline, config 3 and config 4, then every row
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_final.log 2> gpurun_out/r04_bench_final.err || { tail -5 gpurun_out/r04_bench_final.err; exit 1; }
TAG=r04_fixed256 bash scripts/gpu_profile.sh > gpurun_out/prof_r04_fixed256.txt 2>&1 || { tail -20 gpurun_out/prof_r04_fixed256.txt; exit 1; }
TAG=r04_config3 CMD="scripts/bench_rows.py --no-cpu --rows mixed --steps 5 --warmup 1" KREGEX="sbe_decode_kernel" bash scripts/gpu_profile.sh > gpurun_out/prof_r04_config3.txt 2>&1 || { tail -20 gpurun_out/prof_r04_config3.txt; exit 1; }
TAG=r04_config4 CMD="scripts/bench_rows.py --no-cpu --rows var --steps 3 --warmup 1" KREGEX="sbe_enc_pack|sbe_decode_kernel|sbe_enc_sums" bash scripts/gpu_profile.sh > gpurun_out/prof_r04_config4.txt 2>&1 || { tail -20 gpurun_out/prof_r04_config4.txt; exit 1; }
timeout -k 10 500 python scripts/bench_rows.py --no-cpu > gpurun_out/r04_rows.jsonl 2> gpurun_out/r04_rows.err || exit 1
echo done
