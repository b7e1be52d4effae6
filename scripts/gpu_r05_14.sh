# r05 GPU session 14: evidence on the current tree: the default bench, every row (with the CPU
# legs), rocprofv3 kernel trace + PMC of the headline, config 3 and config 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_2.log 2> gpurun_out/r05_bench_2.err || { tail -5 gpurun_out/r05_bench_2.err; exit 1; }
timeout -k 10 600 python -u scripts/bench_rows.py > gpurun_out/r05_rows.jsonl 2> gpurun_out/r05_rows.err || { tail -5 gpurun_out/r05_rows.err; exit 1; }
TAG=r05_fixed256 bash scripts/gpu_profile.sh > gpurun_out/prof_r05_fixed256.txt 2>&1 || { tail -20 gpurun_out/prof_r05_fixed256.txt; exit 1; }
TAG=r05_config3 CMD="scripts/bench_rows.py --no-cpu --rows mixed --steps 5 --warmup 1" KREGEX="sbe_decode_kernel" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_config3.txt 2>&1 || { tail -20 gpurun_out/prof_r05_config3.txt; exit 1; }
TAG=r05_config4 CMD="scripts/bench_rows.py --no-cpu --rows var --steps 3 --warmup 1" KREGEX="sbe_enc_pack|sbe_decode_kernel|sbe_enc_sums" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_config4.txt 2>&1 || { tail -20 gpurun_out/prof_r05_config4.txt; exit 1; }
TAG=r05_reasm CMD="scripts/bench_rows.py --no-cpu --rows reassemble --steps 5 --warmup 1" KREGEX="frag_" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_reasm.txt 2>&1 || { tail -20 gpurun_out/prof_r05_reasm.txt; exit 1; }
cat gpurun_out/r05_bench_2.log; cat gpurun_out/r05_rows.jsonl | cut -c1-300
