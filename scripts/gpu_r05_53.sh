# r05 GPU session 53: fragments per thread of the reassembly scan launches (2 / 4 / 8), A/B with
# output checks; then final evidence on the tree with the staged message table: GPU suite, smoke,
# bench, every row
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_reasm.py abl/fp4.so abl/fp2.so abl/fp8.so --rounds 7 > gpurun_out/r05_53_ab.log 2>&1 || { tail -20 gpurun_out/r05_53_ab.log; exit 1; }
tail -4 gpurun_out/r05_53_ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_gpu_tests_final4.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_final4.log; exit 1; }
tail -1 gpurun_out/r05_gpu_tests_final4.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_final4.log 2>&1 || { tail -20 gpurun_out/r05_smoke_final4.log; exit 1; }
tail -1 gpurun_out/r05_smoke_final4.log
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_final4.log 2> gpurun_out/r05_bench_final4.err || { tail -5 gpurun_out/r05_bench_final4.err; exit 1; }
cut -c1-400 gpurun_out/r05_bench_final4.log
timeout -k 10 600 python -u scripts/bench_rows.py > gpurun_out/r05_rows5.jsonl 2> gpurun_out/r05_rows5.err || { tail -5 gpurun_out/r05_rows5.err; exit 1; }
cut -c1-120 gpurun_out/r05_rows5.jsonl
