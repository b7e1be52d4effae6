# r05 GPU session 44: final evidence after the nontemporal pack loads and the reassembly changes: GPU suite, smoke, bench, headline profile, rows
# rocprofv3 kernel trace + PMC of the headline, config 3, config 4 and reassembly
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_gpu_tests_final2.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/r05_gpu_tests_final2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_final2.log 2>&1 || { tail -20 gpurun_out/r05_smoke_final.log; exit 1; }
tail -1 gpurun_out/r05_smoke_final2.log
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_final2.log 2> gpurun_out/r05_bench_final2.err || { tail -5 gpurun_out/r05_bench_final2.err; exit 1; }
TAG=r05_fixed256g bash scripts/gpu_profile.sh > gpurun_out/prof_r05_fixed256g.txt 2>&1 || { tail -20 gpurun_out/prof_r05_fixed256g.txt; exit 1; }
cut -c1-700 gpurun_out/r05_bench_final2.log
timeout -k 10 600 python -u scripts/bench_rows.py > gpurun_out/r05_rows3.jsonl 2> gpurun_out/r05_rows3.err || { tail -5 gpurun_out/r05_rows3.err; exit 1; }
