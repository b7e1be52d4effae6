# r06 GPU session 26: MATERIALIZE final form (LDS window, batches of 4 chunk loads): parity tests,
# the row with its CPU baseline, kernel trace + PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_materialize.py tests/test_integration_snippets.py tests/test_gpu_parity.py -k "materializ or snippet" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_26_tests.log 2>&1 || { tail -30 gpurun_out/r06_26_tests.log; exit 1; }
tail -1 gpurun_out/r06_26_tests.log
timeout -k 10 300 python -u scripts/bench_rows.py --rows materialize > gpurun_out/r06_rows_mat.jsonl 2> gpurun_out/r06_rows_mat.err || { tail -5 gpurun_out/r06_rows_mat.err; exit 1; }
cut -c1-400 gpurun_out/r06_rows_mat.jsonl
TAG=r06_materialize CMD="scripts/bench_rows.py --no-cpu --rows materialize --steps 5 --warmup 1" KREGEX="mat_" bash scripts/gpu_profile.sh > gpurun_out/prof_r06_materialize.txt 2>&1 || { tail -20 gpurun_out/prof_r06_materialize.txt; exit 1; }
cat gpurun_out/prof_r06_materialize.txt
