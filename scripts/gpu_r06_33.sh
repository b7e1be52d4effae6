# r06 GPU session 33: the 20 KiB wide decode window in-tree: full GPU suite, the session row, and
# the session A/B against the committed 12 KiB build's numbers (profiles/r06_ab_decsess*.log)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06_gpu_tests.log
timeout -k 10 300 python -u scripts/bench_rows.py --rows session > gpurun_out/r06_rows_session.jsonl 2> gpurun_out/r06_rows_session.err || { tail -5 gpurun_out/r06_rows_session.err; exit 1; }
cut -c1-600 gpurun_out/r06_rows_session.jsonl
