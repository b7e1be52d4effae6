set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_seqnum.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_seq.log 2>&1 && tail -2 gpurun_out/pytest_seq.log && \
bash scripts/gpu_bench.sh
