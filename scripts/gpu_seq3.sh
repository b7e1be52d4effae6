set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_seqnum.py tests/test_gpu_host_api.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_seq.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_seq.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/b_fused.log 2>&1 && python scripts/summ.py fused < gpurun_out/b_fused.log && \
timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --separate-seq > gpurun_out/b_sep.log 2>&1 && python scripts/summ.py separate < gpurun_out/b_sep.log || exit 1
done
