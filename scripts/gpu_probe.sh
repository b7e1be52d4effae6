# Diagnosis: step time with / without the library's kernel events, gaps between kernels, sizes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 120 $B > gpurun_out/p_ev.log 2>&1 && tail -1 gpurun_out/p_ev.log | python scripts/summ.py ev4 && \
timeout -k 10 120 $B --event-every 0 > gpurun_out/p_noev.log 2>&1 && tail -1 gpurun_out/p_noev.log | python scripts/summ.py ev0 && \
for n in ${SIZES:-2000000 4000000 8000000}; do
  timeout -k 10 120 $B --event-every 0 --records $n > gpurun_out/p_n$n.log 2>&1 && tail -1 gpurun_out/p_n$n.log | python scripts/summ.py n=$n || exit 1
done && \
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/kt_noev -o run --output-format csv -- $B --event-every 0 > gpurun_out/kt_noev.log 2>&1 && \
python scripts/trace_gaps.py gpurun_out/kt_noev/run_kernel_trace.csv 20
