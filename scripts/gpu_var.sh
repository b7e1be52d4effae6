# Per library variant in build/var/: encode/decode parity subset, bench summary, kernel gaps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --steps 20 --warmup 5"
for f in build/var/*.so; do
  b=$(basename $f .so)
  export SBECODEC_LIB=$PWD/$f
  if [ -z "$NOTEST" ]; then
    timeout -k 10 300 python -m pytest -x -q tests/test_gpu_parity.py ${PYK:+-k "$PYK"} > gpurun_out/var_$b.test.log 2>&1 || { echo "$b: TESTS FAILED"; tail -20 gpurun_out/var_$b.test.log; exit 1; }
    echo "$b: $(tail -1 gpurun_out/var_$b.test.log)"
  fi
  for ev in 0 4; do
    timeout -k 10 120 $B --event-every $ev ${RECS:+--records $RECS} > gpurun_out/var_$b.$ev.log 2>&1 && tail -1 gpurun_out/var_$b.$ev.log | python scripts/summ.py "$b ev=$ev" || exit 1
  done
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/kt_$b -o run --output-format csv -- $B --event-every 0 > gpurun_out/kt_$b.log 2>&1 && python scripts/trace_gaps.py gpurun_out/kt_$b/run_kernel_trace.csv 20 || exit 1
done
