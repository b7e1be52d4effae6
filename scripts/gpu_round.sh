# bench + kernel-trace profile + FETCH/WRITE passes, then per-variant counters / timings
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_bench.sh && bash scripts/gpu_ablate_counters.sh && \
for f in build/var/*.so; do
  SBECODEC_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/var.json 2>/dev/null && python -c "import json; d=json.loads(open('gpurun_out/var.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$f', 'pack_ms=%.4f dec_ms=%.4f'%(k['pack_ms'],k['decode_kernel_ms']))"
done
