set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIPTEST" ] || timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
for f in build/var/*.so; do
  for nrec in ${NRECS:-1000000 16000000}; do
  SBECODEC_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 10 --warmup 3 --records $nrec --no-cpu-baseline > gpurun_out/var.json 2>gpurun_out/var.err || { echo "$f failed"; tail -3 gpurun_out/var.err; break; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/var.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$f', $nrec, 'enc_ms=%.3f pack_ms=%.3f (%.0f GB/s) dec_ms=%.3f (%.0f GB/s) value=%.3g'%(k['encode_ms'],k['pack_ms'],k['pack_gbs'],k['decode_kernel_ms'],k['decode_kernel_gbs'],d['value']))"
  done
done
