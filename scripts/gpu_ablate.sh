set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for f in build/abl/*.so; do
  SBECODEC_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abl.json 2>/dev/null || { echo "$f failed"; break; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abl.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$f', 'enc_ms=%.3f dec_ms=%.3f'%(k['encode_ms'],k['decode_ms']))"
done
