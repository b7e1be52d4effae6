set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ablate_counters.sh
mkdir -p gpurun_out/set2 && mv gpurun_out/abl_* gpurun_out/set2/ 2>/dev/null
PMCSET="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" bash scripts/gpu_ablate_counters.sh
for f in build/var/*.so; do
  SBECODEC_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/var.json 2>/dev/null && python -c "import json; d=json.loads(open('gpurun_out/var.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$f', 'enc_ms=%.3f dec_ms=%.3f'%(k['encode_ms'],k['decode_ms']))"
done
