# r06 GPU session 17: Order JSON payload writer occupancy: 16 texts a wave in 9 KiB with 3 / 4
# waves per SIMD of registers, 32 in 18 KiB at 3, against the product (32 in 18 KiB, 2 waves)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
for lib in abl/oj_base.so abl/oj_16_3.so abl/oj_16_4.so abl/oj_32_3.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 | cut -c1-130 || exit 1
done
done > gpurun_out/r06_ab_ojocc.log
cat gpurun_out/r06_ab_ojocc.log
