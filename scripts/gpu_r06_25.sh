# r06 GPU session 25: MATERIALIZE copy occupancy: LDS window 8 / 12 / 16 KiB with registers for
# 3-4 waves per SIMD, against the 16 KiB window at 3 (mat_base, batches of 4 chunk loads)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
for lib in abl/mat_base.so abl/mat_w8m4.so abl/mat_w12m4.so abl/mat_w16m4.so abl/mat_w8m3.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows materialize --steps 20 --warmup 3 --lib $lib 2>&1 | tail -1 | cut -c1-200 || exit 1
done
done > gpurun_out/r06_ab_mat4.log
cat gpurun_out/r06_ab_mat4.log
