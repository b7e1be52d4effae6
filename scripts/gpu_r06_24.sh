# r06 GPU session 24: MATERIALIZE copy, a lane's chunk loads batched 1 / 4 / 8 (block + tile sums, direct path inlined) against one dependent load a chunk (mat_wave)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out


for r in 1 2; do
for lib in abl/mat_wave.so abl/mat_b1.so abl/mat_b4.so abl/mat_b8.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows materialize --steps 20 --warmup 3 --lib $lib 2>&1 | tail -1 | cut -c1-260 || exit 1
done
done > gpurun_out/r06_ab_mat3.log
cat gpurun_out/r06_ab_mat3.log
