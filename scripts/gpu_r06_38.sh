# r06 GPU session 38: reassembly copy knobs on rotated inputs (bench_rows' row, 3 buffer sets):
# product (4 chunks a lane a step, default-policy source loads) against nontemporal source loads and
# 2 / 8 chunks a lane a step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
for lib in abl/r_base.so abl/r_ntl1.so abl/r_u2.so abl/r_u8.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows reassemble --steps 20 --warmup 3 --lib $lib 2>&1 | tail -1 | cut -c1-200 || exit 1
done
done > gpurun_out/r06_ab_fc_rot.log
cat gpurun_out/r06_ab_fc_rot.log
