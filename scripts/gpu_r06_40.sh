# r06 GPU session 40: MATERIALIZE view loads nontemporal against the default policy (rotated row)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
for lib in abl/m_ntl0.so abl/m_ntl1.so; do
  echo -n "$lib "
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows materialize --steps 20 --warmup 3 --lib $lib 2>&1 | tail -1 | cut -c1-200 || exit 1
done
done > gpurun_out/r06_ab_matntl.log
cat gpurun_out/r06_ab_matntl.log
