# r05 GPU session 52: Order JSON headers sizing without the string staging (A/B, alternating libs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in abl/oj_hs1.so abl/oj_hs0.so abl/oj_hs1.so abl/oj_hs0.so abl/oj_hs1.so abl/oj_hs0.so; do
  echo "== $lib"
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 20 --warmup 3 --lib $lib 2>&1 | tail -1 | cut -c1-160 || exit 1
done > gpurun_out/r05_52_ab.log 2>&1
cat gpurun_out/r05_52_ab.log
