# r05 GPU session 45: Order JSON writer's HBM string reads nontemporal (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in abl/oj_cur.so abl/oj_ntstr.so abl/oj_cur.so abl/oj_ntstr.so; do
  echo "== $lib"
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 | cut -c1-120 || exit 1
done
