# r04 GPU session 21 (run twice): host mirror worker pool A/B (the pool before this round's change / after, with
# spinning off), two interleaved rounds of the per-call latency table, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/abl/old timeout -k 10 240 scripts/host_latency > gpurun_out/r04_pool_ab_old_$r.log 2>&1 || exit 1
  LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/abl/new timeout -k 10 240 scripts/host_latency > gpurun_out/r04_pool_ab_new_$r.log 2>&1 || exit 1
done
