# r06 GPU session 1: the rotated (cache-cold) headline bench and the warm one side by side; the
# staged-input load policy of the pack (default / nontemporal for TM+OrderRequestLite / always) A/B on
# rotated inputs (3 copies) for the fixed-256, config-4 and session workloads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-config5 > gpurun_out/r06_bench_rot.log 2> gpurun_out/r06_bench_rot.err || { tail -5 gpurun_out/r06_bench_rot.err; exit 1; }
cut -c1-300 gpurun_out/r06_bench_rot.log
timeout -k 10 400 python -u scripts/ab_rows.py abl/ntl0.so abl/ntl1.so abl/ntl2.so --work fixed,var,session,lite201 --rotate 3 --rounds 5 > gpurun_out/r06_ab_ntl_rot.log 2>&1 || { tail -20 gpurun_out/r06_ab_ntl_rot.log; exit 1; }
cat gpurun_out/r06_ab_ntl_rot.log
timeout -k 10 300 python -u scripts/ab_rows.py abl/ntl0.so abl/ntl1.so --work fixed,var --rotate 1 --rounds 3 > gpurun_out/r06_ab_ntl_warm.log 2>&1 || { tail -20 gpurun_out/r06_ab_ntl_warm.log; exit 1; }
cat gpurun_out/r06_ab_ntl_warm.log
