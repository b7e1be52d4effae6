# r05 GPU session 51: reassembly message table staged through LDS (parity + A/B); Order JSON row
# profile (kernel trace + PMC) on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reassembly.py > gpurun_out/r05_51_tests.log 2>&1 || { tail -30 gpurun_out/r05_51_tests.log; exit 1; }
tail -1 gpurun_out/r05_51_tests.log
timeout -k 10 300 python -u scripts/ab_reasm.py abl/fs_direct.so abl/fs_stage.so --rounds 7 > gpurun_out/r05_51_ab.log 2>&1 || { tail -20 gpurun_out/r05_51_ab.log; exit 1; }
tail -4 gpurun_out/r05_51_ab.log
TAG=r05_reasm3 CMD="scripts/bench_rows.py --no-cpu --rows reassemble --steps 5 --warmup 1" KREGEX="frag_" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_reasm3.txt 2>&1 || { tail -20 gpurun_out/prof_r05_reasm3.txt; exit 1; }
grep -A3 "kernel stats\|== frag_scan_msgs" gpurun_out/prof_r05_reasm3.txt | grep -v FETCH_SIZE | head -12
TAG=r05_orderjson4 CMD="scripts/bench_rows.py --no-cpu --rows order_json --steps 5 --warmup 1" KREGEX="order_json" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_orderjson4.txt 2>&1 || { tail -20 gpurun_out/prof_r05_orderjson4.txt; exit 1; }
head -8 gpurun_out/prof_r05_orderjson4.txt
