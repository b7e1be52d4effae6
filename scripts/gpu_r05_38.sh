# r05 GPU session 38: frag_copy with nontemporal 16-B stores — parity + A/B, and its PMC; Order JSON plain-string count
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reassembly.py > gpurun_out/r05_38_tests.log 2>&1 || { tail -30 gpurun_out/r05_38_tests.log; exit 1; }
tail -1 gpurun_out/r05_38_tests.log
timeout -k 10 300 python -u scripts/ab_reasm.py abl/fc_plain.so abl/fc_nt.so --rounds 7 > gpurun_out/r05_38_ab.log 2>&1 || { tail -20 gpurun_out/r05_38_ab.log; exit 1; }
grep reassemble gpurun_out/r05_38_ab.log
TAG=r05_reasm2 CMD="scripts/bench_rows.py --no-cpu --rows reassemble --steps 5 --warmup 1" KREGEX="frag_" bash scripts/gpu_profile.sh > gpurun_out/prof_r05_reasm2.txt 2>&1 || { tail -20 gpurun_out/prof_r05_reasm2.txt; exit 1; }
grep -A4 "== frag_copy\|kernel stats" gpurun_out/prof_r05_reasm2.txt | grep -v FETCH_SIZE | head -20
# Order JSON sizing: a plain string counted as len + 2 after one SWAR pass (A/B against the walking count)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_orderjson.py > gpurun_out/r05_38_ojtests.log 2>&1 || { tail -30 gpurun_out/r05_38_ojtests.log; exit 1; }
tail -1 gpurun_out/r05_38_ojtests.log
for lib in abl/oj_walkcount.so aeron-cluster-client-cpp_amd/libsbecodec.so abl/oj_walkcount.so aeron-cluster-client-cpp_amd/libsbecodec.so; do
  echo "== $lib"
  timeout -k 10 120 python scripts/bench_rows.py --no-cpu --rows order_json --steps 10 --warmup 2 --lib $lib 2>&1 | tail -1 | cut -c1-120 || exit 1
done
