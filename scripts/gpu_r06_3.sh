# r06 GPU session 3: big messages copied by all waves (frag_copy tail), reassembly + gather tests,
# reassembly row A/B (r05 / sg_at fix / big-message list), copy ceiling warm + rotated, rotated bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_reassembly.py tests/test_gpu_gather_mock.py > gpurun_out/r06_3_tests.log 2>&1 || { tail -30 gpurun_out/r06_3_tests.log; exit 1; }
grep -h "reassembly 1 M\|passed\|failed" gpurun_out/r06_3_tests.log | tail -3
timeout -k 10 300 python -u scripts/ab_reasm.py abl/ntl0.so abl/head.so abl/big.so --rounds 7 > gpurun_out/r06_ab_reasm_big.log 2>&1 || { tail -20 gpurun_out/r06_ab_reasm_big.log; exit 1; }
tail -4 gpurun_out/r06_ab_reasm_big.log
timeout -k 10 120 scripts/ceiling 1000000 1 > gpurun_out/r06_ceiling_warm.log 2>&1 || { cat gpurun_out/r06_ceiling_warm.log; exit 1; }
timeout -k 10 120 scripts/ceiling 1000000 3 > gpurun_out/r06_ceiling_rot.log 2>&1 || { cat gpurun_out/r06_ceiling_rot.log; exit 1; }
cat gpurun_out/r06_ceiling_warm.log gpurun_out/r06_ceiling_rot.log
timeout -k 10 300 python -u bench.py --no-config5 > gpurun_out/r06_bench_3.log 2> gpurun_out/r06_bench_3.err || { tail -5 gpurun_out/r06_bench_3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06_bench_3.log'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['frac'],r['kernel_ms'],r['frac_warm'],d['kernels']['decode_kernel_ms'])"
