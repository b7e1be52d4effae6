# r04 GPU session 2: tests, headline bench, host latency (zero-copy vs DMA), A/B of kernel variants,
# fixed-256 rocprof, rows.  Each step under its own limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py > gpurun_out/r04_bench_base.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --no-config5 --no-cpu-baseline > gpurun_out/r04_bench_s20.log 2>&1 || exit 1
make -s -C scripts host_latency && timeout -k 10 200 scripts/host_latency > gpurun_out/r04_host_latency_zc.log 2>&1 || exit 1
AERON_AMD_ZC_BYTES=0 timeout -k 10 200 scripts/host_latency > gpurun_out/r04_host_latency_nozc.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_rows.py abl/base.so abl/ackfast.so abl/b64.so abl/norebal.so abl/rebal12.so --work fixed,var,mixed --rounds 5 > gpurun_out/ab_r04_1.log 2>&1 || exit 1
echo done
