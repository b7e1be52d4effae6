set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
make -s -C tests/cpp test_host_api && timeout -k 10 300 tests/cpp/test_host_api > gpurun_out/host_api.log 2>&1; echo "host_api rc=$?" >> gpurun_out/host_api.log
timeout -k 10 300 python bench.py > gpurun_out/r04_bench_base.log 2>&1 || exit 1
make -s -C scripts host_latency && timeout -k 10 300 scripts/host_latency > gpurun_out/r04_host_latency_zc.log 2>&1 || exit 1
AERON_AMD_ZC_BYTES=0 timeout -k 10 300 scripts/host_latency > gpurun_out/r04_host_latency_nozc.log 2>&1 || exit 1
TAG=fixed256_base bash scripts/gpu_profile.sh > gpurun_out/prof_base.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_rows.py --no-cpu --rows mixed,var > gpurun_out/rows_base.log 2>&1
