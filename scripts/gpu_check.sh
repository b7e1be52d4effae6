set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 240 python scripts/probe_encode.py > gpurun_out/probe.log 2>&1; echo "probe rc=$?" >> gpurun_out/probe.log
grep -v "bytes_ok=True" gpurun_out/probe.log | tail -8
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1; cat gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1
cut -c1-200 gpurun_out/prof_kt/run_kernel_stats.csv
