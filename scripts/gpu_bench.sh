set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1 && cat gpurun_out/bench.log && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --records 16000000 --no-cpu-baseline > gpurun_out/bench16m.log 2>&1 && cat gpurun_out/bench16m.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1
echo "rc=$?"
find gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write -name "*.csv" | head -20
