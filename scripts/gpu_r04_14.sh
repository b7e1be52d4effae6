# r04 GPU session 14: serve decode with the staged chunks classified in parallel: phase probe,
# serve parity tests, host-mirror latency
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 scripts/serve_probe abl/serveprof.so > gpurun_out/r04_serve_probe3.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_serve.py tests/test_gpu_seqnum.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_serve_tests.log 2>&1 &&
timeout -k 10 240 scripts/host_latency > gpurun_out/r04_host_latency_serve.log 2>&1
