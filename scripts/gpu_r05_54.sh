# r05 GPU session 54: the rebuilt in-tree library (scan-launch knob, same defaults): reassembly and Order JSON tests, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reassembly.py tests/test_gpu_orderjson.py > gpurun_out/r05_54_tests.log 2>&1 || { tail -30 gpurun_out/r05_54_tests.log; exit 1; }
tail -1 gpurun_out/r05_54_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_54_smoke.log 2>&1 || { tail -20 gpurun_out/r05_54_smoke.log; exit 1; }
tail -1 gpurun_out/r05_54_smoke.log
