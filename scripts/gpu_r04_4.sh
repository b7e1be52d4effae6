# r04 GPU session 4: launch floor, single-call trace, decode-shape A/B for config 3, bench with the
# unsampled timed region
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 scripts/launch_probe > gpurun_out/r04_launch_probe.log 2>&1 || exit 1
cat gpurun_out/r04_launch_probe.log
make -s -C scripts host_latency && AERON_AMD_TRACE=1 timeout -k 10 60 scripts/host_latency 1 > gpurun_out/r04_trace1.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_rows.py abl/ackfast.so abl/dec8k.so abl/dec16k.so --work mixed,fixed --rounds 7 > gpurun_out/ab_r04_2.log 2>&1 || exit 1
cat gpurun_out/ab_r04_2.log
