# r05 GPU session 47: the headline bench itself, A/B in one session: pack staged-input loads plain vs nontemporal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in abl/pk_plain.so aeron-cluster-client-cpp_amd/libsbecodec.so abl/pk_plain.so aeron-cluster-client-cpp_amd/libsbecodec.so; do
  echo "== $lib"
  SBECODEC_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-config5 --no-cpu-baseline > gpurun_out/r05_47.log 2> gpurun_out/r05_47.err || { tail -5 gpurun_out/r05_47.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05_47.log').read().strip().splitlines()[-1]); r=d['roofline']
print(round(d['value']/1e9,3), 'G rec/s', round(d['ms_per_step']*1e3,1), 'us/step', 'pack', round(r['kernel_ms']*1e3,1), 'us', 'decode', round(d['kernels']['decode_kernel_ms']*1e3,1))"
done
