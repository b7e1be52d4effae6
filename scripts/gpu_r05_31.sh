# r05 GPU session 31: decode with every tile on the chunk-parallel _sequence_number classification (SBE_SEQ_LANE_REC=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python scripts/ab_rows.py abl/base.so abl/lr0.so --work fixed,mixed,session --rounds 7 > gpurun_out/r05_31_ab.log 2>&1 || { tail -20 gpurun_out/r05_31_ab.log; exit 1; }
tail -7 gpurun_out/r05_31_ab.log
