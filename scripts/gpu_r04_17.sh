# r04 GPU session 17: per-lane _sequence_number scan with 2 / 4 / 6 / 8 chunk reads in flight (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/ab_rows.py abl/base.so abl/k4.so abl/k6.so abl/k8.so --work mixed,fixed,session,var --rounds 5 > gpurun_out/r04_ab_seqlane_k.log 2>&1
