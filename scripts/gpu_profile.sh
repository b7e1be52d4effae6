# rocprofv3 evidence for one workload (run on the GPU box through gpurun):
#   kernel trace + stats, then one PMC pass per counter group (MI355X_MICROARCH.md §rocprofv3 PMC
#   slots: <= 8 SQ, FETCH_SIZE and WRITE_SIZE in passes of their own), each under its own timeout.
# Env: TAG (output dir suffix), CMD (the python command after `python3`), KREGEX (kernels to count).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-run}
CMD=${CMD:-bench.py --no-config5 --no-cpu-baseline --steps 5 --warmup 2}
K=${KREGEX:-sbe_enc_pack|sbe_decode_kernel|sbe_enc_sums}
O=gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $CMD > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$K" -d $O/pmc$i -o run --output-format csv -- python3 $CMD > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
