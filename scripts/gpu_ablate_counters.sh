# Instruction counters of the pack kernel for each build/var/*.so (one PMC pass per library).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${KREGEX:-sbe_enc_pack}
for f in build/var/*.so; do
  b=$(basename $f .so)
  SBECODEC_LIB=$PWD/$f timeout -k 10 180 rocprofv3 --pmc ${PMCSET:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES} --kernel-include-regex "$K" -d gpurun_out/abl_$b -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$b.log 2>&1
  echo "$b rc=$?"
done
python3 - <<'PY'
import csv,glob,collections
for f in sorted(glob.glob("gpurun_out/abl_*/run_counter_collection.csv")):
    agg=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r['Kernel_Name'][:40],r['Counter_Name'])].append(float(r['Counter_Value']))
    print(f.split('/')[1], " ".join("%s=%.4g"%(k[1],sum(v)/len(v)) for k,v in sorted(agg.items())))
PY
