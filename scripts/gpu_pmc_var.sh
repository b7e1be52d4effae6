# Pack-kernel SQ counters for each library in $LIBS (one pass each).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for f in $LIBS; do
  b=$(basename $f .so)
  SBECODEC_LIB=$PWD/$f timeout -s KILL 120 rocprofv3 --pmc ${PMCSET:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES} --kernel-include-regex "${KREGEX:-sbe_enc_pack}" -d gpurun_out/pv_$b -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 --event-every 0 > gpurun_out/pv_$b.log 2>&1 || { echo "$b failed"; tail -3 gpurun_out/pv_$b.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pv_*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[1][3:], " ".join("%s=%.3g" % (c.replace("SQ_", ""), sum(v) / len(v) / 31250) for c, v in sorted(agg.items())))
PY
