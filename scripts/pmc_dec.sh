set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_dec
mkdir -p $O
for lib in new noscan; do
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
             "SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_BRANCH" \
             "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "sbe_decode_kernel" -d $O/${lib}_$i -o run --output-format csv -- python3 scripts/k_run.py abl/$lib.so --var --k 3 > $O/${lib}_$i.log 2>&1 || { echo "pmc $lib $i failed"; tail -5 $O/${lib}_$i.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for lib in ("new", "noscan"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmc_dec/{lib}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    w = m.get("SQ_WAVES", 1)
    print(lib, " ".join(f"{k}={v:.4g}" for k, v in sorted(m.items())))
    print(lib, "per wave:", " ".join(f"{k}={v / w:.0f}" for k, v in sorted(m.items()) if k != "SQ_WAVES"))
PY
