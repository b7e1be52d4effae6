# PMC instruction counts of one kernel across library variants (abl/<name>.so), on the GPU box:
#   VARIANTS="base nolit" KREGEX=sbe_enc_pack ARGS="--enc" bash scripts/pmc_variants.sh
# One rocprofv3 pass per variant (8 SQ counters), each under its own timeout; prints per-wave means.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_var
mkdir -p $O
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"}
for v in $VARIANTS; do
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-include-regex "$KREGEX" -d $O/$v -o run --output-format csv -- python3 scripts/k_run.py abl/$v.so $ARGS --k 3 > $O/$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
for v in os.environ["VARIANTS"].split():
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmc_var/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(x) / len(x) for k, x in agg.items()}
    w = m.get("SQ_WAVES", 1)
    print(f"{v:10s} waves={w:.0f} " + " ".join(f"{k.replace('SQ_', '')}={x / w:.0f}" for k, x in sorted(m.items()) if k != "SQ_WAVES"))
PY
