"""Summarise a scripts/gpu_profile.sh output directory: per kernel, the rocprofv3 --stats average
duration and every PMC counter averaged over its launches, plus the derived figures used in
DESIGN.md (HBM traffic = 2 x FETCH_SIZE + WRITE_SIZE per MI355X_MICROARCH.md §HBM; wave-cycle
shares; instructions per wave).  Usage: python3 scripts/pmc_summary.py gpurun_out/prof_<tag>"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"Lay<0, 16, 5, true(, \d+)?>", "TM", name)
    name = re.sub(r"Lay<32, 16, 5, true(, \d+)?>", "TMS", name)
    name = re.sub(r"Lay<0, 12, 2, false(, \d+)?>", "L2", name)
    name = re.sub(r"Lay<0, 12, 3, false(, \d+)?>", "L3", name)
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("void ", "")


d = sys.argv[1]
stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    print("== kernel stats (rocprofv3 --kernel-trace --stats)")
    for r in csv.DictReader(open(stats[0])):
        print(f"  {short(r['Name'])[:60]:60s} calls={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:9.2f} us "
              f"min={float(r['MinNs'])/1e3:8.2f} max={float(r['MaxNs'])/1e3:8.2f}")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(f"== {k}")
    print("  " + " ".join(f"{c.replace('SQ_', '')}={v:.4g}" for c, v in sorted(m.items())))
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        print(f"  HBM traffic per launch: {(2 * m['FETCH_SIZE'] + m['WRITE_SIZE']) * 1024 / 1e6:.1f} MB "
              f"(2 x FETCH {m['FETCH_SIZE'] * 2048 / 1e6:.1f} MB + WRITE {m['WRITE_SIZE'] * 1024 / 1e6:.1f} MB)")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        parts = {c: m[c] / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if c in m}
        print("  wave-cycle shares: " + " ".join(f"{c.replace('SQ_', '')}={v:.2f}" for c, v in parts.items()))
    w = m.get("SQ_WAVES")
    if w:
        print("  per wave: " + " ".join(f"{c.replace('SQ_INSTS_', '')}={m[c] / w:.0f}" for c in sorted(m)
                                        if c.startswith("SQ_INSTS_")))
