"""Copy a scripts/gpu_profile.sh run (gpurun_out/prof_<tag>/) into profiles/ and derive
profiles/traffic.json for bench.py's roofline "traffic" field.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the bytes of wide coalesced reads on
gfx950, so traffic = 2 x FETCH_SIZE + WRITE_SIZE, per launch (average over the profiled launches).
Usage: python scripts/collect_profiles.py <prof tag> <profiles prefix, e.g. r02_fixed256>
                                          [records per launch] [--traffic]
  --traffic: also (re)write profiles/traffic.json entries for the kernels this run profiled.
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
# rocprof kernel names -> the names bench.py reports (TopicMessage layout Lay<0, 16, 5, true>,
# packed input, wire length kLenWire = 0)
KERNELS = {"sbe_enc_pack<(anonymous namespace)::Lay<0, 16, 5, true>, true, 0>": "sbe_enc_pack<packed,wire>",
           "sbe_enc_sums<(anonymous namespace)::Lay<0, 16, 5, true>, true, 0>": "sbe_enc_sums<packed,wire>",
           "sbe_enc_pack<(anonymous namespace)::Lay<0, 16, 5, true>, false, 0>": "sbe_enc_pack<plain,wire>",
           "sbe_enc_sums<(anonymous namespace)::Lay<0, 16, 5, true>, false, 0>": "sbe_enc_sums<plain,wire>",
           "sbe_decode_kernel<0u>": "sbe_decode_kernel<parse_message>",
           "sbe_decode_kernel<0u, 16384u>": "sbe_decode_kernel<parse_message>",
           "sbe_decode_kernel<0u, 12288u>": "sbe_decode_kernel<parse_message,wide>",
           "sbe_decode_kernel<0u, 14336u>": "sbe_decode_kernel<parse_message,14k>",
           "sbe_decode_kernel<0u, 8192u>": "sbe_decode_kernel<parse_message,8k>",
           "sbe_seqnum_kernel": "sbe_seqnum_kernel"}


def short(name):
    name = re.sub(r"(Lay<[^>]*?), (32|64)>", r"\1>", name)  # the layout's tile shape argument
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


def counter(d, cname):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == cname:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {short(k): sum(v) / len(v) for k, v in agg.items() if short(k)}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    tag, prefix = args[0], args[1]
    records = int(args[2]) if len(args) > 2 else 1_000_000
    d = os.path.join(OUT, f"prof_{tag}")
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)[0],
                os.path.join(PROF, f"{prefix}_kernel_stats.csv"))
    if os.path.exists(os.path.join(d, "summary.txt")):
        shutil.copy(os.path.join(d, "summary.txt"), os.path.join(PROF, f"{prefix}_summary.txt"))
    # every PMC pass, merged into one CSV (kernel, counter, mean over launches)
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    with open(os.path.join(PROF, f"{prefix}_pmc.csv"), "w", newline="") as fh:
        wr = csv.writer(fh)
        wr.writerow(["kernel", "counter", "mean_per_launch", "launches"])
        for (k, c), v in sorted(agg.items()):
            wr.writerow([short(k) or k[:120], c, sum(v) / len(v), len(v)])
    fetch, write = counter(d, "FETCH_SIZE"), counter(d, "WRITE_SIZE")
    traffic = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        traffic[k] = {"bytes_per_launch": (2 * f + w) * 1024, "records": records, "fetch_kib": f, "write_kib": w,
                      "formula": "2 x FETCH_SIZE + WRITE_SIZE (KiB)", "source": f"profiles/{prefix}_pmc.csv"}
    if "--traffic" in sys.argv:
        p = os.path.join(PROF, "traffic.json")
        cur = json.load(open(p)) if os.path.exists(p) else {}
        cur.update(traffic)
        json.dump(cur, open(p, "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
