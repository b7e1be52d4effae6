"""Copy a gpu_bench.sh run's rocprofv3 outputs into profiles/ and derive profiles/traffic.json.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the bytes of wide coalesced reads on
gfx950, so traffic = 2 x FETCH_SIZE + WRITE_SIZE, per launch (average over the profiled launches).
Usage: python scripts/collect_profiles.py <round tag, e.g. r01> [records per launch]
"""
import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
# rocprof kernel names (TopicMessage layout Lay<0, 16, 5, true>, packed input, wire length)
KERNELS = {"sbe_enc_pack<(anonymous namespace)::Lay<0, 16, 5, true>, true, false>": "sbe_enc_pack<packed,wire>",
           "sbe_decode_kernel<0u>": "sbe_decode_kernel<parse_message>",
           "sbe_seqnum_kernel": "sbe_seqnum_kernel",
           "sbe_enc_sums<(anonymous namespace)::Lay<0, 16, 5, true>, true, false>": "sbe_enc_sums<packed,wire>"}


def short(name):
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


def counter(path, cname):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == cname:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {short(k): sum(v) / len(v) for k, v in agg.items() if short(k)}


def main():
    tag = sys.argv[1]
    records = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, "prof_kt", "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    fetch = counter(os.path.join(OUT, "prof_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter(os.path.join(OUT, "prof_write", "run_counter_collection.csv"), "WRITE_SIZE")
    rows, traffic = [], {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        b = (2 * f + w) * 1024
        rows.append({"kernel": k, "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes_per_launch": b,
                     "records_per_launch": records})
        traffic[k] = {"bytes_per_launch": b, "records": records, "fetch_kib": f, "write_kib": w,
                      "formula": "2 x FETCH_SIZE + WRITE_SIZE (KiB)", "source": f"profiles/{tag}_pmc_traffic.csv"}
    with open(os.path.join(PROF, f"{tag}_pmc_traffic.csv"), "w", newline="") as fh:
        wr = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        wr.writeheader()
        wr.writerows(rows)
    json.dump(traffic, open(os.path.join(PROF, "traffic.json"), "w"), indent=1)
    for name in ("bench.log", "bench16m.log"):
        p = os.path.join(OUT, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(PROF, f"{tag}_{name}"))
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
