"""Per-kernel duration and the idle gap before each kernel, from a rocprofv3 --kernel-trace CSV
(the last `steps` round trips of a bench run).  Usage: trace_gaps.py <kernel_trace.csv> [steps]"""
import collections
import csv
import statistics
import sys

NAMES = ("sbe_enc_pack", "sbe_decode_kernel", "sbe_enc_sums", "sbe_enc_scan", "sbe_enc")


def short(n):
    for k in NAMES:
        if k in n:
            return k
    return None


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = [r for r in csv.DictReader(open(path)) if short(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per_step = len({short(r["Kernel_Name"]) for r in rows})
    seq = rows[-steps * per_step:]
    gaps, durs = collections.defaultdict(list), collections.defaultdict(list)
    for a, b in zip(seq, seq[1:]):
        gaps[short(b["Kernel_Name"])].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    for r in seq:
        durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in durs:
        g = statistics.mean(gaps[k]) if gaps[k] else float("nan")
        print(f"{k:20s} dur {statistics.mean(durs[k]):8.1f} us (min {min(durs[k]):.1f})  gap before {g:6.2f} us")
    span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
    print(f"span per step {span / steps:.1f} us over {steps} steps")


if __name__ == "__main__":
    main()
