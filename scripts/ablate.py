"""Build ablation variants of the product library without touching its source: each variant is the
product's csrc/sbe_codec.hip with a few text substitutions (a phase skipped), compiled to
abl/<name>.so for scripts/ab.py (timing) or rocprofv3 PMC passes (instruction counts).  Timing-only:
the variants produce wrong bytes.  Usage: python scripts/ablate.py name [name ...] | --list"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "aeron-cluster-client-cpp_amd", "csrc", "sbe_codec.hip")
OJ = os.path.join(ROOT, "aeron-cluster-client-cpp_amd", "csrc", "order_json.hpp")
OUT = os.path.join(ROOT, "abl")

# name -> list of (old, new) substitutions (each old string must occur exactly once)
VARIANTS = {
    "base": [],
    # record-lane composition: skip the literal bytes / the zone merges / everything after the gate
    "nolit": [("    ph.lap(2);\n    if (!live) return true;\n    // literal bytes: q = 0",
               "    ph.lap(2);\n    return true;\n    // literal bytes: q = 0")],
    "nofix": [("    ph.lap(1);\n    zone_fixup<LY>(wout, inb, rt, wlen, nb, lane, ra, rb);\n", "    ph.lap(1);\n")],
    # record-lane composition: the chunk groups left out (the rebalance still runs)
    "nogroups": [("    int32_t i0 = 0;\n    for (; __ballot(i0 + 3 < n_mine); i0 += 4)", "    int32_t i0 = 0;\n    for (; __ballot(i0 + 3 < n_mine && n_mine < 0); i0 += 4)"),
                 ("    if (__ballot(i0 + 1 < n_mine)) {\n        group(", "    if (__ballot(i0 + 1 < n_mine && n_mine < 0)) {\n        group("),
                 ("    if (__ballot(i0 < n_mine)) group(", "    if (__ballot(i0 < n_mine && n_mine < 0)) group(")],
    "nocompose": [("    if (__ballot(!ok)) return false;\n", "    if (__ballot(!ok)) return false;\n    return true;\n")],
    # decode tiles of 48 / 32 records (lanes past the tile idle) in 12 / 8 KiB windows: more
    # workgroups per CU (LDS-bound at 16 KiB) against idle parse lanes
    "t48": [("constexpr int kTile = 64; ", "constexpr int kTile = 48; "),
            ("constexpr uint32_t kWin = 16384; ", "constexpr uint32_t kWin = 12288; "),
            ("    const uint64_t r = t0 + (uint64_t)lane;\n    const bool valid = r < a.n;",
             "    const uint64_t r = t0 + (uint64_t)lane;\n    const bool valid = lane < kTile && r < a.n;")],
    "t32": [("constexpr int kTile = 64; ", "constexpr int kTile = 32; "),
            ("constexpr uint32_t kWin = 16384; ", "constexpr uint32_t kWin = 8192; "),
            ("    const uint64_t r = t0 + (uint64_t)lane;\n    const bool valid = r < a.n;",
             "    const uint64_t r = t0 + (uint64_t)lane;\n    const bool valid = lane < kTile && r < a.n;")],
    # the fast loop's input staging (loads + LDS writes)
    "nostage": [("        if (have_next && kPacked) stage_issue(Wn.swb, Wn.nb, lane, I);\n", ""),
                ("        if (kPacked) stage_write(win_in, Wn.nb, lane, I);  // after the compose above read win_in\n", "")],
    # chunk-owner path (long records): skip chunk_pass / literal_pass
    "nochunk": [("    chunk_pass(wout, inb, rt, bk, wlen, nb, kk, lg, lane);\n", "")],
    "nolitpass": [("    literal_pass<LY>(ea, wout, rt, S, wlen, lane);\n}", "}")],
    "nofixw": [("    wsync();\n    zone_fixup<LY>(wout, inb, rt, wlen, nb, lane);\n    wsync();\n    literal_pass", "    wsync();\n    literal_pass")],
    "notables": [("    const bool outside = build_tables<LY>(rt, bk, sbase, S, wrel, wlen, swb, nb, ra, rb, lg, lane);\n",
                  "    const bool outside = false;\n")],
    # the fast path's window store
    # Order JSON writer (substitutions in order_json.hpp, inlined into the variant): number
    # formatting / string quoting / the window stores left out (measure and write agree on sizes)
    "oj_nonum": [("OJ", "    s = fmt_g17(s, q);\n", "    s.put('1');\n"), ("OJ", "    s = fmt_fixed6(s, q);\n", "    s.put('1');\n")],
    "oj_noquote": [("OJ", "__device__ __noinline__ S quoted(S s, gu8* p, uint64_t len) {\n",
                    "__device__ __noinline__ S quoted(S s, gu8* p, uint64_t len) {\n    if (len < ~0ull) { s.put('\"'); s.put('\"'); return s; }\n")],
    "oj_nostore": [("OJ", "        for (uint64_t c = lane; c < nch; c += kWWave) {", "        for (uint64_t c = nch + lane; c < nch; c += kWWave) {")],
    # decode: the Ack printable-run scan / the per-lane _sequence_number scan left out (config 3)
    "noack": [("    // maximal runs of printable bytes over [16, len)", "    if (len) return;\n    // maximal runs of printable bytes over [16, len)")],
    "noseqlane": [("__device__ uint32_t has_seq_key_lane(const LdsRec& R, uint32_t p, uint32_t n) {\n    if (n < 16) return 0u;",
                   "__device__ uint32_t has_seq_key_lane(const LdsRec& R, uint32_t p, uint32_t n) {\n    if (n < ~0u) return 0u;")],
    "nostore": [("            store_window(a.out, a.sink, wout, S.T0 + W.A, S.T0 + (int64_t)W.wrel, "
                 "S.T0 + (int64_t)(W.wrel + W.wlen),\n                         lane);\n", "")],
}


def build(name):
    s = open(SRC).read()
    oj = open(OJ).read()
    for sub in VARIANTS[name]:
        tgt, old, new = sub if len(sub) == 3 else ("SRC", *sub)
        t = oj if tgt == "OJ" else s
        if t.count(old) != 1:
            raise SystemExit(f"{name}: substitution target found {t.count(old)} times: {old[:60]!r}")
        if tgt == "OJ":
            oj = oj.replace(old, new)
        else:
            s = s.replace(old, new)
    s = s.replace('#include "order_json.hpp"', oj)
    tmp = os.path.join(os.path.dirname(SRC), f"_abl_{name}.hip")
    open(tmp, "w").write(s)
    os.makedirs(OUT, exist_ok=True)
    try:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                               tmp, "-o", os.path.join(OUT, f"{name}.so"), "-ldl",
                              ])
    finally:
        os.remove(tmp)


if __name__ == "__main__":
    if sys.argv[1:] == ["--list"]:
        print(" ".join(VARIANTS))
        sys.exit(0)
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(4) as ex:
        list(ex.map(build, sys.argv[1:]))
