"""Interleaved A/B timing of library builds on the reassembly row (1 M fragments: 90 % whole
messages, 10 % BEGIN..END groups of 2-5, scripts/bench_rows.py's row_reassemble workload) in ONE
process: rounds x libraries, HIP events around a block of calls, median / min ms per library.
Every build's output (bytes, msg_off, counts) is checked against the first build's.
Usage: python scripts/ab_reasm.py lib1.so lib2.so ... [--rounds R] [--steps K]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--clean", action="store_true",
                help="no whole message inside a group (every group's bytes in input order: the flat copy)")
args = ap.parse_args()

sbecodec.use_library(os.path.abspath(args.libs[0]))
sbecodec.require_device()
dev = torch.device("cuda:0")
n = 1_000_000
data, off, flags = T.fragment_stream(n, 11, p_single=0.9, maxlen=512, p_group=0.1, p_inner=0.0 if args.clean else 0.1)
d = torch.from_numpy(data).to(dev)
o = torch.from_numpy(off.view(np.int64)).to(dev)
f = torch.from_numpy(flags).to(dev)
out = torch.empty(max(data.size, 16), dtype=torch.uint8, device=dev)
mo = torch.empty(n + 1, dtype=torch.int64, device=dev)
nbytes = 2 * data.size + (8 + 1 + 8) * n
res = {p: [] for p in args.libs}
ref = None
for rnd in range(args.rounds):
    for p in args.libs:
        sbecodec.use_library(os.path.abspath(p))
        ws = torch.empty(int(sbecodec.lib().sbe_reassemble_workspace_size(n)), dtype=torch.uint8, device=dev)
        out.zero_()
        r = sbecodec.reassemble(d, o, f, out=out, msg_off=mo, workspace=ws)
        torch.cuda.synchronize()
        m = int(r.counts[0])
        got = (out[: int(mo[m])].cpu().numpy().tobytes(), mo[: m + 1].cpu().numpy().tobytes(), r.counts.cpu().numpy().tobytes())
        if ref is None:
            ref = got
        elif got != ref:
            raise SystemExit(f"{p}: output differs from {args.libs[0]}")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            sbecodec.reassemble(d, o, f, out=out, msg_off=mo, workspace=ws)
        e1.record()
        torch.cuda.synchronize()
        res[p].append(e0.elapsed_time(e1) / args.steps)
for p in args.libs:
    v = np.array(res[p])
    print(f"reassemble{'(clean)' if args.clean else ''} {os.path.basename(p):24s} med {np.median(v) * 1e3:8.1f} us  min {v.min() * 1e3:8.1f} us  "
          f"{nbytes / (np.median(v) * 1e-3) / 1e12:5.2f} TB/s (all launches)", flush=True)
