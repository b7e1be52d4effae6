"""Interleaved A/B timing of library builds in ONE process (cdna_hip_programming.md §5.4 rule 24):
rounds x libraries, each a timed block of round trips (encode + parse decode) of the bench
workload; prints median / min ms per step and the median pack / decode kernel times per library.
Usage: python scripts/ab.py lib1.so lib2.so ... [--records N] [--rounds R] [--steps K]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--records", type=int, default=1_000_000)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--var", action="store_true", help="variable-length workload (config 4) instead of fixed-256")
ap.add_argument("--session", action="store_true", help="session-framed fixed-256 records (the session row)")
ap.add_argument("--no-check", action="store_true", help="ablation builds: skip the same-output check")
args = ap.parse_args()

sbecodec.use_library(os.path.abspath(args.libs[0]))
sbecodec.require_device()
dev = torch.device("cuda:0")
n = args.records
if args.var:
    a, l, t = T.var_orders_t(n, dev)
else:
    arena, L, ts = T.fixed256_orders(n)
    a = torch.from_numpy(arena).to(dev)
    l = torch.from_numpy(L.view(np.int32)).to(dev)
    t = torch.from_numpy(ts.view(np.int64)).to(dev)
cap = int(l.sum()) + 66 * n
out = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
off = torch.empty(n + 1, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.uint8, device=dev)
res = {p: {"step": [], "pack": [], "dec": []} for p in args.libs}
ref = None
for rnd in range(args.rounds):
    for p in args.libs:
        sbecodec.use_library(os.path.abspath(p))
        ws = sbecodec.alloc_workspace(n, dev)
        dec = sbecodec.alloc_decoded(n, dev)

        def step():
            if args.session:
                sbecodec.encode_session_batch(a, l, t, 7, 8, out=out, out_off=off, status=st, workspace=ws)
            else:
                sbecodec.encode_topic_batch(a, l, t, out=out, out_off=off, status=st, workspace=ws)
            sbecodec.decode_batch(out, off, out=dec)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        if rnd == 0 and not args.no_check:  # every build must produce the same bytes
            h = (int(off[-1]), int(out[: int(off[-1])].to(torch.int64).sum()), int(dec.view_off.to(torch.int64).sum()))
            ref = ref or h
            assert h == ref, f"{p}: output differs from {args.libs[0]}"
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        res[p]["step"].append((time.perf_counter() - t0) / args.steps * 1e6)
        sbecodec.profile_enable(1)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        res[p]["pack"] += sbecodec.profile_read(sbecodec.PROF_PACK)
        res[p]["dec"] += sbecodec.profile_read(sbecodec.PROF_DECODE)
        sbecodec.profile_enable(0)
for p in args.libs:
    r = res[p]
    print(f"{os.path.basename(p):24s} step med {np.median(r['step']):7.1f} min {np.min(r['step']):7.1f} us | "
          f"pack med {np.median(r['pack']) * 1e3:6.1f} us | decode med {np.median(r['dec']) * 1e3:6.1f} us", flush=True)
