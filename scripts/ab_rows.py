"""Interleaved A/B timing of library builds in ONE process over several workloads: for each build,
rounds of timed blocks with HIP events on the pack and decode kernels (the library's profiling
ring), medians per (build, workload).  Every build's output is checked against the first build's
(bytes and descriptors).  Workloads:
  fixed   1 M fixed-256 Order TopicMessages, encode + parse decode (the headline)
  var     4 M variable-length TopicMessages (config 4's generator), encode + parse decode
  mixed   1 M mixed TM / Ack records (config 3), parse decode
  session 1 M session-framed fixed-256, encode + parse decode
  lite301 / lite201  1 M CommitOffsetLite / OrderRequestLite records, encode + Lite decode
Usage: python scripts/ab_rows.py lib1.so lib2.so ... [--work fixed,var,mixed] [--rounds R] [--steps K]"""
import argparse
import ctypes
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
ap.add_argument("--work", default="fixed,var,mixed")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--var-records", type=int, default=4_000_000)
ap.add_argument("--no-check", action="store_true", help="ablation builds (wrong bytes by design): skip the check")
ap.add_argument("--rotate", type=int, default=1,
                help="distinct copies of every workload's inputs and outputs the steps rotate over (R > 1: no "
                     "step finds its inputs in the 256 MB MALL; 1: the same buffers every step)")
ap.add_argument("--phases", action="store_true", help="builds with -DSBE_PACK_PHASES: print the pack loop's phase shares")
args = ap.parse_args()

sbecodec.use_library(os.path.abspath(args.libs[0]))
sbecodec.require_device()
dev = torch.device("cuda:0")


def prep(kind):
    if kind in ("fixed", "session"):
        n = 1_000_000
        arena, L, ts = T.fixed256_orders(n)
        a = torch.from_numpy(arena).to(dev)
        l = torch.from_numpy(L.view(np.int32)).to(dev)
        t = torch.from_numpy(ts.view(np.int64)).to(dev)
        return dict(n=n, a=a, l=l, t=t, enc=True, session=kind == "session")
    if kind == "var":
        n = args.var_records
        a, l, t = T.var_orders_t(n, dev)
        return dict(n=n, a=a, l=l, t=t, enc=True, session=False)
    if kind == "mixed":
        data, off = T.mixed_records(1_000_000)
        return dict(n=1_000_000, data=torch.from_numpy(data).to(dev),
                    off=torch.from_numpy(off.view(np.int64)).to(dev), enc=False)
    if kind.startswith("fixedp"):  # fixed-size TopicMessages with a P-byte payload, random printable bytes
        P = int(kind[6:])
        rec = 34 + 6 + 12 + 29 + P + 32
        n = (4_000_000 * 387) // rec
        lens = torch.tensor([6, 12, 29, P, 32], dtype=torch.int32, device=dev).repeat(n, 1)
        a = torch.randint(32, 127, (n * (rec - 34),), dtype=torch.uint8, device=dev)
        t = torch.arange(n, dtype=torch.int64, device=dev) + 1_760_000_000_000_000_000
        return dict(n=n, a=a, l=lens, t=t, enc=True, session=False)
    if kind.startswith("lite"):
        t_id, n = int(kind[4:]), 1_000_000
        arena, L, tid, seq = T.lite_records(n, t_id)
        return dict(n=n, a=torch.from_numpy(arena).to(dev), l=torch.from_numpy(L.view(np.int32)).to(dev),
                    ti=torch.from_numpy(tid.view(np.int32)).to(dev), sq=torch.from_numpy(seq.view(np.int64)).to(dev),
                    enc=True, session=False, lite=t_id, cap=arena.size + (20 + 2 * T.LITE_NF[t_id]) * n)
    raise SystemExit(f"unknown workload {kind}")


works = {k: prep(k) for k in args.work.split(",")}
for w in works.values():
    n = w["n"]
    w["bytes"] = int(w["off"][-1]) if "off" in w else w["cap"] if "lite" in w else (
        int(w["l"].sum()) + n * (34 if not w["session"] else 32 + 26))
    if w["enc"]:
        cap = w.get("cap", int(w["l"].sum()) + 66 * n)
        w["out"] = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
        w["off_o"] = torch.empty(n + 1, dtype=torch.int64, device=dev)
        w["st"] = torch.empty(n, dtype=torch.uint8, device=dev)
    w["seq"] = torch.zeros(n, dtype=torch.int64, device=dev)

# rotation: R copies of every tensor a step reads or writes (clones: the same bytes at other addresses)
for w in works.values():
    w["sets"] = [{k: v for k, v in w.items() if torch.is_tensor(v)}]
    for _ in range(1, args.rotate):
        w["sets"].append({k: v.clone() for k, v in w["sets"][0].items()})
    w["cur"] = 0

res = {(p, k): {"pack": [], "dec": []} for p in args.libs for k in works}
ref = {}
for rnd in range(args.rounds):
    for p in args.libs:
        sbecodec.use_library(os.path.abspath(p))
        for k, w in works.items():
            n = w["n"]
            ws = sbecodec.alloc_workspace(n, dev) if w["enc"] else None
            decs = [sbecodec.alloc_decoded(n, dev) for _ in w["sets"]]

            def step():
                j = w["cur"] % len(w["sets"])
                w["cur"] += 1
                w.update(w["sets"][j])
                dec = decs[j]
                if "lite" in w:
                    sbecodec.encode_lite_batch(w["lite"], w["a"], w["l"], w["ti"], w["sq"], out=w["out"],
                                               out_off=w["off_o"], status=w["st"], workspace=ws)
                    sbecodec.decode_batch(w["out"], w["off_o"], sbecodec.DEC_LITE, out=dec, in_bytes=w["bytes"])
                    return
                if w["enc"]:
                    if w["session"]:
                        sbecodec.encode_session_batch(w["a"], w["l"], w["t"], 7, 8, out=w["out"], out_off=w["off_o"],
                                                      status=w["st"], workspace=ws)
                    else:
                        sbecodec.encode_topic_batch(w["a"], w["l"], w["t"], out=w["out"], out_off=w["off_o"],
                                                    status=w["st"], workspace=ws)
                    sbecodec.decode_batch(w["out"], w["off_o"], out=dec, seq=w["seq"], in_bytes=w["bytes"])
                else:
                    sbecodec.decode_batch(w["data"], w["off"], out=dec, seq=w["seq"], in_bytes=w["bytes"])

            for _ in range(2):
                step()
            torch.cuda.synchronize()
            dec = decs[(w["cur"] - 1) % len(w["sets"])]
            if rnd == 0 and not args.no_check:  # every build must produce the same bytes and descriptors
                h = (int(dec.status.to(torch.int64).sum()), int(dec.view_off.to(torch.int64).sum()),
                     int(dec.view_len.to(torch.int64).sum()), int(dec.ts.sum()))
                if w["enc"]:
                    m = int(w["off_o"][-1])
                    h += (m, int(w["out"][:m].to(torch.int64).sum()), int(w["off_o"].sum()))
                ref.setdefault(k, h)
                assert h == ref[k], f"{p} {k}: output differs from {args.libs[0]}"
            sbecodec.profile_enable(1)
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            res[(p, k)]["pack"] += sbecodec.profile_read(sbecodec.PROF_PACK)
            res[(p, k)]["dec"] += sbecodec.profile_read(sbecodec.PROF_DECODE)
            sbecodec.profile_enable(0)
            if args.phases and rnd == 0 and w["enc"] and hasattr(sbecodec.lib(), "sbe_debug_phases"):
                nwg = 16384
                buf = np.zeros(8 * nwg, np.uint64)
                sbecodec.lib().sbe_debug_phases(buf.ctypes.data_as(ctypes.c_void_p), nwg)
                ph = buf.reshape(nwg, 8).astype(np.float64)
                live = ph.sum(1) > 0
                tot = ph[live].sum(0)
                names = ["load+win+issue", "chunks", "fixup", "literal", "store", "stage_wr", "slow", "prepare"]
                print(f"phases {k:8s} {os.path.basename(p):18s} waves {int(live.sum())} mean wave clk "
                      f"{ph[live].sum(1).mean():.0f}: " + " ".join(f"{nm} {v / tot.sum():.3f}" for nm, v in zip(names, tot)),
                      flush=True)
            del ws, dec, decs
for k in works:
    for p in args.libs:
        r = res[(p, k)]
        pk = f"pack med {np.median(r['pack']) * 1e3:8.1f} us" if r["pack"] else " " * 21
        if r["pack"] and "lite" not in works[k] and not works[k]["session"]:  # algorithmic TB/s
            alg = 2 * int(works[k]["l"].sum()) + (18 + 34) * works[k]["n"]
            pk += f" {alg / (np.median(r['pack']) * 1e-3) / 1e12:5.2f} TB/s"
        print(f"{k:8s} {os.path.basename(p):22s} {pk} | decode med {np.median(r['dec']) * 1e3:8.1f} us "
              f"(min {np.min(r['dec']) * 1e3:8.1f})", flush=True)
