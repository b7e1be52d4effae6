"""Per-row measurement of the SURVEY §8 rows beyond the headline bench: one JSON line per workload
with records/s (whole calls, device-resident), each dominant kernel's HIP-event duration, its
algorithmic bytes per launch (computed from the actual record sizes) and its fraction of the
8 TB/s HBM peak.  Rows:
  config3_mixed_decode   1 M mixed TopicMessage / Ack records, parse_message
  config4_var_roundtrip  16 M variable-length TopicMessages, encode + parse decode (config 4)
  session_fixed256       1 M session-framed Order TopicMessages (32-B SessionMessageHeader + 248 B)
  lite301 / lite201      1 M CommitOffsetLite / OrderRequestLite records, encode + Lite decode
  order_json             1 M Orders → Order::to_json payload + publish_order headers JSON (two calls)
  reassemble             1 M Aeron fragments (90 % whole messages, the rest BEGIN..END groups),
                         BEGIN/END reassembly (all its launches, torch events around the call)
  materialize            1 M fixed-256 records' parse_message views copied into one arena
                         (sbe_materialize_views, all its launches, torch events around the call)
Rows whose buffers fit the 256 MB MALL a few times over rotate over --rotate (3) copies of their
inputs and outputs (step k uses copy k mod R), as bench.py does, so no step finds its inputs in the
cache a previous step left them in; config 4's 16.8 M-record batch (~6.5 GB) needs no rotation.
Usage: python scripts/bench_rows.py [--steps K] [--rows a,b,...] [--rotate R]  (GPU only)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "aeron-cluster-client-cpp_amd"), os.path.join(ROOT, "tests")]
import sbe_testlib as T  # noqa: E402
import sbecodec  # noqa: E402

PEAK = 8000.0
DESC = 1 + 1 + 8 + 8 + 40  # decode descriptor bytes written per record


def dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a).view({torch.uint8: np.uint8, torch.int32: np.int32,
                                                           torch.int64: np.int64}[dt])).to("cuda")


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    sbecodec.profile_enable(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    pack = sbecodec.profile_read(sbecodec.PROF_PACK)
    deck = sbecodec.profile_read(sbecodec.PROF_DECODE)
    sbecodec.profile_enable(0)
    return el / steps, (float(np.mean(pack)) if pack else None), (float(np.mean(deck)) if deck else None)


ROT = 3  # --rotate


class Rot:
    """R copies of a row's device buffers; next() is the copy for the next step."""

    def __init__(self, make):
        self.sets = [make(k) for k in range(max(ROT, 1))]
        self.k = 0

    def next(self):
        x = self.sets[self.k % len(self.sets)]
        self.k += 1
        return x


CPU_THREADS = 16
CPU_SECONDS = 3.0
NO_CPU = False  # --no-cpu: skip the CPU baselines (profiling runs)


def cpu_rate(fn, n_sample, budget=CPU_SECONDS):
    """records/s of fn() (the oracle restatement of the row on an n_sample-record slice of the same
    workload) repeated for about `budget` seconds on the host cores."""
    if NO_CPU:
        return None
    fn()
    done, t0 = 0, time.perf_counter()
    while True:
        fn()
        done += n_sample
        el = time.perf_counter() - t0
        if el >= budget:
            return done / el


_cpu = None


def line(row, n, step_s, kernels):
    global _cpu
    out = {"row": row, "records": n, "records_per_s": n / step_s, "ms_per_step": step_s * 1e3,
           "input_sets": 1 if row == "config4_var_roundtrip" else max(ROT, 1), "kernels": {}}
    if _cpu is not None:
        out["cpu_baseline"] = _cpu
        _cpu = None
    for name, (ms, nbytes) in kernels.items():
        if ms is None:
            continue
        gbs = nbytes / (ms * 1e-3) / 1e9
        out["kernels"][name] = {"ms": ms, "alg_bytes": nbytes, "GBps": gbs, "frac": gbs / PEAK}
    print(json.dumps(out), flush=True)


def set_cpu(value, sample, cores=CPU_THREADS):
    global _cpu
    if value is None:
        return
    _cpu = {"value": value, "unit": "records/s", "cores": cores, "kind": "port", "sample": sample}


def row_mixed(steps, warmup):
    n = 1_000_000
    data, off = T.mixed_records(n)
    d0, o0 = dev(data, torch.uint8), dev(off.astype(np.uint64), torch.int64)
    R = Rot(lambda k: (d0.clone(), o0.clone(), sbecodec.alloc_decoded(n, "cuda")))
    nb = int(off[-1])

    def step():
        d, o, out = R.next()
        sbecodec.decode_batch(d, o, sbecodec.DEC_PARSE_MESSAGE, out=out, in_bytes=nb)

    s, _, dk = timed(step, steps, warmup)
    k = 200_000
    dk_, ok_ = data[: int(off[k])], off[: k + 1]
    set_cpu(cpu_rate(lambda: T.oracle_decode(dk_, ok_, T.DEC_PARSE, nthreads=CPU_THREADS), k),
            f"{k} records of the same mix, oracle parse_message, OpenMP {CPU_THREADS} threads")
    line("config3_mixed_decode", n, s, {"sbe_decode_kernel<parse_message>": (dk, int(off[-1]) + 8 * n + DESC * n)})


def row_var(steps, warmup):
    n = 16_777_216
    a, l, t = T.var_orders_t(n, "cuda")  # == T.var_orders(n), generated on the device
    cap = sbecodec.output_bound(n, a.numel())
    ob = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    ws = sbecodec.alloc_workspace(n, "cuda")
    dec = sbecodec.alloc_decoded(n, "cuda")
    outb = int(a.numel()) + 34 * n  # the stream's bytes (every record encodable)

    def step():
        sbecodec.encode_topic_batch(a, l, t, out=ob, out_off=oo, status=st, workspace=ws)
        sbecodec.decode_batch(ob, oo, sbecodec.DEC_PARSE_MESSAGE, out=dec, in_bytes=outb)

    s, pk, dk = timed(step, steps, warmup)
    k = 200_000
    ak, Lk, tk = T.var_orders(k)

    def cpu_rt():
        o, oo_, _ = T.oracle_encode(ak, Lk, tk, nthreads=CPU_THREADS)
        T.oracle_decode(o, oo_, T.DEC_PARSE, nthreads=CPU_THREADS)

    set_cpu(cpu_rate(cpu_rt, k), f"{k} variable-length records, oracle encode + parse_message, OpenMP {CPU_THREADS} threads")
    line("config4_var_roundtrip", n, s, {"sbe_enc_pack<packed,wire>": (pk, a.numel() + 28 * n + outb + 9 * n),
                                         "sbe_decode_kernel<parse_message>": (dk, outb + 8 * n + DESC * n)})


def row_session(steps, warmup):
    n = 1_000_000
    arena, L, ts = T.fixed256_orders(n)
    a0, l0, t0 = dev(arena, torch.uint8), dev(L.view(np.int32), torch.int32), dev(ts.view(np.int64), torch.int64)
    ws = sbecodec.alloc_workspace(n, "cuda")
    R = Rot(lambda k: (a0.clone(), l0.clone(), t0.clone(),
                       torch.empty(sbecodec.output_bound(n, arena.size), dtype=torch.uint8, device="cuda"),
                       torch.empty(n + 1, dtype=torch.int64, device="cuda"),
                       torch.empty(n, dtype=torch.uint8, device="cuda"), sbecodec.alloc_decoded(n, "cuda")))

    def step():
        a, l, t, ob, oo, st, dec = R.next()
        sbecodec.encode_session_batch(a, l, t, 7, 8, out=ob, out_off=oo, status=st, workspace=ws)
        sbecodec.decode_batch(ob, oo, sbecodec.DEC_PARSE_MESSAGE, out=dec, in_bytes=n * (32 + 248))

    s, pk, dk = timed(step, steps, warmup)
    rec = 32 + 248
    k = 200_000
    ak, Lk, tk = arena[: 222 * k], L[:k], ts[:k]

    def cpu_rt():
        o, oo_, _ = T.oracle_encode_session(ak, Lk, tk, 7, 8, flags=T.ENC_REF_TRUNCATE8, nthreads=CPU_THREADS)
        T.oracle_decode(o, oo_, T.DEC_PARSE, nthreads=CPU_THREADS)

    set_cpu(cpu_rate(cpu_rt, k), f"{k} records, oracle session encode + parse_message, OpenMP {CPU_THREADS} threads")
    line("session_fixed256", n, s, {"sbe_enc_pack<session,packed,ref>": (pk, n * (222 + 28 + rec + 9)),
                                    "sbe_decode_kernel<parse_message>": (dk, n * (rec + 8 + DESC))})


def row_lite(t_id, steps, warmup):
    n = 1_000_000
    nf = T.LITE_NF[t_id]
    arena, L, tid, seq = T.lite_records(n, t_id)
    a0, l0 = dev(arena, torch.uint8), dev(L.view(np.int32), torch.int32)
    ti0, sq0 = dev(tid.view(np.int32), torch.int32), dev(seq.view(np.int64), torch.int64)
    cap = arena.size + (20 + 2 * nf) * n + 16
    ws = sbecodec.alloc_workspace(n, "cuda")
    outb = arena.size + (20 + 2 * nf) * n
    R = Rot(lambda k: (a0.clone(), l0.clone(), ti0.clone(), sq0.clone(),
                       torch.empty(cap, dtype=torch.uint8, device="cuda"),
                       torch.empty(n + 1, dtype=torch.int64, device="cuda"),
                       torch.empty(n, dtype=torch.uint8, device="cuda"), sbecodec.alloc_decoded(n, "cuda")))

    def step():
        a, l, ti, sq, ob, oo, st, dec = R.next()
        sbecodec.encode_lite_batch(t_id, a, l, ti, sq, out=ob, out_off=oo, status=st, workspace=ws)
        sbecodec.decode_batch(ob, oo, sbecodec.DEC_LITE, out=dec, in_bytes=outb)

    s, pk, dk = timed(step, steps, warmup)
    k = 200_000
    ak, Lk, tk, sk = T.lite_records(k, t_id)

    def cpu_rt():
        o, oo_, _ = T.oracle_encode_lite(t_id, ak, Lk, tk, sk, nthreads=CPU_THREADS)
        T.oracle_decode(o, oo_, T.DEC_LITE, nthreads=CPU_THREADS)

    set_cpu(cpu_rate(cpu_rt, k), f"{k} records, oracle Lite encode + decode, OpenMP {CPU_THREADS} threads")
    line(f"lite{t_id}", n, s, {f"sbe_enc_pack<lite{nf},packed>": (pk, arena.size + (4 * nf + 12) * n + outb + 9 * n),
                               "sbe_decode_kernel<lite>": (dk, outb + 8 * n + DESC * n)})


def row_reassemble(steps, warmup):
    n = 1_000_000
    # 90 % whole messages, 10 % BEGIN..END groups of 2-5 fragments, no strays
    data, off, flags = T.fragment_stream(n, 11, p_single=0.9, maxlen=512, p_group=0.1)
    d0, o0, f0 = dev(data, torch.uint8), dev(off.view(np.int64), torch.int64), dev(flags, torch.uint8)
    ws = torch.empty(int(sbecodec.lib().sbe_reassemble_workspace_size(n)), dtype=torch.uint8, device="cuda")
    R = Rot(lambda k: (d0.clone(), o0.clone(), f0.clone(), torch.empty(max(data.size, 16), dtype=torch.uint8, device="cuda"),
                       torch.empty(n + 1, dtype=torch.int64, device="cuda")))

    def fn():
        d, o, f, out, mo = R.next()
        sbecodec.reassemble(d, o, f, out=out, msg_off=mo, workspace=ws)
    for _ in range(warmup):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    nbytes = 2 * data.size + (8 + 1 + 8) * n  # payload read + written, frag_off + flags read, msg_off written
    k = 200_000
    dk_, ok_, fk_ = data[: int(off[k])], np.ascontiguousarray(off[: k + 1]), np.ascontiguousarray(flags[:k])
    ob_, ab_ = np.zeros(int(off[k]) + 1, np.uint8), np.zeros(int(off[k]) + 1, np.uint8)
    mo_, cn_ = np.zeros(k + 1, np.uint64), np.zeros(2, np.uint64)
    P = T._p
    set_cpu(cpu_rate(lambda: T.oracle().orc_reassemble(P(dk_), P(ok_), P(fk_), k, P(ob_), P(mo_), P(cn_), P(ab_)), k),
            f"{k} fragments of the same stream, oracle LocalFragmentReassembler restatement, 1 thread (sequential by definition)",
            cores=1)
    line("reassemble", n, ms * 1e-3, {"sbe_reassemble_fragments (all launches)": (ms, nbytes)})


def row_order_json(steps, warmup):
    n = 1_000_000
    fields, cid, ts, q = T.realistic_orders(n)
    arena, str_len = T.pack_order_fields(fields)
    args0 = (dev(arena, torch.uint8), dev(str_len.astype(np.int32), torch.int32), dev(cid, torch.int64),
             dev(ts, torch.int64), torch.from_numpy(q).cuda())

    def make(k):
        args = tuple(x.clone() for x in args0)
        outs = {w: sbecodec.order_to_json_batch(*args, what=w)
                for w in (sbecodec.JSON_ORDER_PAYLOAD, sbecodec.JSON_PUBLISH_HEADERS)}
        return args, outs

    R = Rot(make)
    outs = R.sets[0][1]

    def fn():
        args, os_ = R.next()
        for w in os_:
            sbecodec.order_to_json_batch(*args, what=w, out=os_[w].out, out_off=os_[w].out_off, status=os_[w].status)
    for _ in range(warmup):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    text = sum(int(outs[w].out_off[-1]) for w in outs)
    # strings read (payload reads uuid / base twice), lengths + numbers read, text + offsets written
    sl = str_len.astype(np.int64)
    nbytes = int(2 * sl[:, 0].sum() + sl[:, 1:5].sum() + sl[:, 2].sum() + sl[:, 5:8].sum()) + n * (32 + 24) + \
        text + 2 * 8 * n
    k = 100_000
    ak, lk = T.pack_order_fields(fields[:k])
    set_cpu(cpu_rate(lambda: [T.oracle_order_json(ak, lk, cid[:k], ts[:k], q[:k], w, nthreads=CPU_THREADS)
                              for w in (0, 1)], k),
            f"{k} Orders of the same batch, oracle payload + headers JSON (glibc snprintf), OpenMP {CPU_THREADS} threads")
    line("order_json", n, ms * 1e-3, {"sbe_order_to_json_batch x2 (payload + headers)": (ms, nbytes)})


def row_materialize(steps, warmup):
    """MATERIALIZE (sbe_materialize_views) after a parse_message decode of 1 M fixed-256 records:
    every record's views copied into one arena (Σlen read and written, plus the
    descriptors' offsets and lengths and rec_off read and 40 B of arena offsets written a record)."""
    n = 1_000_000
    arena, L, ts = T.fixed256_orders(n)
    data, off, _ = T.oracle_encode(arena, L, ts)
    d0, o0 = dev(data, torch.uint8), dev(off.astype(np.uint64), torch.int64)
    ws = torch.empty(int(sbecodec.lib().sbe_materialize_workspace_size(n)) + 16, dtype=torch.uint8, device="cuda")

    def make(k):
        d, o = d0.clone(), o0.clone()
        dec = sbecodec.decode_batch(d, o, sbecodec.DEC_PARSE_MESSAGE, out=sbecodec.alloc_decoded(n, "cuda"),
                                    in_bytes=data.size)
        return d, o, dec, torch.empty(data.size, dtype=torch.uint8, device="cuda"), \
            torch.empty(5 * n + 1, dtype=torch.int64, device="cuda")
    R = Rot(make)
    torch.cuda.synchronize()
    vbytes = int(R.sets[0][2].view_len[:n].to(torch.int64).sum().item())

    def fn():
        d, o, dec, ar, ao = R.next()
        sbecodec.materialize_views(d, o, dec, arena=ar, arena_capacity=ar.numel(), arena_off=ao, workspace=ws)
    for _ in range(warmup):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    nbytes = 2 * vbytes + (40 + 8 + 40) * n
    k = 200_000
    dk = T.oracle_decode(data[: int(off[k])], off[: k + 1], T.DEC_PARSE, nthreads=CPU_THREADS)
    set_cpu(cpu_rate(lambda: T.oracle_materialize(data[: int(off[k])], off[: k + 1], dk), k),
            f"{k} records of the same batch, the oracle's view copy (numpy gather), 1 thread", cores=1)
    line("materialize", n, ms * 1e-3, {"sbe_materialize_views (all launches)": (ms, nbytes)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", default="mixed,var,session,lite301,lite201,reassemble,order_json,materialize")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baselines")
    ap.add_argument("--lib", help="library build to measure (A/B of variants; default: the product's)")
    ap.add_argument("--rotate", type=int, default=3, help="copies of a row's buffers the steps rotate over")
    args = ap.parse_args()
    global ROT
    ROT = args.rotate
    if args.lib:
        sbecodec.use_library(os.path.abspath(args.lib))
    global NO_CPU
    NO_CPU = args.no_cpu
    sbecodec.require_device()
    for r in args.rows.split(","):
        if r == "mixed":
            row_mixed(args.steps, args.warmup)
        elif r == "var":
            row_var(max(args.steps // 2, 5), args.warmup)
        elif r == "session":
            row_session(args.steps, args.warmup)
        elif r == "reassemble":
            row_reassemble(args.steps, args.warmup)
        elif r == "order_json":
            row_order_json(args.steps, args.warmup)
        elif r == "materialize":
            row_materialize(args.steps, args.warmup)
        elif r.startswith("lite"):
            row_lite(int(r[4:]), args.steps, args.warmup)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
