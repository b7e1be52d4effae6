"""bench.py — SBE records encoded+decoded/sec (device-resident), 256 B Order msgs.

One step = one round trip of the hot path over one batch resident in HBM:
  sbe_encode_topic_batch (wire-correct TopicMessages, packed SoA input → packed stream + offsets)
  → sbe_decode_batch(PARSE_MESSAGE) (stream + offsets → per-record descriptors)
    with ParseResult.sequence_number evaluated in the same launch for flagged records (this
    workload's payloads carry no "_sequence_number" and no escapes, as the Order JSON of the
    reference has none, so nothing is evaluated; --separate-seq uses the standalone launch).
Workload (BASELINE.json configs[1] extended to the metric's encode+decode): 1,000,000 fixed-256 B
Order TopicMessages per GPU (seed 0x5EED0002 + rank), synthetic.

Multi-GPU: one process per GPU (torch.distributed, RCCL), records sharded by contiguous ranges,
no data-path collective: weak scaling (the optional --gather leg times the RCCL gather of the
encoded shards to rank 0 separately, never inside `value`).

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (algorithmic bytes per
launch ÷ its average duration from HIP events on the launch stream) and the CPU baseline (the
oracle restatement, OpenMP, timed on a bounded sample on rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "aeron-cluster-client-cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import sbecodec  # noqa: E402

METRIC = "SBE records encoded+decoded/sec (device-resident), 256 B Order msgs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# algorithmic bytes per 256-B record
ENC_BYTES = 222 + 20 + 8 + 256 + 8 + 1  # pack kernel: strings + lengths + ts read; record + out_off + status written
DEC_BYTES = 256 + 8 + 2 + 8 + 8 + 40    # record + rec_off read; status,flags + hdr + ts + 5 views written


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--records", type=int, default=1_000_000, help="records per GPU")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget (rank 0)")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--separate-seq", action="store_true",
                   help="sequence_number evaluation as its own launch (sbe_eval_sequence_numbers)")
    p.add_argument("--gather", action="store_true", help="also time the RCCL gather of encoded shards")
    p.add_argument("--verify", action="store_true", help="check one step against the oracle (small n)")
    p.add_argument("--event-every", type=int, default=4,
                   help="HIP events on the pack / decode dispatches of every k-th timed step (0: none, "
                        "diagnosis only: kernel times then come from an extra untimed pass)")
    return p.parse_args()


def launched_distributed():
    """Started by torch.distributed.run (even at one process): RCCL is initialised, so a one-GPU
    run exercises the same barrier / max-over-ranks path the multi-GPU runs take."""
    return "LOCAL_RANK" in os.environ and "MASTER_ADDR" in os.environ


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or launched_distributed():
        torch.cuda.set_device(local)
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def barrier(world):
    if dist_on():
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if not dist_on():
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_inputs(n, rank, dev):
    import sbe_testlib as T
    arena, L, ts = T.fixed256_orders(n, seed=0x5EED0002 + rank)
    return (torch.from_numpy(arena).to(dev), torch.from_numpy(L.view(np.int32)).to(dev),
            torch.from_numpy(ts.view(np.int64)).to(dev))


def cpu_baseline(n_sample, budget_s, threads):
    """Oracle restatement (port of src/sbe_encoder.cpp encode + parse_message) on the host cores:
    repeat the round trip over an n_sample-record slice of the same workload until budget_s."""
    import sbe_testlib as T
    arena, L, ts = T.fixed256_orders(n_sample)
    T.oracle_encode(arena[:222], L[:1], ts[:1])  # load/build

    def run(nthreads, budget):
        done, t0 = 0, time.perf_counter()
        while True:
            out, off, _ = T.oracle_encode(arena, L, ts, nthreads=nthreads)
            d = T.oracle_decode(out, off, T.DEC_PARSE, nthreads=nthreads)
            T.oracle_seq_batch(out, off, d, nthreads=nthreads)
            done += n_sample
            el = time.perf_counter() - t0
            if el >= budget:
                return done / el

    r1 = run(1, budget_s * 0.25)
    rt = run(threads, budget_s * 0.75)
    return dict(value=rt, unit="records/s", cores=threads, kind="port",
                sample=f"{n_sample} fixed-256 records, encode+parse_message round trip repeated for "
                       f"{budget_s:.0f} s (oracle/sbe_oracle.c, OpenMP {threads} threads; 1 thread: {r1:.4g} rec/s)",
                value_1thread=r1)


def main():
    args = parse_args()
    world, rank, local = setup_dist(args)
    sbecodec.require_device()
    dev = torch.device("cuda", local)
    n = args.records
    arena, L, ts = make_inputs(n, rank, dev)
    cap = sbecodec.output_bound(n, int(arena.numel()))
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    ws = sbecodec.alloc_workspace(n, dev)
    dec = sbecodec.alloc_decoded(n, dev)
    seq = torch.zeros(n, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    ev_enc = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    ev_dec = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(k=None):
        # k is not None: the untimed pass that brackets the whole encode / decode calls with
        # torch events (the timed steps carry only the library's kernel events)
        if k is not None:
            ev_enc[k][0].record(stream)
        sbecodec.encode_topic_batch(arena, L, ts, out=out, out_off=out_off, status=status, workspace=ws,
                                    stream=stream)
        if k is not None:
            ev_enc[k][1].record(stream)
            ev_dec[k][0].record(stream)
        if args.separate_seq:
            sbecodec.decode_batch(out, out_off, mode=sbecodec.DEC_PARSE_MESSAGE, out=dec, stream=stream)
            sbecodec.eval_sequence_numbers(out, out_off, dec, seq=seq, stream=stream)
        else:
            sbecodec.decode_batch(out, out_off, mode=sbecodec.DEC_PARSE_MESSAGE, out=dec, stream=stream, seq=seq)
        if k is not None:
            ev_dec[k][1].record(stream)

    for _ in range(args.warmup):
        step()
    sbecodec.profile_enable(args.event_every)  # events on the pack / decode dispatches
    if args.verify:
        torch.cuda.synchronize()
        import sbe_testlib as T
        eo, eoff, _ = T.oracle_encode(arena.cpu().numpy(), L.cpu().numpy().view(np.uint32),
                                      ts.cpu().numpy().view(np.uint64))
        assert np.array_equal(out_off.cpu().numpy().view(np.uint64), eoff)
        assert np.array_equal(out[: int(eoff[-1])].cpu().numpy(), eo)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world)
    # the dominant kernels' durations, from the events the library recorded around them on the
    # launch stream inside the timed region
    if args.event_every == 0:  # diagnosis: kernel times from an extra, untimed pass
        sbecodec.profile_enable(1)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    pack_ms = float(np.mean(sbecodec.profile_read(sbecodec.PROF_PACK)))
    deck_ms = float(np.mean(sbecodec.profile_read(sbecodec.PROF_DECODE)))
    sbecodec.profile_enable(0)

    # informational, untimed: whole-call encode (sums + scan + pack) and decode times
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_enc]))
    dec_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_dec]))
    total = n * world * args.steps
    value = total / el

    gather = None
    if args.gather and world > 1:
        gather = time_gather(out, out_off, n, world, rank, dev)

    if rank == 0:
        enc_gbs = n * ENC_BYTES / (enc_ms * 1e-3) / 1e9
        dec_gbs = n * DEC_BYTES / (dec_ms * 1e-3) / 1e9
        pack_gbs = n * ENC_BYTES / (pack_ms * 1e-3) / 1e9
        deck_gbs = n * DEC_BYTES / (deck_ms * 1e-3) / 1e9
        if pack_ms >= deck_ms:
            dom = dict(kernel="sbe_enc_pack<packed,wire>", bytes_per_record=ENC_BYTES, ms=pack_ms, gbs=pack_gbs)
        else:
            dom = dict(kernel="sbe_decode_kernel<parse_message>", bytes_per_record=DEC_BYTES, ms=deck_ms,
                       gbs=deck_gbs)
        traffic = measured_traffic(dom["kernel"], n)
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            cpu = cpu_baseline(min(n, 200_000), args.cpu_seconds, args.cpu_threads)
        line = {
            "metric": METRIC, "value": value, "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "roundtrip_fixed256_orders", "records_per_gpu": n, "record_bytes": 256,
                       "encode": "wire-correct TopicMessage, packed SoA input",
                       "decode": "parse_message descriptors (views) + sequence_number evaluation", "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": dom["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": dom["gbs"] / HBM_PEAK_GBS, "traffic": traffic, "kernel": dom["kernel"],
                         "kernel_ms": dom["ms"], "bytes_per_record": dom["bytes_per_record"],
                         "timing": (f"HIP events on the kernel's dispatch in every {args.event_every}th timed step"
                                    if args.event_every else "HIP events, untimed pass (diagnosis run)")},
            "kernels": {"encode_ms": enc_ms, "encode_gbs": enc_gbs, "decode_ms": dec_ms, "decode_gbs": dec_gbs,
                        "pack_ms": pack_ms, "pack_gbs": pack_gbs, "decode_kernel_ms": deck_ms,
                        "decode_kernel_gbs": deck_gbs,
                        "roundtrip_gbs": n * (ENC_BYTES + DEC_BYTES) / ((enc_ms + dec_ms) * 1e-3) / 1e9},
            "cpu_baseline": cpu,
        }
        if gather is not None:
            line["gather"] = gather
        print(json.dumps(line), flush=True)
    if dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()


def measured_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the committed PMC summary (scripts/gpu_counters.sh →
    profiles/traffic.json: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM), scaled from the
    records per launch it was measured at; None when no summary covers the kernel."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(path))[kernel]
    except (OSError, KeyError, ValueError):
        return None
    return d["bytes_per_launch"] * n / d["records"]


def time_gather(out, out_off, n, world, rank, dev):
    """RCCL gatherv of the encoded shards to rank 0 (grouped send/recv at prefix offsets)."""
    sys.path.insert(0, os.path.join(ROOT, "aeron-cluster-client-cpp_amd"))
    import shard
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    g = shard.gather_encoded(out, out_off, n, root=0)
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world)
    nbytes = int(out_off[n].item()) * world
    return {"seconds": el, "bytes": nbytes, "GBps_into_root": nbytes * (world - 1) / world / el / 1e9,
            "ok": bool(g is not None) if rank == 0 else True}


if __name__ == "__main__":
    main()
