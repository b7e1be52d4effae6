"""bench.py — SBE records encoded+decoded/sec (device-resident), 256 B Order msgs.

One step = one round trip of the hot path over one batch resident in HBM:
  sbe_encode_topic_batch (wire-correct TopicMessages, packed SoA input → packed stream + offsets)
  → sbe_decode_batch(PARSE_MESSAGE) (stream + offsets → per-record descriptors)
    with ParseResult.sequence_number evaluated in the same launch for flagged records (this
    workload's payloads carry no "_sequence_number" and no escapes, as the Order JSON of the
    reference has none, so nothing is evaluated; --separate-seq uses the standalone launch).
Workload (BASELINE.json configs[1] extended to the metric's encode+decode): 1,000,000 fixed-256 B
Order TopicMessages per GPU (seed 0x5EED0002 + rank), synthetic.  The
steps rotate over --sets (3) distinct sets of inputs and outputs, so that no step reads what the
previous one left in the 256 MB MALL (a 1 M-record set is ~0.58 GB); the roofline comes from the
rotated steps, and the one-set (warm-cache) figure rides beside it as `frac_warm`.

Multi-GPU: one process per GPU (torch.distributed, RCCL).  `--gpus N` outside a launcher starts
N ranks through torch.distributed.run before touching the GPU.  The headline shards records by
contiguous ranges with no data-path collective: weak scaling, `value` = all ranks' records ÷ the
slowest rank's time.  The `config5` object (BASELINE.json configs[4]) is strong
scaling: one 134,217,728-record fixed-256 batch split over the ranks with shard.shard_range,
encode-only and encode + the RCCL gather of the encoded shards to rank 0 (sbe_gather_encoded),
each with absolute rec/s and its fraction of the HBM / xGMI roofline.

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (SURVEY §8(d)'s
algorithmic bytes per launch ÷ its average duration from HIP events on the launch stream) and the
CPU baseline (the oracle restatement, OpenMP, timed on a bounded sample on rank 0 at N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "aeron-cluster-client-cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import sbecodec  # noqa: E402  (lazy: the library loads on first use)

METRIC = "SBE records encoded+decoded/sec (device-resident), 256 B Order msgs"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
XGMI_ROOT_GBS = 7 * 153.0  # root ingress: 7 xGMI links x ~153 GB/s
# algorithmic bytes per 256-B record, SURVEY §8(d) (the roofline figures):
#   encode 8 ts + 10 lengths + 222 strings read + 256 record written; decode 256 record + 8
#   rec_off read + 48 descriptor written
ENC_BYTES = 496
DEC_BYTES = 312
# the same with what the kernels also move: u32 lengths (20 B, not 10), out_off + status written;
# the decode descriptor as laid out here (58 B)
ENC_BYTES_ALL = 222 + 20 + 8 + 256 + 8 + 1
DEC_BYTES_ALL = 256 + 8 + 2 + 8 + 8 + 40


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--records", type=int, default=1_000_000, help="records per GPU (headline)")
    p.add_argument("--sets", type=int, default=3,
                   help="distinct input / output buffer sets the steps rotate over (step k uses set k mod S). "
                        "Three 1 M-record sets put ~1.7 GB of other traffic between two reads of one set, so no "
                        "step finds its inputs in the 256 MB MALL; --sets 1 is the old warm-cache workload")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget (rank 0)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="host threads of the CPU baseline (0: the cores this process may use, capped by "
                        "OMP_NUM_THREADS, which the GPU box sets to its 16-core share)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-config5", action="store_true", help="skip the config-5 strong-scaling leg")
    p.add_argument("--config5-records", type=int, default=134_217_728)
    p.add_argument("--config5-steps", type=int, default=3)
    p.add_argument("--separate-seq", action="store_true",
                   help="sequence_number evaluation as its own launch (sbe_eval_sequence_numbers)")
    p.add_argument("--verify", action="store_true", help="check one step against the oracle (small n)")
    p.add_argument("--settle-ms", type=float, default=500.0,
                   help="untimed round trips before the warmup steps, until the GPU has run this long")
    p.add_argument("--event-every", type=int, default=10,
                   help="HIP events on the pack / decode dispatches of every k-th timed step (0: none).  "
                        "A timed dispatch costs the GPU ~5 us, so the timed region samples sparsely; the "
                        "roofline comes from the sampled pass that follows it (--sample-steps)")
    p.add_argument("--sample-steps", type=int, default=0,
                   help="steps of the sampled pass right after the timed region, HIP events on every pack / "
                        "decode dispatch (0: max(steps, 20), at most 256)")
    return p.parse_args()


def launched_distributed():
    """Started by torch.distributed.run (even at one process): RCCL is initialised, so a one-GPU
    run exercises the same barrier / max-over-ranks path the multi-GPU runs take."""
    return "LOCAL_RANK" in os.environ and "MASTER_ADDR" in os.environ


def spawn_ranks(n):
    """`--gpus N` without a launcher: run this script under torch.distributed.run with N ranks, one
    per GPU, as a child process (nothing here has touched the GPU), and exit with its status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


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


def host_cpu():
    """nproc, the cores this process may run on, and the CPU model (state them)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity": allowed, "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def default_cpu_threads():
    cpu = host_cpu()
    t = cpu["affinity"] or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        t = min(t, int(omp))
    return max(1, t)


def cpu_baseline(n_sample, budget_s, threads):
    """Timed on the host cores, same run, bounded sample of the headline workload:
    - the oracle restatement (a C port of src/sbe_encoder.cpp encode + parse_message), one thread and
      `threads` OpenMP threads: the full round trip;
    - the reference's own compiled code where it compiles here: the SBE flyweight sequence of
      SBEEncoder::encode_topic_message (src/sbe_encoder.cpp:141-164, oracle/_ref built from
      /root/reference/include/model), encode only, one thread and `threads` threads.
    Neither is the reference's full speed: its parse_message also builds std::strings, runs jsoncpp
    and evaluates DEBUG_LOG arguments per record."""
    import sbe_testlib as T
    arena, L, ts = T.fixed256_orders(n_sample)
    T.oracle_encode(arena[:222], L[:1], ts[:1])  # load/build

    def timed(fn, budget):
        done, t0 = 0, time.perf_counter()
        while True:
            fn()
            done += n_sample
            el = time.perf_counter() - t0
            if el >= budget:
                return done / el

    def roundtrip(nthreads):
        out, off, _ = T.oracle_encode(arena, L, ts, nthreads=nthreads)
        d = T.oracle_decode(out, off, T.DEC_PARSE, nthreads=nthreads)
        T.oracle_seq_batch(out, off, d, nthreads=nthreads)

    r1 = timed(lambda: roundtrip(1), budget_s * 0.2)
    rt = timed(lambda: roundtrip(threads), budget_s * 0.4)
    ref = None
    if T.ref_available():
        eo, eoff, _ = T.oracle_encode(arena, L, ts, flags=1)  # REF_TRUNCATE8: encode_topic_message's bytes
        ro, roff = T.ref_encode_batch(arena, L, ts, wire=False, nthreads=threads)
        same = bool(np.array_equal(ro, eo) and np.array_equal(roff, eoff))
        run, _, _ = T.ref_encode_prepared(arena, L, ts, wire=False)
        f1 = timed(lambda: run(1), budget_s * 0.15)
        ft = timed(lambda: run(threads), budget_s * 0.25)
        ref = {"what": "SBEEncoder::encode_topic_message's flyweight sequence (src/sbe_encoder.cpp:141-164), "
                       "the reference's generated TopicMessage.h compiled from /root/reference (oracle/_ref), "
                       "encode only, records/s",
               "value_1thread": f1, "value": ft, "threads": threads, "bytes_equal_to_restatement": same}
    return dict(value=rt, unit="records/s", cores=threads, kind="port",
                sample=f"{n_sample} fixed-256 records, encode+parse_message round trip repeated for "
                       f"{budget_s * 0.6:.0f} s (oracle/sbe_oracle.c, a C restatement, OpenMP {threads} threads; "
                       f"1 thread: {r1:.4g} rec/s)",
                value_1thread=r1, host=host_cpu(), reference_flyweights_encode=ref,
                reference_indicative={
                    "note": "the reference's own functions, survey container (Xeon, 8 vCPU), BASELINE.md §2; "
                            "the restatement runs without their std::string / jsoncpp / DEBUG_LOG costs",
                    "encode_topic_message_1thread": "20-24 M rec/s",
                    "parse_message_tm_1thread": "2.4-2.6 M rec/s (jsoncpp stubbed)",
                    "parse_message_tm_8threads": "2.3 M rec/s"})


def config5(args, world, rank, dev):
    """BASELINE.json configs[4] / SURVEY §8(e): one config5_records fixed-256 batch split over the
    ranks (shard.shard_range), encoded on every rank at once (no collective), then gathered to
    rank 0 over RCCL with sbe_gather_encoded.  Strong scaling: the batch size is fixed."""
    import shard
    import sbe_testlib as T
    N = args.config5_records
    lo, hi = shard.shard_range(N, world, rank)
    m = hi - lo
    arena, L, ts = T.config5_shard(lo, hi, dev)
    out = torch.empty(sbecodec.output_bound(m, int(arena.numel())), dtype=torch.uint8, device=dev)
    out_off = torch.empty(m + 1, dtype=torch.int64, device=dev)
    status = torch.empty(max(m, 1), dtype=torch.uint8, device=dev)
    ws = sbecodec.alloc_workspace(m, dev)

    def enc():
        sbecodec.encode_topic_batch(arena, L, ts, out=out, out_off=out_off, status=status, workspace=ws)

    enc()
    torch.cuda.synchronize()
    reps = max(1, args.config5_steps)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        enc()
    torch.cuda.synchronize()
    barrier(world)
    t_enc = max_over_ranks((time.perf_counter() - t0) / reps, world)
    ok = int(out_off[m].item()) == 256 * m and int((status[:m] != 0).sum().item()) == 0
    res = {"workload": "config5_fixed256_sharded", "records": N, "records_per_rank_max": -(-N // world),
           "scaling": "strong", "split": "shard.shard_range (contiguous)",
           "encode": {"seconds": t_enc, "records_per_s": N / t_enc,
                      "GBps": N * ENC_BYTES / t_enc / 1e9,
                      "frac_of_hbm_aggregate": N * ENC_BYTES / t_enc / 1e9 / (HBM_PEAK_GBS * world)}}
    if world > 1:
        g = shard.RcclGather()
        dst = dst_off = None
        if rank == 0:
            dst = torch.empty(sbecodec.output_bound(N, 222 * N), dtype=torch.uint8, device=dev)
            dst_off = torch.empty(N + 1, dtype=torch.int64, device=dev)
        g.gather(out, out_off, m, root=0, dst=dst, dst_off=dst_off)  # warm the RCCL connections
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            enc()
            _, _, nbytes, nrec = g.gather(out, out_off, m, root=0, dst=dst, dst_off=dst_off)
        torch.cuda.synchronize()
        barrier(world)
        t_eg = max_over_ranks((time.perf_counter() - t0) / reps, world)
        verify = None
        if rank == 0:
            ok = ok and nbytes == 256 * N and nrec == N
            # byte check of the whole gathered stream on the root (outside the timed region): every
            # record is a function of its global index (T.config5_shard), so the root re-encodes the
            # batch chunk by chunk on its own GPU and compares bytes and offsets with what arrived
            verify = verify_gathered(dst, dst_off, N, dev, ws)
            ok = ok and verify["mismatched_chunks"] == 0
        into_root = 256 * (N - m) if rank == 0 else 0
        into_root = int(max_over_ranks(float(into_root), world))
        res["encode_gather"] = {"seconds": t_eg, "records_per_s": N / t_eg,
                                "gather_seconds": max(t_eg - t_enc, 0.0),
                                "GBps_into_root": into_root / max(t_eg - t_enc, 1e-9) / 1e9,
                                "frac_of_xgmi_root_ingress": into_root / max(t_eg - t_enc, 1e-9) / 1e9 / XGMI_ROOT_GBS,
                                "collective": "sbe_gather_encoded (ncclAllGather of sizes + grouped ncclSend/ncclRecv)"}
        if rank == 0:
            res["encode_gather"]["verify"] = verify
        # fixed-256 shards have known sizes: the sized gather (no size all-gather, no host wait per
        # gather), every rank's encode and transfers enqueued back to back
        sizes = [(256 * (b - a), b - a) for a, b in (shard.shard_range(N, world, r) for r in range(world))]
        cap, off_cap = sbecodec.output_bound(N, 222 * N), N + 1  # the root's buffers, known to every rank
        g.gather_sized(sizes, out, out_off, root=0, dst=dst, dst_off=dst_off, dst_capacity=cap,
                       dst_off_capacity=off_cap)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            enc()
            g.gather_sized(sizes, out, out_off, root=0, dst=dst, dst_off=dst_off, dst_capacity=cap,
                           dst_off_capacity=off_cap)
        torch.cuda.synchronize()
        barrier(world)
        t_egs = max_over_ranks((time.perf_counter() - t0) / reps, world)
        verify_s = None
        if rank == 0:
            verify_s = verify_gathered(dst, dst_off, N, dev, ws)
            ok = ok and verify_s["mismatched_chunks"] == 0
        res["encode_gather_sized"] = {"seconds": t_egs, "records_per_s": N / t_egs,
                                      "gather_seconds": max(t_egs - t_enc, 0.0),
                                      "GBps_into_root": into_root / max(t_egs - t_enc, 1e-9) / 1e9,
                                      "frac_of_xgmi_root_ingress":
                                          into_root / max(t_egs - t_enc, 1e-9) / 1e9 / XGMI_ROOT_GBS,
                                      "collective": "sbe_gather_encoded_sized (grouped ncclSend/ncclRecv only)"}
        if rank == 0:
            res["encode_gather_sized"]["verify"] = verify_s
        g.close()
        del dst, dst_off
    else:
        res["encode_gather"] = {"seconds": t_enc, "records_per_s": N / t_enc,
                                "note": "one GPU: the encoded batch already sits on the root"}
    res["ok"] = bool(ok)
    del arena, L, ts, out, out_off, status, ws
    torch.cuda.empty_cache()
    return res


def verify_gathered(dst, dst_off, N, dev, ws, chunk=1 << 22):
    """The root's gathered config-5 stream == a single-GPU encode of the same records: records
    [a, b) regenerated from their global indices, encoded here, compared byte for byte with
    dst[256 a : 256 b] and dst_off[a : b + 1] (fixed-256 records: offsets 256 i)."""
    import sbe_testlib as T
    bad, t0 = 0, time.perf_counter()
    out = torch.empty(256 * chunk + 16, dtype=torch.uint8, device=dev)
    off = torch.empty(chunk + 1, dtype=torch.int64, device=dev)
    for a in range(0, N, chunk):
        b = min(N, a + chunk)
        arena, L, ts = T.config5_shard(a, b, dev)
        sbecodec.encode_topic_batch(arena, L, ts, out=out, out_off=off[: b - a + 1], status=False, workspace=ws)
        same = torch.equal(out[: 256 * (b - a)], dst[256 * a: 256 * b]) and \
            torch.equal(off[: b - a + 1] + 256 * a, dst_off[a: b + 1])
        bad += 0 if same else 1
    torch.cuda.synchronize()
    return {"records": N, "chunk_records": chunk, "mismatched_chunks": bad,
            "method": "root re-encodes the closed-form config-5 records chunk by chunk and compares bytes + offsets",
            "seconds": time.perf_counter() - t0}


def main():
    args = parse_args()
    if args.sample_steps <= 0:
        args.sample_steps = min(256, max(args.steps, 20))
    if args.gpus > 1 and not launched_distributed():
        sys.exit(spawn_ranks(args.gpus))
    world, rank, local = setup_dist(args)
    sbecodec.require_device()
    dev = torch.device("cuda", local)
    n = args.records
    nsets = max(1, args.sets)
    # S distinct sets of inputs and outputs (step k uses set k mod S): every set has its own arena,
    # lengths, timestamps, encoded stream, offsets, status and descriptors, so a step reads nothing
    # that the previous step left in the caches (MI355X_MICROARCH.md: 256 MB MALL)
    sets = []
    for k in range(nsets):
        arena, L, ts = make_inputs(n, rank + (k << 16), dev)
        cap = sbecodec.output_bound(n, int(arena.numel()))
        sets.append(dict(arena=arena, L=L, ts=ts, out=torch.empty(cap, dtype=torch.uint8, device=dev),
                         out_off=torch.empty(n + 1, dtype=torch.int64, device=dev),
                         status=torch.empty(n, dtype=torch.uint8, device=dev),
                         dec=sbecodec.alloc_decoded(n, dev), seq=torch.zeros(n, dtype=torch.int64, device=dev)))
    ws = sbecodec.alloc_workspace(n, dev)
    stream = torch.cuda.current_stream()

    ev_enc = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    ev_dec = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    rot = {"i": 0, "only": None}  # next set; "only": pin every step to one set (the warm-cache pass)

    def step(k=None):
        # k is not None: the untimed pass that brackets the whole encode / decode calls with
        # torch events (the timed steps carry only the library's kernel events)
        b = sets[rot["only"] if rot["only"] is not None else rot["i"] % nsets]
        rot["i"] += 1
        if k is not None:
            ev_enc[k][0].record(stream)
        sbecodec.encode_topic_batch(b["arena"], b["L"], b["ts"], out=b["out"], out_off=b["out_off"],
                                    status=b["status"], workspace=ws, stream=stream)
        if k is not None:
            ev_enc[k][1].record(stream)
            ev_dec[k][0].record(stream)
        if args.separate_seq:
            sbecodec.decode_batch(b["out"], b["out_off"], mode=sbecodec.DEC_PARSE_MESSAGE, out=b["dec"], stream=stream)
            sbecodec.eval_sequence_numbers(b["out"], b["out_off"], b["dec"], seq=b["seq"], stream=stream)
        else:
            sbecodec.decode_batch(b["out"], b["out_off"], mode=sbecodec.DEC_PARSE_MESSAGE, out=b["dec"],
                                  stream=stream, seq=b["seq"])
        if k is not None:
            ev_dec[k][1].record(stream)

    if args.verify:
        import sbe_testlib as T
        for _ in range(nsets):
            b = sets[rot["i"] % nsets]
            step()
            torch.cuda.synchronize()
            eo, eoff, _ = T.oracle_encode(b["arena"].cpu().numpy(), b["L"].cpu().numpy().view(np.uint32),
                                          b["ts"].cpu().numpy().view(np.uint64))
            assert np.array_equal(b["out_off"].cpu().numpy().view(np.uint64), eoff)
            assert np.array_equal(b["out"][: int(eoff[-1])].cpu().numpy(), eo)
    # host-side setup before the warmup, so the GPU goes from the warmup steps straight into the
    # timed ones: creating the profiling events takes ~1 ms of host time, during which an idle GPU
    # lowers its clocks
    sbecodec.profile_enable(args.event_every)  # events on the pack / decode dispatches
    # settle: untimed round trips until the GPU has run the workload for settle_ms (its clocks ramp
    # up over the first tens of milliseconds of sustained load; a 5-step warmup is ~1 ms), then the
    # W warmup steps, then the timed K steps, with no host gap in between
    settle_steps, t_set = 0, time.perf_counter()
    while args.settle_ms > 0 and settle_steps < 10000:
        for _ in range(10):
            step()
        settle_steps += 10
        torch.cuda.synchronize()
        if (time.perf_counter() - t_set) * 1e3 >= args.settle_ms:
            break
    for _ in range(args.warmup):
        step()
    sbecodec.profile_enable(args.event_every)  # restart the rings: warmup launches are not sampled
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world)
    # the in-region samples (every event_every-th step), then the sampled pass: the same steps on
    # the same stream right after the timed region, HIP events on every pack / decode dispatch
    # (hipExtLaunchKernel timestamps of the kernel itself); its mean is the roofline's duration
    inreg_pack = sbecodec.profile_read(sbecodec.PROF_PACK) if args.event_every else []
    inreg_deck = sbecodec.profile_read(sbecodec.PROF_DECODE) if args.event_every else []
    sbecodec.profile_enable(1)
    for _ in range(args.sample_steps):
        step()
    torch.cuda.synchronize()
    pack_samples = sbecodec.profile_read(sbecodec.PROF_PACK)
    deck_samples = sbecodec.profile_read(sbecodec.PROF_DECODE)
    pack_ms = float(np.mean(pack_samples))
    deck_ms = float(np.mean(deck_samples))
    # the warm-cache figure (rounds 1-5's workload): the same number of steps on set 0 alone, so
    # each step re-reads what the previous one left in the MALL; reported beside, never the roofline
    rot["only"] = 0
    for _ in range(10):
        step()
    sbecodec.profile_enable(1)
    for _ in range(args.sample_steps):
        step()
    torch.cuda.synchronize()
    pack_warm = float(np.mean(sbecodec.profile_read(sbecodec.PROF_PACK)))
    deck_warm = float(np.mean(sbecodec.profile_read(sbecodec.PROF_DECODE)))
    rot["only"] = None
    sbecodec.profile_enable(0)

    # informational, untimed: whole-call encode (sums + pack) and decode times
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_enc]))
    dec_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_dec]))
    total = n * world * args.steps
    value = total / el

    c5 = None
    if not args.no_config5:
        sets.clear()
        torch.cuda.empty_cache()
        try:
            c5 = config5(args, world, rank, dev)
        except Exception as e:  # the headline line must still come out
            c5 = {"workload": "config5_fixed256_sharded", "error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        def gbs(b, ms):
            return n * b / (ms * 1e-3) / 1e9

        if pack_ms >= deck_ms:
            dom = dict(kernel="sbe_enc_pack<packed,wire>", bytes_per_record=ENC_BYTES, bytes_all=ENC_BYTES_ALL,
                       ms=pack_ms, samples=pack_samples, inreg=inreg_pack, warm=pack_warm)
        else:
            dom = dict(kernel="sbe_decode_kernel<parse_message>", bytes_per_record=DEC_BYTES,
                       bytes_all=DEC_BYTES_ALL, ms=deck_ms, samples=deck_samples, inreg=inreg_deck, warm=deck_warm)
        traffic = measured_traffic(dom["kernel"], n)
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            cpu = cpu_baseline(min(n, 200_000), args.cpu_seconds, args.cpu_threads or default_cpu_threads())
        ach = gbs(dom["bytes_per_record"], dom["ms"])
        line = {
            "metric": METRIC, "value": value, "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "roundtrip_fixed256_orders", "records_per_gpu": n, "record_bytes": 256,
                       "encode": "wire-correct TopicMessage, packed SoA input",
                       "decode": "parse_message descriptors (views) + sequence_number evaluation",
                       "parallelism": f"shard{world}", "settle": {"ms": args.settle_ms, "steps": settle_steps},
                       "input_sets": nsets,
                       "rotation": (f"step k encodes set k mod {nsets} and decodes that set's stream; every set has "
                                    f"its own inputs and outputs ({nsets} x ~{(n * (250 + 256 + 58 + 17)) / 1e9:.2f} GB)")},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "kernel": dom["kernel"],
                         "kernel_ms": dom["ms"], "bytes_per_record": dom["bytes_per_record"],
                         "bytes_source": "SURVEY §8(d) algorithmic bytes per 256-B record",
                         "achieved_incl_offsets": gbs(dom["bytes_all"], dom["ms"]),
                         "bytes_per_record_incl_offsets": dom["bytes_all"],
                         "timing": (f"HIP events on every dispatch of the kernel in {args.sample_steps} steps run right "
                                    f"after the timed region (same stream, inputs and clocks): {len(dom['samples'])} "
                                    f"samples; the timed region itself samples every {args.event_every}th step "
                                    f"(kernel_ms_in_region, {len(dom['inreg'])} samples), since a timed dispatch "
                                    f"costs the GPU ~5 us"),
                         "samples": len(dom["samples"]),
                         "kernel_ms_in_region": float(np.mean(dom["inreg"])) if dom["inreg"] else None,
                         "kernel_ms_min": float(np.min(dom["samples"])),
                         "kernel_ms_median": float(np.median(dom["samples"])),
                         "kernel_ms_max": float(np.max(dom["samples"])),
                         "cache": (f"inputs rotated over {nsets} sets (cache-cold for the MALL)" if nsets > 1 else
                                   "one input set re-read every step (warm: part of it is served by the MALL)"),
                         "kernel_ms_warm": dom["warm"], "achieved_warm": gbs(dom["bytes_per_record"], dom["warm"]),
                         "frac_warm": gbs(dom["bytes_per_record"], dom["warm"]) / HBM_PEAK_GBS},
            "kernels": {"encode_ms": enc_ms, "decode_ms": dec_ms, "pack_ms": pack_ms,
                        "pack_gbs": gbs(ENC_BYTES, pack_ms), "decode_kernel_ms": deck_ms,
                        "pack_ms_warm": pack_warm, "decode_kernel_ms_warm": deck_warm,
                        "decode_kernel_gbs": gbs(DEC_BYTES, deck_ms),
                        "roundtrip_gbs": n * (ENC_BYTES + DEC_BYTES) / ((enc_ms + dec_ms) * 1e-3) / 1e9},
            "cpu_baseline": cpu,
        }
        if c5 is not None:
            line["config5"] = c5
        print(json.dumps(line), flush=True)
    if dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()


def measured_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the committed PMC summary (profiles/traffic.json:
    FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM), scaled from the records per launch it
    was measured at; None when no summary covers the kernel."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        d = json.load(open(path))[kernel]
    except (OSError, KeyError, ValueError):
        return None
    return d["bytes_per_launch"] * n / d["records"]


if __name__ == "__main__":
    main()
