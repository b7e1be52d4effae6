"""GPU: BASELINE.json configs[4] / SURVEY §8(e) on one GPU — the 134,217,728-record fixed-256
batch encoded whole and as the 8 shard_range shards an 8-GPU node would encode; the shards'
streams concatenate (what the gather assembles) to exactly the single-batch stream, and sampled
records match the oracle.  Plus sbe_gather_encoded on a one-rank RCCL communicator."""
import os

import numpy as np
import pytest
import torch

import sbe_testlib as T
import shard

pytestmark = pytest.mark.gpu


def _encode(codec, arena, L, ts, out, out_off, status, ws):
    codec.encode_topic_batch(arena, L, ts, out=out, out_off=out_off, status=status, workspace=ws)


def test_config5_sharded_encode_equals_single_batch(codec):
    N, W = T.CONFIG5_RECORDS, 8
    dev = torch.device("cuda")
    arena, L, ts = T.config5_shard(0, N, dev)
    out = torch.empty(codec.output_bound(N, int(arena.numel())), dtype=torch.uint8, device=dev)
    out_off = torch.empty(N + 1, dtype=torch.int64, device=dev)
    status = torch.empty(N, dtype=torch.uint8, device=dev)
    ws = codec.alloc_workspace(N, dev)
    _encode(codec, arena, L, ts, out, out_off, status, ws)
    torch.cuda.synchronize()
    assert int(out_off[N].item()) == 256 * N and int(status.max().item()) == 0
    assert torch.equal(out_off, torch.arange(N + 1, dtype=torch.int64, device=dev) * 256)

    # the 8 shards, each generated on its own (global indices) and encoded on its own
    m_max = -(-N // W)
    s_out = torch.empty(codec.output_bound(m_max, 222 * m_max), dtype=torch.uint8, device=dev)
    s_off = torch.empty(m_max + 1, dtype=torch.int64, device=dev)
    s_st = torch.empty(m_max, dtype=torch.uint8, device=dev)
    s_ws = codec.alloc_workspace(m_max, dev)
    for r in range(W):
        lo, hi = shard.shard_range(N, W, r)
        m = hi - lo
        sa, sL, sts = T.config5_shard(lo, hi, dev)
        assert torch.equal(sa, arena[222 * lo: 222 * hi]) and torch.equal(sts, ts[lo:hi])
        _encode(codec, sa, sL, sts, s_out, s_off[: m + 1], s_st[:m], s_ws)
        base = 256 * lo
        assert torch.equal(s_off[: m + 1] + base, out_off[lo: hi + 1]), f"shard {r} offsets"
        assert torch.equal(s_out[: 256 * m], out[base: base + 256 * m]), f"shard {r} bytes"
        del sa, sL, sts
    del s_out, s_off, s_st, s_ws

    # sampled records against the oracle (their inputs copied back)
    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([rng.integers(0, N, 3000), [0, N - 1], [N // W * r for r in range(W)]]))
    it = torch.from_numpy(idx.astype(np.int64)).to(dev)
    rec_in = arena.view(N, 222)[it].cpu().numpy()
    rec_ts = ts[it].cpu().numpy().view(np.uint64)
    got = out.view(-1)[: 256 * N].view(N, 256)[it].cpu().numpy()
    eo, eoff, est = T.oracle_encode(rec_in.reshape(-1), np.tile(np.array([6, 12, 29, 143, 32], np.uint32),
                                                              (len(idx), 1)), rec_ts)
    assert np.array_equal(eoff, np.arange(len(idx) + 1, dtype=np.uint64) * 256)
    assert np.array_equal(got.reshape(-1), eo)


def test_gather_one_rank_communicator(codec):
    """sbe_gather_encoded on a world-1 RCCL communicator: the root's own shard is copied and its
    offsets rebased (the path every root takes for its own shard)."""
    dev = torch.device("cuda")
    comm = codec.Comm(1, 0, codec.comm_unique_id())
    try:
        arena, L, ts = T.var_orders(5000, seed=17)
        a = torch.from_numpy(arena).to(dev)
        Ld = torch.from_numpy(L.view(np.int32)).to(dev)
        t = torch.from_numpy(ts.view(np.int64)).to(dev)
        enc = codec.encode_topic_batch(a, Ld, t)
        n = 5000
        total = int(enc.out_off[n].item())
        dst = torch.zeros(total + 64, dtype=torch.uint8, device=dev)
        dst_off = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
        s, o, nbytes, nrec = codec.gather_encoded(comm, enc.out, enc.out_off, n, root=0, dst=dst, dst_off=dst_off)
        torch.cuda.synchronize()
        assert nbytes == total and nrec == n
        assert torch.equal(s, enc.out[:total]) and torch.equal(o, enc.out_off)
        small = torch.empty(total - 1, dtype=torch.uint8, device=dev)
        with pytest.raises(codec.SbeError, match="ENOSPC"):
            codec.gather_encoded(comm, enc.out, enc.out_off, n, root=0, dst=small, dst_off=dst_off)
        # an offsets array one entry short is refused before any write
        short_off = torch.full((n,), -1, dtype=torch.int64, device=dev)
        with pytest.raises(codec.SbeError, match="ENOSPC"):
            codec.gather_encoded(comm, enc.out, enc.out_off, n, root=0, dst=dst, dst_off=short_off)
        torch.cuda.synchronize()
        assert int((short_off != -1).sum().item()) == 0
        with pytest.raises(codec.SbeError, match="n \\+ 1"):
            codec.gather_encoded(comm, enc.out, enc.out_off[:n], n, root=0, dst=dst, dst_off=dst_off)
    finally:
        comm.close()


def test_bench_gather_verifier_catches_a_bad_byte(codec):
    """bench.py's config-5 gather check (verify_gathered) on a one-GPU stand-in for the root's
    gathered stream: clean → no mismatch; one flipped byte or one wrong offset → that chunk."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    dev = torch.device("cuda")
    N = 3_000_000
    arena, L, ts = T.config5_shard(0, N, dev)
    enc = codec.encode_topic_batch(arena, L, ts)
    ws = codec.alloc_workspace(1 << 20, dev)
    dst, dst_off = enc.out, enc.out_off
    assert bench.verify_gathered(dst, dst_off, N, dev, ws, chunk=1 << 20)["mismatched_chunks"] == 0
    dst[256 * 2_500_000 + 77] ^= 1
    assert bench.verify_gathered(dst, dst_off, N, dev, ws, chunk=1 << 20)["mismatched_chunks"] == 1
    dst[256 * 2_500_000 + 77] ^= 1
    dst_off[5] += 1
    assert bench.verify_gathered(dst, dst_off, N, dev, ws, chunk=1 << 20)["mismatched_chunks"] == 1
