"""MATERIALIZE (sbe_materialize_views, include/sbecodec.h) on the GPU against the oracle: after a
decode, every record's five views copied into one arena, so the strings outlive the input as the
reference's ParseResult strings do (include/aeron_cluster/sbe_messages.hpp:306-328).  Bit-exact
bytes and offsets vs the views of the oracle's own decode (tests/sbe_testlib.py oracle_materialize),
in every decode mode, on mixed, fixed-256, variable-length (views up to 65534 B), session-framed,
Lite and edge records, with short capacities (nothing
past the capacity is written) and an empty batch."""
import numpy as np
import pytest

import sbe_testlib as T


def run(codec, data, off, mode, cap=None, pad=0):
    import torch
    d = torch.from_numpy(data if data.size else np.zeros(16, np.uint8)).cuda()
    o = torch.from_numpy(np.asarray(off, np.uint64).view(np.int64)).cuda()
    dec = codec.decode_batch(d, o, mode=mode, in_bytes=int(off[-1] - off[0]))
    arena = None
    if cap is not None:
        arena = torch.full((cap + pad,), 0xA5, dtype=torch.uint8, device="cuda")
    m = codec.materialize_views(d, o, dec, arena=arena, arena_capacity=cap)
    torch.cuda.synchronize()
    return m.arena.cpu().numpy(), m.arena_off.cpu().numpy().view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("work", ["mixed", "fixed", "edges"])
def test_gpu_materialize_matches_oracle(codec, mode, work):
    if work == "mixed":
        data, off = T.mixed_records(60000, seed=0x5EED0A11)
    elif work == "fixed":
        arena, L, ts = T.fixed256_orders(30000)
        data, off, _ = T.oracle_encode(arena, L, ts)
    else:  # every reference branch's edge record, 40 times over at shifting offsets
        recs = [r for _, r in T.edge_records()] * 40
        off = np.zeros(len(recs) + 1, np.uint64)
        off[1:] = np.cumsum([len(r) for r in recs])
        data = np.frombuffer(b"".join(recs), np.uint8).copy()
    dec = T.oracle_decode(data, off, mode)
    exp, exp_off = T.oracle_materialize(data, off, dec)
    got, got_off = run(codec, data, off, mode)
    assert np.array_equal(got_off, exp_off)
    assert got[: exp.size].tobytes() == exp.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("work", ["var_long", "session"])
def test_gpu_materialize_long_views_and_frames(codec, work):
    """Views of every length up to 65534 B (a thread copies its record's views in 16-byte steps; the
    last step of a view may run into the next view of the same record, never past the record's
    arena range) and session frames (views into the schema-111-wrapped record)."""
    if work == "var_long":
        arena, L, ts = T.var_orders(6000, seed=77)
        L = L.copy()
        rng = np.random.default_rng(5)
        idx = rng.choice(len(L), 40, replace=False)
        L[idx, 3] = rng.integers(1, 65535, idx.size)
        L[idx[:5], 4] = 65534
        L[idx[5:10]] = 0
        arena = rng.integers(32, 127, int(L.sum(dtype=np.int64)), dtype=np.uint8)
        data, off, _ = T.oracle_encode(arena, L, ts)
    else:
        arena, L, ts = T.var_orders(8000, seed=78)
        data, off, _ = T.oracle_encode_session(arena, L, ts, 7, -3, None, T.ENC_REF_TRUNCATE8, 0)
    for mode in (0, 1):
        dec = T.oracle_decode(data, off, mode)
        exp, exp_off = T.oracle_materialize(data, off, dec)
        got, got_off = run(codec, data, off, mode)
        assert np.array_equal(got_off, exp_off)
        assert got[: exp.size].tobytes() == exp.tobytes()


@pytest.mark.gpu
def test_gpu_materialize_lite(codec):
    arena, L, tid, seq = T.lite_records(40000, 201)
    data, off, _ = T.oracle_encode_lite(201, arena, L, tid, seq)
    dec = T.oracle_decode(data, off, T.DEC_LITE)
    exp, exp_off = T.oracle_materialize(data, off, dec)
    got, got_off = run(codec, data, off, T.DEC_LITE)
    assert np.array_equal(got_off, exp_off)
    assert got[: exp.size].tobytes() == exp.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("frac", [0.0, 0.37, 0.999])
def test_gpu_materialize_short_capacity(codec, frac):
    """A view that would end past the capacity is not written, nor is any byte past it; the
    offsets still describe the full layout; every view that fits is exact."""
    data, off = T.mixed_records(5000, seed=0x5EED0A12)
    dec = T.oracle_decode(data, off, 0)
    exp, exp_off = T.oracle_materialize(data, off, dec)
    cap = int(frac * exp.size)
    got, got_off = run(codec, data, off, 0, cap=cap, pad=4096)
    assert np.array_equal(got_off, exp_off)
    assert (got[cap:] == 0xA5).all()
    ends = exp_off[1:].astype(np.int64)
    starts = exp_off[:-1].astype(np.int64)
    fit = ends <= cap
    for s, e in zip(starts[fit][-200:], ends[fit][-200:]):  # the last views that fit, and all bytes below
        assert got[s:e].tobytes() == exp[s:e].tobytes()
    full = int(ends[fit].max()) if fit.any() else 0
    k = np.nonzero(~fit)[0]
    lim = int(starts[k[0]]) if k.size else full
    assert got[:lim].tobytes() == exp[:lim].tobytes()


@pytest.mark.gpu
def test_gpu_materialize_empty(codec):
    import torch
    d = torch.zeros(16, dtype=torch.uint8, device="cuda")
    o = torch.zeros(1, dtype=torch.int64, device="cuda")
    dec = codec.alloc_decoded(0, d.device)
    m = codec.materialize_views(d, o, dec)
    torch.cuda.synchronize()
    assert int(m.arena_off[0]) == 0 and m.arena_off.numel() == 1
