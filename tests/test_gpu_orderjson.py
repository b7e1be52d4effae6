"""Order JSON on the GPU (sbe_order_to_json_batch) against the oracle, byte-exact.

Order::to_json (src/order_types.cpp:122-181) and publish_order's headers JSON
(src/cluster_client.cpp:308-323).  The oracle is pinned as described in
tests/test_oracle_orderjson.py (jsoncpp itself absent: parity unpinned against it)."""
import numpy as np
import pytest

import sbe_testlib as T


def gpu_json(codec, fields, cid, ts, q, what, with_off=False, out_capacity=None):
    import torch
    arena, str_len = T.pack_order_fields(fields)
    str_off = None
    if with_off:  # the same strings, record order reversed in the arena
        n = len(fields)
        pieces, offs, at = [], np.zeros((n, 8), np.uint32), 0
        for i in reversed(range(n)):
            for j in range(8):
                offs[i, j] = at
                pieces.append(fields[i][j])
                at += len(fields[i][j])
        arena = np.frombuffer(b"".join(pieces), np.uint8) if at else np.zeros(1, np.uint8)
        str_off = torch.from_numpy(offs.astype(np.int32)).cuda()
    if arena.size == 0:
        arena = np.zeros(1, np.uint8)
    r = codec.order_to_json_batch(torch.from_numpy(arena.copy()).cuda(),
                                  torch.from_numpy(str_len.astype(np.int32)).cuda(),
                                  torch.from_numpy(np.asarray(cid, np.int64)).cuda(),
                                  torch.from_numpy(np.asarray(ts, np.int64)).cuda(),
                                  torch.from_numpy(np.asarray(q, np.float64)).cuda(), what,
                                  str_off=str_off, out_capacity=out_capacity)
    torch.cuda.synchronize()
    off = r.out_off.cpu().numpy().astype(np.uint64)
    return r.out.cpu().numpy(), off, r.status.cpu().numpy()[: len(fields)]


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,hard,what,with_off", [
    (1, 0, True, 0, False), (300, 1, True, 0, False), (300, 2, True, 1, False), (4099, 3, True, 0, True),
    (20000, 4, False, 0, False), (20000, 5, True, 1, True), (100000, 6, True, 0, False)])
def test_gpu_matches_oracle(codec, n, seed, hard, what, with_off):
    fields, cid, ts, q = T.order_batch(n, seed, hard)
    arena, str_len = T.pack_order_fields(fields)
    exp, exp_off = T.oracle_order_json(arena, str_len, cid, ts, q, what, nthreads=8)
    out, off, st = gpu_json(codec, fields, cid, ts, q, what, with_off)
    assert np.array_equal(off, exp_off)
    assert (st == 0).all()
    got = out[: int(off[-1])].tobytes()
    if got != exp:
        bad = next(i for i in range(n) if got[int(off[i]):int(off[i + 1])] != exp[int(off[i]):int(off[i + 1])])
        raise AssertionError(f"record {bad}: q={q[bad]!r}\n gpu {got[int(off[bad]):int(off[bad + 1])]!r}\n"
                             f" orc {exp[int(off[bad]):int(off[bad + 1])]!r}")


@pytest.mark.gpu
def test_gpu_every_edge_double(codec):
    vals = list(T.EDGE_DOUBLES)
    rng = np.random.default_rng(99)
    vals += list(rng.integers(0, 2 ** 64, 20000, dtype=np.uint64).view(np.float64))
    for e in range(-1075, 1024, 7):  # one value per binade region, with neighbours
        x = np.ldexp(1.0, e) if e > -1075 else 5e-324
        vals += [x, np.nextafter(x, 0), np.nextafter(x, np.inf), -x * 1.5]
    n = len(vals)
    fields = [[b"u", b"i", b"B", b"Q", b"S", b"o", b"m", b"CREATED"]] * n
    cid = np.zeros(n, np.int64)
    ts = np.zeros(n, np.int64)
    q = np.array(vals, np.float64)
    arena, str_len = T.pack_order_fields(fields)
    exp, exp_off = T.oracle_order_json(arena, str_len, cid, ts, q, 0, nthreads=8)
    out, off, _ = gpu_json(codec, fields, cid, ts, q, 0)
    assert np.array_equal(off, exp_off)
    got = out[: int(off[-1])].tobytes()
    for i in range(n):
        a, b = int(off[i]), int(off[i + 1])
        assert got[a:b] == exp[a:b], (q[i], got[a:b][-200:], exp[a:b][-200:])


@pytest.mark.gpu
def test_gpu_overflow_and_empty(codec):
    import torch
    fields, cid, ts, q = T.order_batch(100, 8)
    arena, str_len = T.pack_order_fields(fields)
    exp, exp_off = T.oracle_order_json(arena, str_len, cid, ts, q, 0)
    cap = int(exp_off[60]) + 5
    out, off, st = gpu_json(codec, fields, cid, ts, q, 0, out_capacity=cap)
    assert np.array_equal(off, exp_off)
    fits = exp_off[1:] <= cap
    assert (st[fits] == 0).all() and (st[~fits] == 6).all()
    assert out[:int(exp_off[60])].tobytes() == exp[:int(exp_off[60])]
    r = codec.order_to_json_batch(torch.zeros(1, dtype=torch.uint8, device="cuda"),
                                  torch.zeros(0, dtype=torch.int32, device="cuda"),
                                  torch.zeros(0, dtype=torch.int64, device="cuda"),
                                  torch.zeros(0, dtype=torch.int64, device="cuda"),
                                  torch.zeros(0, dtype=torch.float64, device="cuda"))
    torch.cuda.synchronize()
    assert int(r.out_off[0]) == 0


@pytest.mark.gpu
def test_gpu_publish_order_pipeline(codec):
    """Orders → payload + headers JSON on the device → TopicMessage encode → parse_message decode:
    the decoded payload / headers views are the oracle's JSON texts."""
    import torch
    n = 2000
    fields, cid, ts, q = T.order_batch(n, 21, hard=False)
    arena, str_len = T.pack_order_fields(fields)
    pay, pay_off = T.oracle_order_json(arena, str_len, cid, ts, q, 0)
    hdr, hdr_off = T.oracle_order_json(arena, str_len, cid, ts, q, 1)
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).cuda()
    args = (dev(arena, np.uint8), dev(str_len, np.int32), dev(cid, np.int64), dev(ts, np.int64), dev(q, np.float64))
    P = codec.order_to_json_batch(*args, what=0)
    H = codec.order_to_json_batch(*args, what=1)
    # TopicMessage fields topic, messageType, uuid, payload, headers with str_off into three arenas
    topic, mtype = b"orders", b"CREATE_ORDER"
    lit = torch.from_numpy(np.frombuffer(topic + mtype, np.uint8).copy()).cuda()
    ids = torch.from_numpy(np.frombuffer(b"".join(f[6] for f in fields) or b"\0", np.uint8).copy()).cuda()
    id_len = torch.tensor([len(f[6]) for f in fields], dtype=torch.int64)
    id_off = torch.cumsum(id_len, 0) - id_len
    big = torch.cat([lit, ids, P.out[: int(P.out_off[-1])], H.out[: int(H.out_off[-1])]])
    b_ids, b_pay = lit.numel(), lit.numel() + ids.numel()
    b_hdr = b_pay + int(P.out_off[-1])
    off = torch.zeros(n, 5, dtype=torch.int64)
    ln = torch.zeros(n, 5, dtype=torch.int64)
    off[:, 0], ln[:, 0] = 0, len(topic)
    off[:, 1], ln[:, 1] = len(topic), len(mtype)
    off[:, 2], ln[:, 2] = b_ids + id_off, id_len
    po, ho = P.out_off.cpu(), H.out_off.cpu()
    off[:, 3], ln[:, 3] = b_pay + po[:-1], po[1:] - po[:-1]
    off[:, 4], ln[:, 4] = b_hdr + ho[:-1], ho[1:] - ho[:-1]
    enc = codec.encode_topic_batch(big, ln.to(torch.int32).cuda(), torch.full((n,), 7, dtype=torch.int64).cuda(),
                                   str_off=off.to(torch.int32).cuda())
    dec = codec.decode_batch(enc.out, enc.out_off, codec.DEC_PARSE_MESSAGE)
    torch.cuda.synchronize()
    d = dec.numpy()
    data = enc.out.cpu().numpy()
    ro = enc.out_off.cpu().numpy()
    for i in range(0, n, 13):
        rec = data[int(ro[i]):int(ro[i + 1])].tobytes()
        vo, vl = d["view_off"][i], d["view_len"][i]
        assert d["status"][i] == codec.ST_TM
        assert rec[vo[3]:vo[3] + vl[3]] == pay[int(pay_off[i]):int(pay_off[i + 1])]
        assert rec[vo[4]:vo[4] + vl[4]] == hdr[int(hdr_off[i]):int(hdr_off[i + 1])]


@pytest.mark.gpu
def test_gpu_side_stream_regrow(codec):
    """A self-sized call on a side stream that is not torch's current stream: the regrow read of
    out_off[n] waits for that stream: sizes, statuses and texts are the oracle's."""
    import torch
    n = 2000
    fields, cid, ts, q = T.order_batch(n, 11, True)
    # long strings of control bytes (each escapes to 6 bytes): the kernels run for a while
    fields = [tuple((b"\x01" * 700) if j == 0 else f for j, f in enumerate(rec)) for rec in fields]
    arena, str_len = T.pack_order_fields(fields)
    exp, exp_off = T.oracle_order_json(arena, str_len, cid, ts, q, 0, nthreads=8)
    side = torch.cuda.Stream()
    dev_in = [torch.from_numpy(arena.copy()).cuda(), torch.from_numpy(str_len.astype(np.int32)).cuda(),
              torch.from_numpy(np.asarray(cid, np.int64)).cuda(), torch.from_numpy(np.asarray(ts, np.int64)).cuda(),
              torch.from_numpy(np.asarray(q, np.float64)).cuda()]
    torch.cuda.synchronize()
    r = codec.order_to_json_batch(*dev_in, 0, stream=side)
    side.synchronize()
    off = r.out_off.cpu().numpy().astype(np.uint64)
    assert np.array_equal(off, exp_off)
    assert (r.status.cpu().numpy()[:n] == 0).all()
    assert r.out[: int(off[-1])].cpu().numpy().tobytes() == exp


@pytest.mark.gpu
@pytest.mark.parametrize("what", [0, 1])
def test_gpu_window_edges(codec, what):
    """Texts of every size class in one batch: most fit a tile's LDS window, some only a window of
    their own (several passes), some exceed any window (written straight to HBM); with a capacity
    that cuts the batch in the middle of a large text."""
    n = 700
    fields, cid, ts, q = T.order_batch(n, 31, True)
    big = {0: b"\x01" * 3500, 6: b"\x01" * 3500}  # payload prints field 0 twice; headers print field 6
    fields = [tuple((big[j] * (1 + (i % 3))) if (i % 37 == 5 and j in big) else
                    ((b"\x02" * 600) if (i % 11 == 3 and j in big) else f) for j, f in enumerate(rec))
              for i, rec in enumerate(fields)]
    arena, str_len = T.pack_order_fields(fields)
    exp, exp_off = T.oracle_order_json(arena, str_len, cid, ts, q, what, nthreads=8)
    sizes = np.diff(exp_off.astype(np.int64))
    assert sizes.max() > 20000 and (sizes > 3000).sum() > 20  # both size classes are present
    for cap in (None, int(exp_off[400]) - 7):
        out, off, st = gpu_json(codec, fields, cid, ts, q, what, out_capacity=cap)
        assert np.array_equal(off, exp_off)
        limit = int(off[-1]) if cap is None else cap
        fits = exp_off[1:] <= limit
        assert (st[fits] == 0).all() and (st[~fits] == 6).all()
        for i in np.nonzero(fits)[0]:
            a, b = int(off[i]), int(off[i + 1])
            assert out[a:b].tobytes() == exp[a:b], i


@pytest.mark.gpu
@pytest.mark.parametrize("what", [0, 1])
def test_gpu_arena_at_allocation_end(codec, what):
    """the sizing launch stages each wave's string range with 16-byte loads; the range's
    last partial chunk is read bytewise, so nothing past the last string byte is read.  The packed
    arena here ends exactly at the end of a 2 MiB allocation, at an address that is not 16-byte
    aligned; the texts must equal the oracle's."""
    import torch
    fields, cid, ts, q = T.order_batch(3000, 77, True)
    arena, str_len = T.pack_order_fields(fields)
    if arena.size % 16 == 0:  # keep the end unaligned
        fields[0] = [fields[0][0] + b"x"] + list(fields[0][1:])
        arena, str_len = T.pack_order_fields(fields)
    exp, exp_off = T.oracle_order_json(arena, str_len, cid, ts, q, what, nthreads=8)
    buf = torch.zeros(1 << 21, dtype=torch.uint8, device="cuda")
    assert arena.size < buf.numel()
    a = buf[buf.numel() - arena.size:]
    a.copy_(torch.from_numpy(arena))
    r = codec.order_to_json_batch(a, torch.from_numpy(str_len.astype(np.int32)).cuda(),
                                  torch.from_numpy(np.asarray(cid, np.int64)).cuda(),
                                  torch.from_numpy(np.asarray(ts, np.int64)).cuda(),
                                  torch.from_numpy(np.asarray(q, np.float64)).cuda(), what)
    torch.cuda.synchronize()
    off = r.out_off.cpu().numpy().astype(np.uint64)
    assert np.array_equal(off, exp_off)
    assert r.out.cpu().numpy()[: int(off[-1])].tobytes() == exp
