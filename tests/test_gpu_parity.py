"""GPU parity: the HIP codec (through the C ABI) against the oracle, bit-exact.

Sizes keep the oracle to seconds; full-size configurations are checked through size-independent
properties (round trip, offsets monotone, byte checksums) in test_gpu_scale.py.
"""
import numpy as np
import pytest
import torch

import sbe_testlib as T

pytestmark = pytest.mark.gpu


def to_dev(a, dtype):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view({torch.uint8: np.uint8, torch.int32: np.int32, torch.int64: np.int64}[dtype])
                            ).to("cuda")


def gpu_encode(codec, arena, str_len, ts, str_off=None, flags=0, ts_default=0):
    a = to_dev(arena if arena.size else np.zeros(16, np.uint8), torch.uint8)
    L = to_dev(np.asarray(str_len, np.uint32).reshape(-1, 5), torch.int32)
    t = to_dev(np.asarray(ts, np.uint64), torch.int64)
    o = None if str_off is None else to_dev(np.asarray(str_off, np.uint32).reshape(-1, 5), torch.int32)
    enc = codec.encode_topic_batch(a, L, t, str_off=o, flags=flags, ts_default=ts_default)
    torch.cuda.synchronize()
    off = enc.out_off.cpu().numpy().view(np.uint64)
    n = ts.size
    out = enc.out[: int(off[n])].cpu().numpy()
    return out, off, enc.status.cpu().numpy()


# the decode kernel shapes (LDS windows of a 64-record tile, chosen by sbe_decode_batch_sized from
# the average record size in_bytes / n): 16 KiB (in_bytes 0: unknown), 13 KiB (over 320 B), 20 KiB
# (257..320 B), 15 KiB (113..204 B), 8 KiB (up to 112 B).  Values: in_bytes for a batch of n records.
SHAPES = {"w16k": lambda n: 0, "w13k": lambda n: 1 << 62, "w20k": lambda n: 300 * n, "w15k": lambda n: 150 * n,
          "w8k": lambda n: 1}


@pytest.fixture(params=list(SHAPES))
def shape(request):
    return SHAPES[request.param]


def gpu_decode(codec, data, rec_off, mode, in_bytes=0):
    if callable(in_bytes):  # a SHAPES entry
        in_bytes = in_bytes(len(rec_off) - 1)
    d = to_dev(data if data.size else np.zeros(16, np.uint8), torch.uint8)
    r = to_dev(np.asarray(rec_off, np.uint64), torch.int64)
    dec = codec.decode_batch(d, r, mode=mode, in_bytes=in_bytes)
    torch.cuda.synchronize()
    return dec.numpy()


def assert_same_decode(got, exp):
    for k in exp:
        g, e = got[k], exp[k]
        if not np.array_equal(g, e):
            bad = np.nonzero((g != e).reshape(len(e), -1).any(1))[0]
            raise AssertionError(f"{k} differs at records {bad[:10]}: got {g[bad[:3]]} expected {e[bad[:3]]}")


def check_encode(codec, arena, str_len, ts, str_off=None, flags=0, ts_default=0):
    go, goff, gst = gpu_encode(codec, arena, str_len, ts, str_off, flags, ts_default)
    eo, eoff, est = T.oracle_encode(arena, str_len, ts, str_off, flags, ts_default)
    np.testing.assert_array_equal(goff, eoff)
    np.testing.assert_array_equal(gst, est)
    if not np.array_equal(go, eo):
        i = int(np.nonzero(go != eo)[0][0])
        rec = int(np.searchsorted(eoff, i, side="right") - 1)
        raise AssertionError(f"output byte {i} (record {rec}) differs: {go[i]} != {eo[i]}")
    return go, goff


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 64 * 37 + 5])
def test_encode_fixed256(codec, n, flags):
    arena, L, ts = T.fixed256_orders(n)
    check_encode(codec, arena, L, ts, flags=flags)


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
def test_encode_var(codec, flags):
    arena, L, ts = T.var_orders(20000)
    check_encode(codec, arena, L, ts, flags=flags)


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
@pytest.mark.parametrize("pattern", ["one_big", "alternating", "random"])
def test_encode_unequal_records(codec, flags, pattern):
    """Windows whose records differ wildly in length (the rebalanced record-lane bulk pass: a
    record served by up to 63 lanes, lanes spanning 1-chunk records, records of 1..7000 B)."""
    rng = np.random.default_rng({"one_big": 11, "alternating": 12, "random": 13}[pattern])
    n = 3000
    if pattern == "one_big":      # one ~7 KB record per 32-record tile, the rest tiny
        big = (np.arange(n) % 32) == rng.integers(0, 32)
    elif pattern == "alternating":
        big = (np.arange(n) % 2) == 0
    else:
        big = rng.random(n) < 0.1
    L = np.zeros((n, 5), np.uint32)
    L[:, :3] = rng.integers(0, 4, (n, 3))
    L[:, 3] = np.where(big, rng.integers(2000, 7000, n), rng.integers(0, 20, n))
    L[:, 4] = rng.integers(0, 3, n)
    if pattern == "alternating":
        L[:, 3] = np.where(big, rng.integers(200, 900, n), L[:, 3])
    arena = rng.integers(32, 127, int(L.sum()), dtype=np.uint8)
    ts = rng.integers(1, 1 << 62, n, dtype=np.uint64)
    check_encode(codec, arena, L, ts, flags=flags)


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
def test_encode_gather_mode(codec, flags):
    # explicit per-field offsets into a shuffled arena, ragged alignment
    arena, L, ts = T.var_orders(5000, seed=99)
    n = ts.size
    starts = np.zeros(n * 5 + 1, np.int64)
    starts[1:] = np.cumsum(L.reshape(-1).astype(np.int64))
    perm = np.random.default_rng(3).permutation(n * 5)
    pieces = [arena[starts[k]: starts[k + 1]] for k in range(n * 5)]
    new = np.zeros(len(arena) + 3 * n * 5 + 7, np.uint8)
    off = np.zeros(n * 5, np.uint32)
    at = 7
    for k in perm:
        off[k] = at
        new[at: at + len(pieces[k])] = pieces[k]
        at += len(pieces[k]) + (k % 3)
    check_encode(codec, new, L, ts, str_off=off, flags=flags)


def test_encode_edges(codec):
    rng = np.random.default_rng(7)
    lens = [[0, 0, 0, 0, 0], [1, 0, 0, 0, 0], [0, 0, 0, 0, 1], [6, 12, 29, 0, 0],
            [65534, 0, 1, 2, 3], [65535, 0, 0, 0, 0], [0, 65535, 0, 0, 0], [0, 0, 65535, 0, 0],
            [0, 0, 0, 65535, 0], [0, 0, 0, 0, 65535], [70000, 70000, 0, 0, 1],
            [3, 3, 3, 65534, 65534], [65534] * 5, [5, 6, 7, 8, 9]]
    for _ in range(200):
        lens.append(list(rng.integers(0, 40, 5)))
    L = np.array(lens, np.uint32)
    n = len(L)
    arena = rng.integers(0, 256, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    ts = rng.integers(0, 2**63, n, dtype=np.uint64)
    ts[::7] = 0  # 0 → ts_default (the reference substitutes its clock, src/sbe_encoder.cpp:134-138)
    for flags in (0, T.ENC_REF_TRUNCATE8):
        check_encode(codec, arena, L, ts, flags=flags, ts_default=1_760_000_000_123)


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
@pytest.mark.parametrize("pattern", ["sprinkled", "zero_run", "long_run"])
def test_encode_virtual_tiles_with_edges(codec, pattern, flags):
    """The virtual-tile pack loop (chosen per launch from the first superblock's average tile, see
    vt_pays in sbe_codec.hip) over E109 records, tiles with no output and records spanning windows."""
    arena, L, ts = T.vt_mixed(3 * 4096 + 123, pattern)
    check_encode(codec, arena, L, ts, flags=flags, ts_default=1_760_000_000_456)


def field_length_records():
    """Every field length 0..80 in every field position, the other fields (7L + 13k) mod 81: 405
    records whose tiles mix empty, 1..3-byte and ~80-byte strings (the C++ host test builds the same
    records, tests/cpp/test_host_api.cpp)."""
    recs, ts = [], []
    for f in range(5):
        for n in range(81):
            r = []
            for k in range(5):
                m = n if k == f else (n * 7 + k * 13) % 81
                r.append(bytes(ord("A") + (j * 31 + k * 7 + n) % 58 for j in range(m)))
            recs.append(r)
            ts.append(1_700_000_000_000_000_000 + 1_000_003 * n + f)
    arena = np.frombuffer(b"".join(b"".join(r) for r in recs), np.uint8).copy()
    L = np.array([[len(s) for s in r] for r in recs], np.uint32)
    return arena, L, np.array(ts, np.uint64)


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
def test_encode_field_lengths(codec, flags):
    arena, L, ts = field_length_records()
    check_encode(codec, arena, L, ts, flags=flags)


def _publish_lens(rng, n_small):
    """Lengths of ClusterClient::publish_topic records: the u16 wrap edges on every field, mixed
    into ordinary records so tiles hold both wrapped and plain records."""
    lens = []
    for L in (65534, 65535, 65536, 65537, 70000, 131072, 131073):
        for k in range(5):
            f = [6, 12, 23, int(rng.integers(0, 300)), 2]
            f[k] = L
            lens.append(f)
    for _ in range(n_small):
        lens.append([int(rng.integers(0, 30)), 12, 23, int(rng.integers(0, 500)), int(rng.integers(2, 40))])
    rng.shuffle(lens)
    return np.array(lens, np.uint32)


@pytest.mark.parametrize("gather", [False, True])
def test_encode_publish_topic(codec, gather):
    """SBE_ENC_PUBLISH_TOPIC (src/cluster_client.cpp:1850-1857, TopicMessage.h:515-529): lengths mod
    65536, no E109, wire length; packed and gather input."""
    rng = np.random.default_rng(11)
    L = _publish_lens(rng, 600)
    n = len(L)
    arena = rng.integers(0, 256, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    ts = rng.integers(1, 2**63, n, dtype=np.uint64)
    if not gather:
        check_encode(codec, arena, L, ts, flags=T.ENC_PUBLISH_TOPIC)
        return
    starts = np.zeros(n * 5 + 1, np.int64)
    starts[1:] = np.cumsum(L.reshape(-1).astype(np.int64))
    perm = rng.permutation(n * 5)
    new = np.zeros(len(arena) + 3 * n * 5 + 5, np.uint8)
    off = np.zeros(n * 5, np.uint32)
    at = 5
    for k in perm:
        off[k] = at
        new[at: at + starts[k + 1] - starts[k]] = arena[starts[k]: starts[k + 1]]
        at += int(starts[k + 1] - starts[k]) + int(k % 3)
    check_encode(codec, new, L, ts, str_off=off, flags=T.ENC_PUBLISH_TOPIC)


def test_encode_publish_topic_plain_records(codec):
    """Publish mode on records below 65536 B per field is the wire encoding (config-2 records)."""
    arena, L, ts = T.fixed256_orders(64 * 37 + 5)
    go, goff = check_encode(codec, arena, L, ts, flags=T.ENC_PUBLISH_TOPIC)
    wo, woff, _ = T.oracle_encode(arena, L, ts)
    assert np.array_equal(go, wo) and np.array_equal(goff, woff)


def test_encode_publish_flag_rules(codec):
    arena, L, ts = T.fixed256_orders(4)
    a, Ld, t = to_dev(arena, torch.uint8), to_dev(L, torch.int32), to_dev(ts, torch.int64)
    with pytest.raises(codec.SbeError):
        codec.encode_topic_batch(a, Ld, t, flags=T.ENC_PUBLISH_TOPIC | T.ENC_REF_TRUNCATE8)
    with pytest.raises(codec.SbeError):
        codec.encode_session_batch(a, Ld, t, 1, 2, flags=T.ENC_PUBLISH_TOPIC)


def test_encode_empty_batch(codec):
    out, off, st = gpu_encode(codec, np.zeros(0, np.uint8), np.zeros((0, 5), np.uint32), np.zeros(0, np.uint64))
    assert off.tolist() == [0] and out.size == 0


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
def test_decode_edges(codec, shape, mode):
    recs = [r for _, r in T.edge_records()]
    data, off = T.pack_records(recs)
    assert_same_decode(gpu_decode(codec, data, off, mode, in_bytes=shape), T.oracle_decode(data, off, mode))


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
def test_decode_edges_every_alignment(codec, shape, mode):
    # the same records behind 0..15 bytes of lead-in, so each one starts at every offset mod 16
    recs = [r for _, r in T.edge_records()]
    for lead in range(16):
        allr = [b"\0" * lead] + recs
        data, off = T.pack_records(allr)
        assert_same_decode(gpu_decode(codec, data, off, mode, in_bytes=shape), T.oracle_decode(data, off, mode))


def seq_key_records():
    """"_sequence_number" (and near misses) at every payload position and alignment, 'q'-dense
    filler, the key split across the payload/headers boundary and inside other fields."""
    key = b"_sequence_number"
    misses = [key[:-1] + b"X", b"X" + key[1:], key[:8] + b"Q" + key[9:], b"qqqq_seqqsequ"]
    rng = np.random.default_rng(3)
    recs = []
    for plen in (16, 17, 18, 19, 20, 31, 33, 47, 64, 95):
        for pos in range(0, plen - len(key) + 1):
            for fill in (b"a", b"q", b"e"):
                pay = bytearray(fill * plen)
                pay[pos:pos + len(key)] = key
                recs.append(T.tm_wire([b"t" * (pos % 5), b"ty", b"u" * (plen % 7), bytes(pay), b"{}"], pos))
    for m in misses:
        for pos in range(0, 24):
            pay = b"q" * pos + m + b"u" * (pos % 3)
            recs.append(T.tm_wire([b"tp", b"", b"id", pay, b"h"], pos))
    for cut in range(1, len(key)):  # key split between payload and headers: not in the payload
        recs.append(T.tm_wire([b"t", b"y", b"u", b"xx" + key[:cut], key[cut:] + b"yy"], cut))
        recs.append(T.tm_wire([key, b"y", key, b"p" * cut, key], cut))
    for k in range(300):  # random 'q'/'_'-rich payloads
        n = int(rng.integers(0, 200))
        pay = rng.choice(np.frombuffer(b"q_sequnbr", np.uint8), n).tobytes()
        if k % 3 == 0 and n >= 16:
            at = int(rng.integers(0, n - 15))
            pay = pay[:at] + key + pay[at + 16:]
        recs.append(T.tm_wire([b"topic", b"TYPE", b"id", pay, b"{}"], k))
    return recs


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
def test_decode_seq_key_positions(codec, shape, mode):
    recs = seq_key_records()
    for lead in (0, 1, 2, 3, 5, 9, 14):
        data, off = T.pack_records([b"\0" * lead] + recs)
        exp = T.oracle_decode(data, off, mode)
        if mode == T.DEC_PARSE:
            assert 100 < int((exp["flags"] & T.FL_SEQ_KEY != 0).sum()) < len(recs)
        assert_same_decode(gpu_decode(codec, data, off, mode, in_bytes=shape), exp)


def long_seq_key_records(seed):
    """Payloads longer than the per-lane scan limit (the window-wide scan path): keys at random
    positions and alignments, keys in the other fields only (never flagged), several keys per
    record (a lane's chunks with two hits: the per-lane fallback), split keys, near misses."""
    key = b"_sequence_number"
    rng = np.random.default_rng(seed)
    recs = []
    for k in range(700):
        plen = int(rng.integers(257, 700)) if k % 5 else int(rng.integers(16, 256))
        pay = bytearray(rng.choice(np.frombuffer(b"q_sequnbr{}:,", np.uint8), plen).tobytes())
        kind = k % 7
        if kind in (0, 1, 2):
            at = int(rng.integers(0, plen - 15))
            pay[at:at + 16] = key
        if kind == 2 and plen > 80:
            at = int(rng.integers(0, plen - 15))
            pay[at:at + 16] = key
        if kind == 3:
            at = int(rng.integers(0, plen - 15))
            pay[at:at + 16] = key[:9] + b"X" + key[10:]
        other = key if kind == 4 else b"id"
        if kind == 5:  # split between payload and headers
            pay[-5:] = key[:5]
            recs.append(T.tm_wire([b"orders", b"T", other, bytes(pay), key[5:] + b"zz"], k))
            continue
        recs.append(T.tm_wire([b"orders", other, b"u" * (k % 5), bytes(pay), b"{}"], k))
    return recs


@pytest.mark.parametrize("seed", [1, 2])
def test_decode_seq_key_long_payloads(codec, shape, seed):
    recs = long_seq_key_records(seed)
    for lead in (0, 3, 8):
        data, off = T.pack_records([b"\0" * lead] + recs)
        exp = T.oracle_decode(data, off, T.DEC_PARSE)
        assert 100 < int((exp["flags"] & T.FL_SEQ_KEY != 0).sum()) < len(recs)
        assert_same_decode(gpu_decode(codec, data, off, T.DEC_PARSE, in_bytes=shape), exp)


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
def test_decode_mixed(codec, shape, mode):
    data, off = T.mixed_records(50000)
    assert_same_decode(gpu_decode(codec, data, off, mode, in_bytes=shape), T.oracle_decode(data, off, mode))


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
def test_decode_large_records(codec, shape, mode):
    # records far larger than the 16 KiB LDS window (global-memory read path)
    rng = np.random.default_rng(11)
    recs = []
    for k in range(200):
        f = [rng.integers(32, 127, int(rng.integers(0, 9000)), dtype=np.uint8).tobytes() for _ in range(5)]
        r = T.tm_wire(f, k)
        recs.append(r if k % 4 else r + b"\0" * 8)
        recs.append(T.ack_wire(f[0][:500], f[1][:300], f[2][:70], k) + b"\0" * (k % 9))
    data, off = T.pack_records(recs)
    assert_same_decode(gpu_decode(codec, data, off, mode, in_bytes=shape), T.oracle_decode(data, off, mode))


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
def test_decode_window_chains(codec, shape, mode):
    # tiles that take many windows: records of 0.3-6 KiB (a 64-record tile spans up to ~30 windows),
    # records larger than any window among them
    # (parsed from HBM between staged ones), and runs of short records between long ones
    rng = np.random.default_rng(29)
    recs = []
    for k in range(1500):
        kind = k % 11
        if kind == 0:
            plen = int(rng.integers(16500, 20000))  # past every window
        elif kind in (1, 2):
            plen = int(rng.integers(0, 40))
        else:
            plen = int(rng.integers(300, 6000))
        pay = rng.integers(32, 127, plen, dtype=np.uint8).tobytes()
        if k % 13 == 0 and plen >= 16:
            at = int(rng.integers(0, plen - 15))
            pay = pay[:at] + b"_sequence_number" + pay[at + 16:]
        if k % 7 == 3:
            recs.append(T.ack_wire(pay[:200], b"orders", pay[200:240], k))
        else:
            recs.append(T.tm_wire([b"orders", b"T", b"u" * (k % 30), pay, b"{}"], k) + b"\0" * (k % 5))
    for lead in (0, 7):
        data, off = T.pack_records([b"\0" * lead] + recs)
        assert_same_decode(gpu_decode(codec, data, off, mode, in_bytes=shape), T.oracle_decode(data, off, mode))


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
def test_roundtrip_materialized(codec, flags):
    # encode on the GPU, decode on the GPU, rebuild ParseResults: fields come back byte-identical
    arena, L, ts = T.var_orders(3000, seed=5)
    out, off, st = gpu_encode(codec, arena, L, ts, flags=flags)
    dec = gpu_decode(codec, out, off, T.DEC_PARSE)
    starts = np.concatenate([[0], np.cumsum(L.reshape(-1).astype(np.int64))])
    for i in range(ts.size):
        rec = bytes(out[off[i]: off[i + 1]])
        pr = T.materialize_parse(rec, T.row(dec, i))
        f = [bytes(arena[starts[5 * i + k]: starts[5 * i + k + 1]]) for k in range(5)]
        assert pr["success"] and pr["message_type"] == f[1] and pr["message_id"] == f[2] and pr["payload"] == f[3]
        assert pr["timestamp"] == int(ts[i]) and pr["block_length"] == 16
        # wire form keeps headers; the reference-truncated form loses them to E100
        assert pr["headers"] == (b"" if flags else f[4])


@pytest.mark.parametrize("kind", ["fixed", "var", "session"])
def test_encode_capacity_overflow(codec, kind):
    """out_capacity smaller than the stream: records ending past it get SBE_ENC_OVERFLOW, offsets
    are unchanged, every record that fits is bit-exact, and nothing is written past the capacity."""
    if kind == "var":
        arena, L, ts = T.var_orders(3000, seed=21)
    else:
        arena, L, ts = T.fixed256_orders(3000)
    if kind == "session":
        eo, eoff, est = T.oracle_encode_session(arena, L, ts, 5, 6)
    else:
        eo, eoff, est = T.oracle_encode(arena, L, ts)
    for cap in (int(eoff[-1]) // 3 + 5, int(eoff[-1]) - 1, 4096 + 7):
        guard = 8192
        big = torch.full((cap + guard,), 0xAB, dtype=torch.uint8, device="cuda")
        a = to_dev(arena, torch.uint8)
        l = to_dev(L.view(np.int32), torch.int32)
        t = to_dev(ts.view(np.int64), torch.int64)
        if kind == "session":
            enc = codec.encode_session_batch(a, l, t, 5, 6, flags=0, out=big[:cap])
        else:
            enc = codec.encode_topic_batch(a, l, t, out=big[:cap])
        torch.cuda.synchronize()
        off = enc.out_off.cpu().numpy().view(np.uint64)
        st = enc.status.cpu().numpy()
        np.testing.assert_array_equal(off, eoff)
        fits = eoff[1:] <= cap
        np.testing.assert_array_equal(st[fits], est[fits])
        assert (st[~fits] == T.ENC_OVERFLOW).all()
        got = big.cpu().numpy()
        assert (got[cap:] == 0xAB).all(), "write past out_capacity"
        last = int(eoff[1:][fits][-1]) if fits.any() else 0
        np.testing.assert_array_equal(got[:last], eo[:last])


def test_encode_input_offsets_past_2gib(codec):
    """E109 records whose strings total more than 2 GiB inside one tile, then valid records: the
    valid records' input offsets come from 64-bit tile sums (a lane read of a sum with bit 31 set
    once sign-extended into the high word)."""
    n_bad, big = 32, 70_000_000
    arena_v, L_v, ts_v = T.fixed256_orders(40)
    dev = torch.device("cuda")
    arena = torch.zeros(n_bad * big + arena_v.size, dtype=torch.uint8, device=dev)
    arena[n_bad * big:] = torch.from_numpy(arena_v).to(dev)
    L = np.concatenate([np.tile(np.array([[big, 0, 0, 0, 0]], np.uint32), (n_bad, 1)), L_v.reshape(-1, 5)])
    ts = np.concatenate([np.arange(1, n_bad + 1, dtype=np.uint64), ts_v])
    enc = codec.encode_topic_batch(arena, to_dev(L, torch.int32), to_dev(ts, torch.int64))
    torch.cuda.synchronize()
    n = n_bad + 40
    off = enc.out_off.cpu().numpy().view(np.uint64)
    st = enc.status.cpu().numpy()
    eo, eoff, est = T.oracle_encode(arena_v, L_v, ts_v)
    assert (st[:n_bad] == 1).all() and np.array_equal(st[n_bad:], est)
    assert (off[: n_bad + 1] == 0).all() and np.array_equal(off[n_bad:], eoff)
    assert np.array_equal(enc.out[: int(off[n])].cpu().numpy(), eo)
    del arena
