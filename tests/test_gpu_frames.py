"""GPU parity for the SURVEY §8(f) rows built on the same kernels: session-framed TopicMessages
(sbe_encode_session_batch) and the Lite templates (sbe_encode_lite_batch, sbe_decode_batch LITE),
through the C ABI against the oracle, bit-exact."""
import numpy as np
import pytest
import torch

import sbe_testlib as T
from test_gpu_parity import SHAPES, assert_same_decode, gpu_decode, shape, to_dev  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


def assert_same_stream(go, goff, gst, eo, eoff, est):
    np.testing.assert_array_equal(goff, eoff)
    np.testing.assert_array_equal(gst, est)
    if not np.array_equal(go, eo):
        i = int(np.nonzero(go != eo)[0][0])
        rec = int(np.searchsorted(eoff, i, side="right") - 1)
        raise AssertionError(f"output byte {i} (record {rec}) differs: {go[i]} != {eo[i]}")


def fetch(enc, n):
    torch.cuda.synchronize()
    off = enc.out_off.cpu().numpy().view(np.uint64)
    return enc.out[: int(off[n])].cpu().numpy(), off, enc.status.cpu().numpy()


def check_session(codec, arena, L, ts, term, sess, str_off=None, flags=T.ENC_REF_TRUNCATE8, ts_default=0):
    a = to_dev(arena if arena.size else np.zeros(16, np.uint8), torch.uint8)
    o = None if str_off is None else to_dev(np.asarray(str_off, np.uint32).reshape(-1, 5), torch.int32)
    enc = codec.encode_session_batch(a, to_dev(np.asarray(L, np.uint32).reshape(-1, 5), torch.int32),
                                     to_dev(np.asarray(ts, np.uint64), torch.int64), term, sess, str_off=o,
                                     flags=flags, ts_default=ts_default)
    got = fetch(enc, ts.size)
    exp = T.oracle_encode_session(arena, L, ts, term, sess, str_off, flags, ts_default)
    assert_same_stream(*got, *exp)
    return got


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
@pytest.mark.parametrize("n", [1, 33, 1000, 4096 * 3 + 17])
def test_session_fixed256(codec, n, flags):
    arena, L, ts = T.fixed256_orders(n)
    check_session(codec, arena, L, ts, 0x0102030405060708, -7, flags=flags)


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
def test_session_var_and_gather(codec, flags):
    arena, L, ts = T.var_orders(20000, seed=5)
    check_session(codec, arena, L, ts, 3, 2**62, flags=flags)
    n = 3000
    arena, L, ts = T.var_orders(n, seed=6)
    starts = np.zeros(n * 5 + 1, np.int64)
    starts[1:] = np.cumsum(L.reshape(-1).astype(np.int64))
    off = (starts[:-1] + 5).astype(np.uint32)  # ragged: shifted arena
    shifted = np.concatenate([np.full(5, 0xEE, np.uint8), arena])
    check_session(codec, shifted, L, ts, -1, 1, str_off=off, flags=flags)


def test_session_edges(codec):
    rng = np.random.default_rng(11)
    lens = [[0, 0, 0, 0, 0], [65534, 0, 0, 0, 1], [0, 0, 0, 65535, 0], [70000, 1, 1, 1, 1], [1, 2, 3, 4, 5]]
    lens += [list(rng.integers(0, 30, 5)) for _ in range(300)]
    L = np.array(lens, np.uint32)
    arena = rng.integers(0, 256, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    ts = rng.integers(0, 2**63, len(L), dtype=np.uint64)
    ts[::5] = 0
    for flags in (0, T.ENC_REF_TRUNCATE8):
        check_session(codec, arena, L, ts, 42, 43, flags=flags, ts_default=99)


@pytest.mark.parametrize("pattern", ["sprinkled", "zero_run", "long_run"])
def test_session_virtual_tiles_with_edges(codec, pattern):
    arena, L, ts = T.vt_mixed(3 * 4096 + 77, pattern, seed=22)
    for flags in (0, T.ENC_REF_TRUNCATE8):
        check_session(codec, arena, L, ts, 5, -9, flags=flags, ts_default=77)


def lite_gpu(codec, t, arena, L, tid, seq, str_off=None):
    nf = T.LITE_NF[t]
    a = to_dev(arena if arena.size else np.zeros(16, np.uint8), torch.uint8)
    o = None if str_off is None else to_dev(np.asarray(str_off, np.uint32).reshape(-1, nf), torch.int32)
    enc = codec.encode_lite_batch(t, a, to_dev(np.asarray(L, np.uint32).reshape(-1, nf), torch.int32),
                                  to_dev(np.asarray(tid, np.uint32), torch.int32),
                                  to_dev(np.asarray(seq, np.uint64), torch.int64), str_off=o)
    return fetch(enc, seq.size)


@pytest.mark.parametrize("t", [301, 201, 202])
@pytest.mark.parametrize("n", [1, 100, 50000])
def test_lite_encode(codec, t, n):
    arena, L, tid, seq = T.lite_records(n, t)
    assert_same_stream(*lite_gpu(codec, t, arena, L, tid, seq), *T.oracle_encode_lite(t, arena, L, tid, seq))


@pytest.mark.parametrize("t", [301, 201])
def test_lite_encode_gather_and_edges(codec, t):
    nf = T.LITE_NF[t]
    rng = np.random.default_rng(t + 1)
    lens = [[0] * nf, [65534] + [0] * (nf - 1), [65535] + [1] * (nf - 1), [1] * (nf - 1) + [70000]]
    lens += [list(rng.integers(0, 50, nf)) for _ in range(500)]
    L = np.array(lens, np.uint32)
    arena = rng.integers(0, 256, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    tid = rng.integers(0, 2**32, len(L), dtype=np.uint64).astype(np.uint32)
    seq = rng.integers(0, 2**64 - 1, len(L), dtype=np.uint64)
    assert_same_stream(*lite_gpu(codec, t, arena, L, tid, seq), *T.oracle_encode_lite(t, arena, L, tid, seq))
    starts = np.zeros(L.size + 1, np.int64)
    starts[1:] = np.cumsum(L.reshape(-1).astype(np.int64))
    off = (starts[:-1] + 3).astype(np.uint32)
    shifted = np.concatenate([np.zeros(3, np.uint8), arena])
    assert_same_stream(*lite_gpu(codec, t, shifted, L, tid, seq, off),
                       *T.oracle_encode_lite(t, shifted, L, tid, seq, off))


@pytest.mark.parametrize("lo,hi", [(60, 260), (0, 900)])
def test_lite301_windows_past_three_rows(codec, lo, hi):
    """CommitOffsetLite windows of 3-8 KiB (the store rows past the first three, which the
    ~77-B records of the usual batch never reach), packed and gather input."""
    rng = np.random.default_rng(lo + hi)
    L = rng.integers(lo, hi, (3000, 2)).astype(np.uint32)
    L[rng.random(3000) < 0.3] = rng.integers(0, 20, 2)  # small records in between
    arena = rng.integers(0, 256, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    tid = rng.integers(0, 2**32, len(L), dtype=np.uint64).astype(np.uint32)
    seq = rng.integers(0, 2**64 - 1, len(L), dtype=np.uint64)
    assert_same_stream(*lite_gpu(codec, 301, arena, L, tid, seq), *T.oracle_encode_lite(301, arena, L, tid, seq))
    starts = np.zeros(L.size + 1, np.int64)
    starts[1:] = np.cumsum(L.reshape(-1).astype(np.int64))
    off = (starts[:-1] + 5).astype(np.uint32)
    shifted = np.concatenate([np.zeros(5, np.uint8), arena])
    assert_same_stream(*lite_gpu(codec, 301, shifted, L, tid, seq, off),
                       *T.oracle_encode_lite(301, shifted, L, tid, seq, off))


def lite_decode_records():
    """Every Lite decode fixture record, plus TopicMessages and junk, at every start alignment."""
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lite_ref.json")))
    recs = [bytes.fromhex(c["rec"]) for c in gold["decode"]]
    recs += [b"", b"\x0c\x00", T.tm_wire([b"orders", b"X", b"u", b"{}", b""], 5), bytes(19), bytes(25)]
    return recs


def test_lite_decode_edges_every_alignment(codec, shape):
    base = lite_decode_records()
    for shift in range(16):
        recs = [bytes(shift)] + base if shift else base
        data, off = T.pack_records(recs)
        assert_same_decode(gpu_decode(codec, data, off, T.DEC_LITE, in_bytes=shape),
                           T.oracle_decode(data, off, T.DEC_LITE))


@pytest.mark.parametrize("t", [301, 202])
def test_lite_roundtrip_on_device(codec, t):
    arena, L, tid, seq = T.lite_records(200000, t, seed=17)
    out, off, st = lite_gpu(codec, t, arena, L, tid, seq)
    assert (st == 0).all()
    dec = gpu_decode(codec, out, off, T.DEC_LITE)
    assert (dec["status"] == T.ST_LITE).all()
    np.testing.assert_array_equal(dec["ts"], seq)
    np.testing.assert_array_equal(dec["view_off"][:, 4], tid)
    nf = T.LITE_NF[t]
    np.testing.assert_array_equal(dec["view_len"][:, :nf], L)
    assert_same_decode(dec, T.oracle_decode(out, off, T.DEC_LITE))
