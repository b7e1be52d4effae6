"""GPU parity at BASELINE.json's full configuration sizes.

- config 2: 1 M fixed-256 Order records, encode (wire-correct and reference-truncated), bit-exact
  against the oracle over the whole batch;
- config 3: 1 M mixed TopicMessage / Ack records, decode in both modes, bit-exact against the
  oracle over the whole batch;
- config 4: 16 M variable-length Order records, encode → decode round trip on the GPU: the
  encoding bit-exact against the oracle's over the whole batch, and size-independent properties
  of the decode (every record a TopicMessage, views == the encoded field layout, the strings
  recovered byte for byte).

The oracle runs multi-threaded here (C with OpenMP).
"""
import numpy as np
import pytest
import torch

import sbe_testlib as T

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16
DEV = "cuda"


def _dev(a, dtype):
    a = np.ascontiguousarray(a)
    view = {torch.uint8: np.uint8, torch.int32: np.int32, torch.int64: np.int64}[dtype]
    return torch.from_numpy(a.view(view)).to(DEV)


def _first_diff(got, exp):
    return int(np.nonzero(got != exp)[0][0])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
def test_config2_encode_1m_bit_exact(codec, flags):
    n = 1_000_000
    arena, L, ts = T.fixed256_orders(n)
    enc = codec.encode_topic_batch(_dev(arena, torch.uint8), _dev(L, torch.int32), _dev(ts, torch.int64),
                                   flags=flags)
    torch.cuda.synchronize()
    eo, eoff, est = T.oracle_encode(arena, L, ts, flags=flags, nthreads=ORACLE_THREADS)
    off = enc.out_off.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(off, eoff)
    rec = 256 - (8 if flags else 0)
    assert int(off[-1]) == rec * n and np.all(np.diff(off.astype(np.int64)) == rec)
    np.testing.assert_array_equal(enc.status.cpu().numpy(), est)
    got = enc.out[: int(off[-1])].cpu().numpy()
    if not np.array_equal(got, eo):
        i = _first_diff(got, eo)
        raise AssertionError(f"byte {i} (record {i // rec}) differs: {got[i]} != {eo[i]}")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
def test_config3_mixed_decode_1m_bit_exact(codec, mode):
    n = 1_000_000
    data, off = T.mixed_records(n)
    dec = codec.decode_batch(_dev(data, torch.uint8), _dev(off, torch.int64), mode=mode)
    torch.cuda.synchronize()
    got = dec.numpy()
    exp = T.oracle_decode(data, off, mode, nthreads=ORACLE_THREADS)
    for k in exp:
        g, e = got[k], exp[k]
        if not np.array_equal(g, e):
            bad = np.nonzero((g != e).reshape(len(e), -1).any(1))[0]
            raise AssertionError(f"{k} differs at {bad.size} records, first {bad[:5]}")
    # the mix the workload promises
    st = got["status"]
    if mode == T.DEC_PARSE:
        assert 0.67 < np.mean(st == T.ST_TM) < 0.71 and 0.29 < np.mean(st == T.ST_ACK) < 0.33
    else:
        assert np.mean(st == T.ST_EG_ACK) > 0.13 and np.mean(st == T.ST_EG_ACK_SIMPLE) > 0.005


@pytest.mark.timeout(900)
def test_config4_roundtrip_16m_var(codec):
    n = 16 * 1024 * 1024
    d_arena, d_len, d_ts = T.var_orders_t(n, DEV)  # T.var_orders(n), generated on the device
    arena, L = d_arena.cpu().numpy(), d_len.cpu().numpy().view(np.uint32)
    ts = d_ts.cpu().numpy().view(np.uint64)
    enc = codec.encode_topic_batch(d_arena, d_len, d_ts)
    # the stream's size is known (every record encodable): the wide-record decode kernel runs
    dec = codec.decode_batch(enc.out, enc.out_off, mode=codec.DEC_PARSE_MESSAGE, in_bytes=int(d_arena.numel()) + 34 * n)
    torch.cuda.synchronize()

    # encode: bit-exact against the oracle over the whole batch
    eo, eoff, _ = T.oracle_encode(arena, L, ts, nthreads=ORACLE_THREADS)
    off = enc.out_off.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(off, eoff)
    assert int((enc.status != 0).sum()) == 0
    got = enc.out[: int(off[-1])].cpu().numpy()
    if not np.array_equal(got, eo):
        i = _first_diff(got, eo)
        raise AssertionError(f"byte {i} differs: {got[i]} != {eo[i]}")
    del got, eo, arena

    # decode of the GPU stream: size-independent properties, on the device
    assert int((dec.status != T.ST_TM).sum()) == 0
    assert int((dec.flags != 0).sum()) == 0          # no seq key, nothing swallowed, not wrapped
    assert torch.equal(dec.ts, d_ts)
    Ld = d_len.view(n, 5).to(torch.int64)
    assert torch.equal(dec.view_len.view(n, 5).to(torch.int64), Ld)
    # string f of a wire record starts at 26 + Σ_{g<f} (L_g + 2)
    cols, o = [], torch.full((n,), 26, dtype=torch.int64, device=DEV)
    for f in range(5):  # (column by column: torch's cumsum over a short dim of 16 M rows fails to launch)
        cols.append(o)
        o = o + Ld[:, f] + 2
    exp_off = torch.stack(cols, dim=1)
    assert torch.equal(dec.view_off.view(n, 5).to(torch.int64), exp_off)
    # the strings come back byte for byte: gathered through the decoded views, in record and
    # field order, they are the input arena (slices of 1 M records bound the index tensors)
    a_off = torch.zeros(n + 1, dtype=torch.int64, device=DEV)
    a_off[1:] = torch.cumsum(Ld.sum(1), 0)
    step = 1 << 20
    for r0 in range(0, n, step):
        r1 = min(n, r0 + step)
        lens = dec.view_len[r0:r1].reshape(-1).to(torch.int64)
        starts = (enc.out_off[r0:r1].unsqueeze(1) + dec.view_off[r0:r1].to(torch.int64)).reshape(-1)
        first = torch.cumsum(lens, 0) - lens
        idx = torch.repeat_interleave(starts - first, lens) + torch.arange(int(lens.sum()), device=DEV)
        assert torch.equal(enc.out[idx], d_arena[int(a_off[r0]): int(a_off[r1])]), \
            f"strings differ in records [{r0},{r1})"
