"""GPU: ParseResult.sequence_number (src/sbe_encoder.cpp:1031-1125) evaluated on the device
(sbe_eval_sequence_numbers) and the SBE_FL_SEQ_KEY / SBE_FL_SEQ_ESC flags of the decode kernel,
bit-exact against the oracle (orc_seq_eval / orc_decode_batch).  jsoncpp itself is absent, so the
oracle is a restatement (parity unpinned against jsoncpp; see test_oracle_seqnum.py)."""
import random

import numpy as np
import pytest
import torch

import sbe_testlib as T
from test_gpu_parity import assert_same_decode, to_dev
from test_oracle_seqnum import HAND_CASES, _rand_doc, _rand_number

pytestmark = pytest.mark.gpu

KEY = b"_sequence_number"


def _mangle(r: random.Random, doc: str) -> bytes:
    """jsoncpp-only syntax and escapes around a standard document."""
    b = doc.encode()
    k = r.randrange(9)
    if k == 0:
        b = b"/* c */" + b
    elif k == 1:
        b = b.replace(b", ", b" // x\n, ", 1)
    elif k == 2:
        b = b.replace(b"}", b",}", 1)
    elif k == 3:
        b = b.replace(b"_sequence_number", b"\\u005fsequence_number", 1)
    elif k == 4:
        b = b.replace(b"_sequence_number", b"_sequence_numbe\\u0072", 1)
    elif k == 5:
        b = b + b" \\ trailing"
    elif k == 6:
        b = b.replace(b'"message"', b'"m\\u0065ssage"', 1)
    elif k == 7:
        b = b"\xef\xbb\xbf" + b
    return b


def seq_payloads(seed: int, n: int):
    r = random.Random(seed)
    pays = [(d.encode() if isinstance(d, str) else d) for d, _ in HAND_CASES]
    for i in range(n):
        k = i % 4
        if k == 0:
            pays.append(_rand_doc(r).encode())
        elif k == 1:
            pays.append(_mangle(r, _rand_doc(r)))
        elif k == 2:
            pays.append(b'{"_sequence_number": ' + _rand_number(r).encode() + b"}")
        else:  # byte soup: backslashes, quotes, key fragments
            m = r.randrange(0, 300)
            soup = bytes(r.choice(b'q_sequnbr\\"{}:, 0123456789') for _ in range(m))
            if m >= 16 and r.random() < 0.5:
                at = r.randrange(0, m - 15)
                soup = soup[:at] + KEY + soup[at + 16:]
            pays.append(soup)
    return pays


def padded(r: random.Random, pay: bytes, size: int) -> bytes:
    """pay followed by whitespace up to size bytes (the root is still the same document)."""
    return pay + b" " * max(0, size - len(pay))


def run(codec, recs, lead):
    data, off = T.pack_records([b"\0" * lead] + recs)
    exp = T.oracle_decode(data, off, T.DEC_PARSE)
    exp_seq = T.oracle_seq_batch(data, off, exp)
    d = to_dev(data, torch.uint8)
    ro = to_dev(np.asarray(off, np.uint64), torch.int64)
    dec = codec.decode_batch(d, ro, mode=codec.DEC_PARSE_MESSAGE, seq=True)  # evaluated in the decode launch
    seq = codec.eval_sequence_numbers(d, ro, dec)                           # the standalone launch
    torch.cuda.synchronize()
    got = dec.numpy()
    assert_same_decode(got, exp)
    for s in (dec.seq, seq):
        got_seq = s.cpu().numpy().view(np.uint64)
        bad = np.nonzero(got_seq != exp_seq)[0]
        assert bad.size == 0, [(int(i), data[int(off[i]):int(off[i + 1])].tobytes()[:200], int(got_seq[i]),
                                int(exp_seq[i])) for i in bad[:5]]
    return exp, exp_seq


@pytest.mark.parametrize("lead", [0, 3, 9])
def test_seq_short_payloads(codec, lead):
    recs = [T.tm_wire([b"orders", b"T", b"id", p, b"{}"], i + 1) for i, p in enumerate(seq_payloads(7, 3000))]
    exp, exp_seq = run(codec, recs, lead)
    fl = exp["flags"]
    assert int((fl & T.FL_SEQ_ESC != 0).sum()) > 300
    assert int((exp_seq != 0).sum()) > 500


@pytest.mark.parametrize("lead", [0, 5])
def test_seq_long_payloads(codec, lead):
    """Payloads longer than the per-lane scan (window-wide scan, its many-hit fallback) and
    records longer than the LDS window (the HBM reader)."""
    r = random.Random(11)
    recs = []
    for i, p in enumerate(seq_payloads(12, 1200)):
        size = r.choice([300, 700, 2000, 20000]) if i % 50 == 0 else r.choice([257, 400, 900])
        recs.append(T.tm_wire([b"orders", b"T", b"id", padded(r, p, size), b"{}"], i + 1))
    exp, exp_seq = run(codec, recs, lead)
    assert int((exp["flags"] & T.FL_SEQ_ESC != 0).sum()) > 100
    assert int((exp_seq != 0).sum()) > 200


@pytest.mark.parametrize("lead", [0, 7])
def test_seq_lane_scan_records_to_320(codec, lead):
    """Tiles whose records are all at most 320 B (the per-lane scan's limit, e.g. 280-B session
    frames) with payloads of 200-280 B: keys and escapes at every position of the lane scan."""
    r = random.Random(17)
    recs = []
    for i, p in enumerate(q for q in seq_payloads(14, 800) if len(q) <= 240):
        size = r.randint(max(160, len(p)), 260)
        tm = T.tm_wire([b"orders", b"T", b"id", padded(r, p, size), b"{}"], i + 1)
        recs.append(T.session_wrap(tm) if i % 3 == 0 and len(tm) + 32 <= 320 else tm)
    assert max(len(x) for x in recs) <= 320
    exp, exp_seq = run(codec, recs, lead)
    assert int((exp_seq != 0).sum()) > 50


def test_seq_wrapped_and_unflagged(codec):
    """Session-wrapped records are evaluated too; records of other kinds are never written."""
    r = random.Random(3)
    recs = []
    for i, p in enumerate(seq_payloads(13, 400)):
        tm = T.tm_wire([b"orders", b"T", b"id", p, b"{}"], i + 1)
        recs.append(T.session_wrap(tm) if i % 2 else tm)
        recs.append(T.ack_wire(b"msg_" + str(i).encode(), b"orders", b"\\corr", 1_760_000_000_000 + i))
    exp, exp_seq = run(codec, recs, 0)
    assert not exp_seq[exp["status"] != T.ST_TM].any()


def test_seq_bench_workload_has_no_candidates(codec):
    """The headline workload's payloads carry neither the key nor a backslash: the evaluation
    launch writes nothing there."""
    arena, L, ts = T.fixed256_orders(20000)
    eo, eoff, _ = T.oracle_encode(arena, L, ts)
    exp = T.oracle_decode(eo, eoff, T.DEC_PARSE)
    assert not (exp["flags"] & (T.FL_SEQ_KEY | T.FL_SEQ_ESC)).any()
    d = to_dev(eo, torch.uint8)
    ro = to_dev(np.asarray(eoff, np.uint64), torch.int64)
    seq1 = torch.full((20000,), 77, dtype=torch.int64, device="cuda")
    dec = codec.decode_batch(d, ro, mode=codec.DEC_PARSE_MESSAGE, seq=seq1)
    seq = torch.full((20000,), 77, dtype=torch.int64, device="cuda")
    codec.eval_sequence_numbers(d, ro, dec, seq=seq)
    torch.cuda.synchronize()
    assert bool((seq == 77).all()) and bool((seq1 == 77).all())
