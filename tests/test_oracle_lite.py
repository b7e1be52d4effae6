"""CPU: the oracle restatement of the SURVEY §8(f) rows built this round — Lite templates
(CommitOffsetLite 301, OrderRequestLite 201, OrderNotificationLite 202) and session framing —
against the reference's own SBE flyweights (tests/golden/lite_ref.json, live oracle/_ref) and the
session header restated from src/session_manager.cpp:936-967.  Bit-exact."""
import json
import os
import struct

import numpy as np
import pytest

import sbe_testlib as T
from test_oracle_golden import fields_of, same

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LITE = json.load(open(os.path.join(GOLD, "lite_ref.json")))


def lite_encode_one(t, fields, tid, seq):
    L = np.array([[len(f) for f in fields]], np.uint32)
    arena = np.frombuffer(b"".join(fields), np.uint8) if sum(len(f) for f in fields) else np.zeros(0, np.uint8)
    out, off, st = T.oracle_encode_lite(t, arena, L, np.array([tid], np.uint32), np.array([seq], np.uint64))
    return bytes(out[int(off[0]):int(off[1])]), int(st[0])


@pytest.mark.parametrize("case", LITE["encode"], ids=lambda c: f"{c['template']}-{c['topic_id']}-{c['status']}")
def test_lite_encode_matches_reference_flyweights(case):
    got, st = lite_encode_one(case["template"], fields_of(case["fields"]), case["topic_id"], int(case["sequence"]))
    assert st == case["status"]
    if st == 0:
        assert same(case["record"], got)
    else:
        assert got == b""


def _rec(case):
    return bytes.fromhex(case["rec"])


@pytest.mark.parametrize("case", LITE["decode"], ids=lambda c: c["name"])
def test_lite_decode_matches_reference_flyweights(case):
    rec = _rec(case)
    d = T.oracle_decode(*T.pack_records([rec]), mode=T.DEC_LITE)
    row = T.row(d, 0)
    assert tuple(int(x) for x in row["hdr"]) == struct.unpack("<4H", rec[:8])
    if case["e100"]:
        assert row["status"] == T.ST_LITE_E100
        assert not any(row["view_len"]) and not any(row["view_off"])
        return
    assert row["status"] == T.ST_LITE
    assert int(row["ts"]) == int(case["sequence"]) and int(row["view_off"][4]) == case["topic_id"]
    for k, fb in enumerate(case["fields"]):
        o, n = int(row["view_off"][k]), int(row["view_len"][k])
        assert same(fb, rec[o:o + n])


def test_lite_decode_rejects_other_records():
    tm = T.tm_wire([b"orders", b"X", b"u", b"{}", b""], 5)
    cases = [b"", b"\x0c\x00\x2d\x01\x01", tm, tm[:2] + struct.pack("<H", 301) + b"\x02\x00" + tm[6:],
             struct.pack("<4H", 12, 999, 1, 1) + bytes(30)]
    d = T.oracle_decode(*T.pack_records(cases), mode=T.DEC_LITE)
    assert list(d["status"]) == [T.ST_LITE_NOT_LITE] * 5
    # records shorter than the 12 fixed bytes: the flyweight would read past the record → E100
    short = struct.pack("<4H", 0, 301, 1, 1) + bytes(11)
    d = T.oracle_decode(*T.pack_records([short]), mode=T.DEC_LITE)
    assert d["status"][0] == T.ST_LITE_E100


def test_session_header_bytes():
    """create_session_message_header_buffer + update_session_header (src/session_manager.cpp:936-967,
    :1018-1046): {blockLength 24, templateId 1, schemaId 111, version 8}, i64 leadershipTermId,
    i64 clusterSessionId, i64 timestamp 0; send_combined_message puts it before the business
    message with no gap (:1118-1144)."""
    arena, L, ts = T.fixed256_orders(20)
    for flags in (0, T.ENC_REF_TRUNCATE8):
        plain, poff, pst = T.oracle_encode(arena, L, ts, flags=flags)
        fr, foff, fst = T.oracle_encode_session(arena, L, ts, 0x0102030405060708, -2, flags=flags)
        assert (pst == fst).all()
        hdr = struct.pack("<4Hqqq", 24, 1, 111, 8, 0x0102030405060708, -2, 0)
        for i in range(20):
            rec = bytes(fr[foff[i]:foff[i + 1]])
            assert rec == hdr + bytes(plain[poff[i]:poff[i + 1]])


def test_session_e109_and_default_timestamp():
    fields = [b"t", b"m", b"u", b"\x5a" * 65535, b""]
    L = np.array([[len(f) for f in fields], [1, 1, 1, 1, 1]], np.uint32)
    arena = np.frombuffer(b"".join(fields) + b"abcde", np.uint8)
    out, off, st = T.oracle_encode_session(arena, L, np.array([1, 0], np.uint64), 3, 4, ts_default=777)
    assert list(st) == [4, 0] and int(off[1]) == 0
    rec = bytes(out[int(off[1]):int(off[2])])
    assert len(rec) == 32 + 34 + 5 and struct.unpack("<Q", rec[40:48])[0] == 777


@pytest.mark.skipif(not T.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("t", [301, 201, 202])
def test_lite_random_vs_ref(t):
    rng = np.random.default_rng(t)
    nf = T.LITE_NF[t]
    n = 300
    fields = [[bytes(rng.integers(0, 256, int(rng.choice([0, 1, 3, 17, 29, 200])), dtype=np.uint8))
               for _ in range(nf)] for _ in range(n)]
    tid = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    seq = rng.integers(0, 2**63, n, dtype=np.uint64)
    L = np.array([[len(f) for f in r] for r in fields], np.uint32)
    arena = np.frombuffer(b"".join(b"".join(r) for r in fields), np.uint8)
    out, off, st = T.oracle_encode_lite(t, arena, L, tid, seq)
    recs = []
    for i in range(n):
        rc, ref = T.ref_lite_encode(t, fields[i], int(tid[i]), int(seq[i]))
        assert rc == 0 and bytes(out[off[i]:off[i + 1]]) == ref, i
        # mutate: truncate / slack / blockLength / a length field
        b = bytearray(ref)
        op = rng.integers(0, 4)
        if op == 0:
            b = b[: int(rng.integers(20, len(b) + 1))]
        elif op == 1:
            b += bytes(int(rng.integers(1, 9)))
        elif op == 2:
            b[0:2] = int(rng.integers(0, 40)).to_bytes(2, "little")
        elif len(b) > 22:
            b[20:22] = int(rng.integers(0, 300)).to_bytes(2, "little")
        recs.append(bytes(b))
    d = T.oracle_decode(*T.pack_records(recs), mode=T.DEC_LITE)
    for i, r in enumerate(recs):
        row = T.row(d, i)
        rc, rtid, rseq, f = T.ref_lite_decode(r)
        if rc:
            assert row["status"] == T.ST_LITE_E100, i
            continue
        assert row["status"] == T.ST_LITE and int(row["ts"]) == rseq and int(row["view_off"][4]) == rtid, i
        for k in range(nf):
            o, m = int(row["view_off"][k]), int(row["view_len"][k])
            assert r[o:o + m] == f[k], (i, k)
