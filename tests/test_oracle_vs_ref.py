"""CPU: the oracle restatement against the reference's own flyweights (oracle/_ref) on seeded
random inputs — encode (both lengths) and the three flyweight decode sequences.  Skipped where
oracle/_ref was not built (it needs /root/reference, absent on the GPU box)."""
import numpy as np
import pytest

import sbe_testlib as T

pytestmark = pytest.mark.skipif(not T.ref_available(), reason="oracle/_ref not built (needs /root/reference)")


def rand_fields(rng):
    out = []
    for _ in range(5):
        n = int(rng.choice([0, 1, 2, 3, 5, 16, 29, 100, 300]))
        if rng.random() < 0.5:
            out.append(bytes(rng.integers(32, 127, n, dtype=np.uint8)))
        else:
            out.append(bytes(rng.integers(0, 256, n, dtype=np.uint8)))
    return out


def test_encode_random_vs_ref():
    rng = np.random.default_rng(2024)
    recs = [rand_fields(rng) for _ in range(400)]
    ts = rng.integers(1, 2**63, len(recs), dtype=np.uint64)
    L = np.array([[len(f) for f in r] for r in recs], np.uint32)
    arena = np.frombuffer(b"".join(b"".join(r) for r in recs), np.uint8)
    for flags, wire in ((0, True), (T.ENC_REF_TRUNCATE8, False)):
        out, off, st = T.oracle_encode(arena, L, ts, flags=flags)
        for i, r in enumerate(recs):
            rc, ref = T.ref_encode(r, int(ts[i]), wire=wire)
            assert rc == 0 and bytes(out[off[i]:off[i + 1]]) == ref, i


def mutate(rng, rec):
    """Truncate, extend, or rewrite header/length bytes of a record."""
    b = bytearray(rec)
    op = rng.integers(0, 5)
    if op == 0 and len(b) > 8:
        b = b[: int(rng.integers(8, len(b)))]
    elif op == 1:
        b += bytes(rng.integers(0, 256, int(rng.integers(1, 20)), dtype=np.uint8))
    elif op == 2:
        b[0:2] = int(rng.integers(0, 64)).to_bytes(2, "little")  # blockLength
    elif op == 3 and len(b) > 30:
        p = int(rng.integers(16, len(b) - 2))
        b[p: p + 2] = int(rng.integers(0, 400)).to_bytes(2, "little")
    return bytes(b)


def test_tm_flyweight_decodes_random_vs_ref():
    rng = np.random.default_rng(7)
    for _ in range(3000):
        rec = mutate(rng, T.tm_wire(rand_fields(rng), int(rng.integers(0, 2**63))))
        if len(rec) < 8 or rec[2:6] != b"\x01\x00\x01\x00":
            continue
        d = T.oracle_decode(*T.pack_records([rec]), mode=T.DEC_PARSE)
        pr = T.materialize_parse(rec, T.row(d, 0))
        rc, ts, f, hok = T.ref_tm_decode(rec)
        assert pr["success"] == (rc == 0), rec.hex()
        if rc == 0:
            assert pr["timestamp"] == T._i64(ts)
            assert [pr["message_type"], pr["message_id"], pr["payload"]] == f[1:4]
            assert pr["headers"] == (f[4] if hok else b"")
        d = T.oracle_decode(*T.pack_records([rec]), mode=T.DEC_EGRESS)
        out = T.materialize_egress(rec, T.row(d, 0))
        rc, f = T.ref_egress_tm(rec)
        if rc:
            assert out == ("throw", b"buffer too short [E100]"), rec.hex()
        elif f[0] == b"":
            assert out == ("none",)
        else:
            assert out == ("tm", tuple(f)), rec.hex()


def test_ack_flyweight_decodes_random_vs_ref():
    rng = np.random.default_rng(11)
    for _ in range(3000):
        f = rand_fields(rng)[:3]
        rec = mutate(rng, T.ack_wire(*f, int(rng.integers(0, 2**63))) + b"\0" * int(rng.integers(0, 12)))
        if len(rec) < 16 or rec[2:6] != b"\x02\x00\x01\x00" or (len(rec) == 16 and rec[:2] == b"\x08\x00"):
            continue
        d = T.oracle_decode(*T.pack_records([rec]), mode=T.DEC_EGRESS)
        out = T.materialize_egress(rec, T.row(d, 0))
        rc, ts, fl = T.ref_ack_decode(rec)
        if rc:
            assert out[0] != "ack", rec.hex()
        else:
            assert out[0] == "ack" and [out[1]["message_id"], out[1]["topic"], out[1]["correlation_id"]] == fl
            assert out[1]["timestamp_nanos"] == int(T.oracle().orc_to_nanos_auto(ts))
