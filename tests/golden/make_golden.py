"""Generate the golden fixtures under tests/golden/ (run in the container where /root/reference
is present and oracle/_ref/libsbe_ref_fw.so has been built by `make -C oracle`).

Every expected value in encode_ref.json / decode_tm_ref.json / ack_ref.json / egress_tm_ref.json
is produced by the reference's own SBE-generated flyweights (include/model/*.h compiled unmodified,
driven in the reference's call order by oracle/ref_flyweights.cpp).  survey_probes.json holds the
outputs of the reference functions themselves as recorded in SURVEY.md Appendix B (probe runs of
the compiled reference in the survey container); those expectations are transcribed, not computed.

Inputs only are derived from tests/sbe_testlib.py generators and tests/sbe_testlib.edge_records().
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import sbe_testlib as T  # noqa: E402


def hx(b):
    return bytes(b).hex()


def blob(b):
    """Bytes up to 1 KiB inline as hex; larger ones as length + sha256 + head/tail (the test
    regenerates the input from the committed generators and compares digests)."""
    import hashlib
    b = bytes(b)
    if len(b) <= 1024:
        return hx(b)
    return {"len": len(b), "sha256": hashlib.sha256(b).hexdigest(), "head": hx(b[:64]), "tail": hx(b[-64:])}


def field_spec(f):
    """Large uniform fields are stored as {fill, len}; others as hex."""
    b = bytes(f)
    if len(b) > 512 and len(set(b)) == 1:
        return {"fill": b[0], "len": len(b)}
    return hx(b)


def encode_cases():
    cases = []
    # SURVEY Appendix B probe input
    cases.append(([b"orders", b"CREATE_ORDER", b"msg_1", b'{"a":1}', b'{"h":2}'], 0x1122334455667788))
    arena, L, ts = T.fixed256_orders(3)
    at = 0
    for i in range(3):
        f = []
        for k in range(5):
            f.append(bytes(arena[at: at + L[i, k]]))
            at += int(L[i, k])
        cases.append((f, int(ts[i])))
    arena, L, ts = T.var_orders(8, seed=77)
    at = 0
    for i in range(8):
        f = []
        for k in range(5):
            f.append(bytes(arena[at: at + L[i, k]]))
            at += int(L[i, k])
        cases.append((f, int(ts[i])))
    cases.append(([b""] * 5, 1))
    cases.append(([b"t", b"", b"", b"", b""], 2**64 - 1))
    cases.append(([b"orders", b"CREATE_ORDER", b"id", b"{}", b""], 5))
    cases.append(([b"\x00\xff", b"\n\r", b"\x80", b"", b"\x7f" * 5], 12345))
    big = b"\x41" * 65534
    cases.append(([big, b"x", b"", b"", b""], 7))
    for k in range(5):
        f = [b"a", b"b", b"c", b"d", b"e"]
        f[k] = b"\x5a" * 65535
        cases.append((f, 9))
    return cases


def publish_cases():
    """ClusterClient::publish_topic inputs: typical publishes (uuid "pub_<ns>", headers "{}" when the
    caller's were empty) and every field at lengths 65534 / 65535 / 65536 / 70000 / 131073 (the
    put*(const char*, int) overloads write the length mod 65536 and that many bytes)."""
    cases = []
    uid = b"pub_1760000000123456789"
    cases.append(([b"orders", b"CREATE_ORDER", uid, b'{"side":"BUY","qty":"1"}', b"{}"], 1760000000123456789))
    cases.append(([b"", b"", uid, b"", b"{}"], 1))
    cases.append(([b"_subscriptions", b"SUBSCRIPTION", uid, b'{"topic":"orders"}', b'{"h":2}'], 2**64 - 1))
    for L in (65534, 65535, 65536, 70000, 131073):
        for k in range(5):
            f = [b"orders", b"CREATE_ORDER", uid, b'{"a":1}', b"{}"]
            f[k] = bytes([0x41 + k]) * L
            cases.append((f, 7 + L))
    return cases


def main():
    if not T.ref_available():
        sys.exit("oracle/_ref/libsbe_ref_fw.so is missing: run `make -C oracle` with /root/reference present")
    out = []
    for fields, ts in encode_cases():
        rc_t, ref_t = T.ref_encode(fields, ts, wire=False)
        rc_w, ref_w = T.ref_encode(fields, ts, wire=True)
        assert rc_t == rc_w
        out.append({"fields": [field_spec(f) for f in fields], "ts": str(ts), "status": rc_t,
                    "ref_truncated": blob(ref_t), "wire": blob(ref_w)})
    json.dump({"source": "reference flyweights via oracle/_ref (SBEEncoder::encode_topic_message call order, "
                         "src/sbe_encoder.cpp:141-164; wire length per src/cluster_client.cpp:1857)",
               "cases": out}, open(os.path.join(HERE, "encode_ref.json"), "w"), indent=1)

    pub = []
    for fields, ts in publish_cases():
        rc, rec = T.ref_publish(fields, ts)
        assert rc == 0
        pub.append({"fields": [field_spec(f) for f in fields], "ts": str(ts), "record": blob(rec)})
    json.dump({"source": "reference flyweights via oracle/_ref (ClusterClient::publish_topic encoder block, "
                         "src/cluster_client.cpp:1823-1858: MessageHeader setters, wrapForEncode(buf, 8, size-8), "
                         "put*(const char*, int), 8 + encodedLength())",
               "cases": pub}, open(os.path.join(HERE, "publish_ref.json"), "w"), indent=1)

    recs = T.edge_records()
    tm, ack, eg = [], [], []
    for name, r in recs:
        if len(r) >= 8 and r[2:6] == b"\x01\x00\x01\x00":  # template 1, schema 1
            rc, ts, f, hok = T.ref_tm_decode(r)
            tm.append({"name": name, "rec": blob(r), "e100": rc, "ts": str(ts) if rc == 0 else None,
                       "fields": [blob(x) for x in f] if rc == 0 else None, "headers_ok": hok if rc == 0 else None})
            rc, f = T.ref_egress_tm(r)
            eg.append({"name": name, "rec": blob(r), "throws": rc, "fields": [blob(x) for x in f] if rc == 0 else None})
        if len(r) >= 16 and r[2:6] == b"\x02\x00\x01\x00":  # template 2, schema 1, full-ack branch
            if len(r) == 16 and r[0:2] == b"\x08\x00":
                continue  # simple control ack branch never reaches the flyweights
            rc, ts, f = T.ref_ack_decode(r)
            ack.append({"name": name, "rec": blob(r), "fails": rc, "ts": str(ts) if rc == 0 else None,
                        "fields": [blob(x) for x in f] if rc == 0 else None})
    src = "reference flyweights via oracle/_ref"
    json.dump({"source": src + " (decode_topic_message_with_sbe flyweight sequence, src/sbe_encoder.cpp:966-1135)",
               "cases": tm}, open(os.path.join(HERE, "decode_tm_ref.json"), "w"), indent=1)
    json.dump({"source": src + " (decode_ack full-ack flyweight sequence, src/ack_decoder.cpp:55-101)",
               "cases": ack}, open(os.path.join(HERE, "ack_ref.json"), "w"), indent=1)
    json.dump({"source": src + " (MessageHandler::on_egress TopicMessage sequence, message_handler.hpp:47-60)",
               "cases": eg}, open(os.path.join(HERE, "egress_tm_ref.json"), "w"), indent=1)
    print(f"encode {len(out)}, publish {len(pub)}, tm {len(tm)}, ack {len(ack)}, egress {len(eg)}")
    lite = lite_cases()
    json.dump({"source": src + " (CommitOffsetLite / OrderRequestLite / OrderNotificationLite: "
                               "build_commit_offset_message call order src/commit_manager.cpp:114-130 for encode; "
                               "wrapForDecode + topicId + sequence + getXAsString for decode)",
               **lite}, open(os.path.join(HERE, "lite_ref.json"), "w"), indent=1)
    print(f"lite encode {len(lite['encode'])}, lite decode {len(lite['decode'])}")


def lite_encode_inputs():
    """(template, fields, topic_id, sequence) encode cases: typical, empty, non-printable, the
    65534 boundary and E109 on every field."""
    cases = []
    for t in (301, 201, 202):
        nf = T.LITE_NF[t]
        base = [b"msg_1760000000000000000_00042", b"orders:17", b'{"symbol":"BTC-USD","qty":"1"}'][:nf]
        cases.append((t, base, 1, 1))
        cases.append((t, [b""] * nf, 0, 0))
        cases.append((t, [b"\x00\xff\n", b"x", b"\x7f" * 3][:nf], 2**32 - 1, 2**64 - 1))
        cases.append((t, [b"\x41" * 65534] + [b"y"] * (nf - 1), 3, 12345))
        for k in range(nf):
            f = [b"a", b"b", b"c"][:nf]
            f[k] = b"\x5a" * 65535
            cases.append((t, f, 4, 9))
    return cases


def lite_decode_records():
    """Valid Lite records and mutations of them: every truncation length >= 20, blockLength and
    version variants, a corrupted length field, trailing slack."""
    recs = []
    for t in (301, 201, 202):
        nf = T.LITE_NF[t]
        f = [b"m_7", b"orders:3", b'{"q":1}'][:nf]
        rc, r = T.ref_lite_encode(t, f, 7, 0x0102030405060708)
        assert rc == 0
        recs.append((f"t{t}_ok", r))
        recs.append((f"t{t}_slack", r + b"\x00" * 5))
        for cut in range(20, len(r)):
            recs.append((f"t{t}_cut{cut}", r[:cut]))
        for blk in (0, 4, 11, 13, 16, 40):
            recs.append((f"t{t}_blk{blk}", blk.to_bytes(2, "little") + r[2:]))
        recs.append((f"t{t}_ver9", r[:6] + b"\x09\x00" + r[8:]))
        bad = bytearray(r)
        bad[20:22] = (len(r)).to_bytes(2, "little")
        recs.append((f"t{t}_badlen", bytes(bad)))
        empty = T.ref_lite_encode(t, [b""] * nf, 0, 0)[1]
        recs.append((f"t{t}_empty", empty))
    return recs


def lite_cases():
    enc = []
    for t, fields, tid, seq in lite_encode_inputs():
        rc, r = T.ref_lite_encode(t, fields, tid, seq)
        enc.append({"template": t, "fields": [field_spec(x) for x in fields], "topic_id": tid, "sequence": str(seq),
                    "status": rc, "record": blob(r)})
    dec = []
    for name, r in lite_decode_records():
        rc, tid, seq, f = T.ref_lite_decode(r)
        nf = T.LITE_NF[int.from_bytes(r[2:4], "little")]
        dec.append({"name": name, "rec": blob(r), "e100": rc, "topic_id": tid if rc == 0 else None,
                    "sequence": str(seq) if rc == 0 else None,
                    "fields": [blob(x) for x in f[:nf]] if rc == 0 else None})
    return {"encode": enc, "decode": dec}


if __name__ == "__main__":
    main()
