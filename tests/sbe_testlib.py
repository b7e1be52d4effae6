"""Test-side helpers: oracle bindings (ctypes over oracle/liboracle.so), seeded record generators,
and the ParseResult / AckInfo / on_egress materialisers that turn device descriptors back into
the reference's result objects (include/aeron_cluster/sbe_messages.hpp:306-328,
include/aeron_cluster/ack_decoder.hpp:9-15, include/aeron_cluster/message_handler.hpp:35-68).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use the oracle.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "aeron-cluster-client-cpp_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")
REF_LIB = os.path.join(ORACLE_DIR, "_ref", "libsbe_ref_fw.so")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

# status / flag constants (include/sbecodec.h)
ENC_REF_TRUNCATE8 = 1
ENC_PUBLISH_TOPIC = 2
ENC_OVERFLOW = 6
DEC_PARSE, DEC_EGRESS, DEC_LITE = 0, 1, 2
ST_LITE, ST_LITE_E100, ST_LITE_NOT_LITE = 48, 49, 50
LITE_NF = {301: 2, 201: 3, 202: 3}
ST_TM, ST_ACK, ST_SESSION_EVENT = 0, 1, 2
ST_ERR_NULL_EMPTY, ST_ERR_HEADER, ST_ERR_UNKNOWN_TYPE = 16, 17, 18
ST_ERR_SESSION_EVENT, ST_ERR_SESSION_SHORT, ST_ERR_EMBEDDED_SHORT = 19, 20, 21
ST_ERR_EMBEDDED_TEMPLATE, ST_ERR_EMBEDDED_SCHEMA, ST_ERR_DIRECT_TEMPLATE = 22, 23, 24
ST_ERR_TM_E100, ST_ERR_ACK_SHORT = 25, 26
ST_EG_ACK_SIMPLE, ST_EG_ACK, ST_EG_TM, ST_EG_NONE, ST_EG_THROW_E100 = 32, 33, 34, 35, 36
FL_ID_DEFAULT, FL_PAYLOAD_DEFAULT, FL_HEADERS_E100, FL_SEQ_KEY, FL_WRAPPED, FL_SEQ_ESC = 1, 2, 4, 8, 16, 32

U64 = np.uint64


# ------------------------------------------------------------------------------------------
# oracle
# ------------------------------------------------------------------------------------------
def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True, stdout=subprocess.DEVNULL)


_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_LIB):
            build_oracle()
        L = ctypes.CDLL(ORACLE_LIB)
        vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        i64 = ctypes.c_int64
        L.orc_encode_batch.argtypes = [vp, vp, vp, vp, u64, u64, u32, vp, vp, vp, i]
        L.orc_encode_session_batch.argtypes = [vp, vp, vp, vp, u64, u64, u32, i64, i64, vp, vp, vp, i]
        L.orc_encode_lite_batch.argtypes = [vp, vp, vp, vp, vp, u64, u32, vp, vp, vp, i]
        L.orc_reassemble.argtypes = [vp, vp, vp, u64, vp, vp, vp, vp]
        L.orc_decode_batch.argtypes = [vp, vp, u64, u32, vp, vp, vp, vp, vp, vp, i]
        L.orc_seq_eval.restype = u64
        L.orc_seq_eval.argtypes = [vp, u64]
        L.orc_seq_batch.argtypes = [vp, vp, u64, vp, vp, vp, vp, vp, i]
        L.orc_order_json_one.restype = u64
        L.orc_order_json_one.argtypes = [vp, vp, i64, i64, ctypes.c_double, u32, vp]
        L.orc_order_json_batch.argtypes = [vp, vp, vp, vp, vp, vp, u64, u32, vp, vp, i]
        L.orc_to_nanos_auto.restype = u64
        L.orc_to_nanos_auto.argtypes = [u64]
        _oracle = L
    return _oracle


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def oracle_encode(arena, str_len, ts, str_off=None, flags=0, ts_default=0, nthreads=1):
    """arena uint8[], str_len uint32[n,5], ts uint64[n] → (out bytes, out_off uint64[n+1], status)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    str_len = np.ascontiguousarray(str_len, dtype=np.uint32).reshape(-1, 5)
    ts = np.ascontiguousarray(ts, dtype=np.uint64)
    n = ts.size
    if str_off is not None:
        str_off = np.ascontiguousarray(str_off, dtype=np.uint32).reshape(-1, 5)
    cap = int(str_len.sum(dtype=np.uint64)) + 34 * n + 16
    out = np.zeros(cap, dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    oracle().orc_encode_batch(_p(arena if arena.size else np.zeros(1, np.uint8)), _p(str_off), _p(str_len),
                              _p(ts), n, ts_default, flags, _p(out), _p(out_off), _p(status), nthreads)
    return out[: int(out_off[n])], out_off, status[:n]


def oracle_encode_session(arena, str_len, ts, term_id, session_id, str_off=None, flags=0, ts_default=0,
                          nthreads=1):
    """Session-framed TopicMessages (32-B SessionMessageHeader + record) → (out, out_off, status)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    str_len = np.ascontiguousarray(str_len, dtype=np.uint32).reshape(-1, 5)
    ts = np.ascontiguousarray(ts, dtype=np.uint64)
    n = ts.size
    if str_off is not None:
        str_off = np.ascontiguousarray(str_off, dtype=np.uint32).reshape(-1, 5)
    cap = int(str_len.sum(dtype=np.uint64)) + 66 * n + 16
    out = np.zeros(cap, dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    oracle().orc_encode_session_batch(_p(arena if arena.size else np.zeros(1, np.uint8)), _p(str_off), _p(str_len),
                                      _p(ts), n, ts_default, flags, term_id, session_id, _p(out), _p(out_off),
                                      _p(status), nthreads)
    return out[: int(out_off[n])], out_off, status[:n]


def oracle_encode_lite(template_id, arena, str_len, topic_id, sequence, str_off=None, nthreads=1):
    """Lite records (201 / 202 / 301): str_len uint32[n, nf] → (out, out_off, status)."""
    nf = LITE_NF[template_id]
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    str_len = np.ascontiguousarray(str_len, dtype=np.uint32).reshape(-1, nf)
    topic_id = np.ascontiguousarray(topic_id, dtype=np.uint32)
    sequence = np.ascontiguousarray(sequence, dtype=np.uint64)
    n = sequence.size
    if str_off is not None:
        str_off = np.ascontiguousarray(str_off, dtype=np.uint32).reshape(-1, nf)
    cap = int(str_len.sum(dtype=np.uint64)) + (20 + 2 * nf) * n + 16
    out = np.zeros(cap, dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    rc = oracle().orc_encode_lite_batch(_p(arena if arena.size else np.zeros(1, np.uint8)), _p(str_off),
                                        _p(str_len), _p(topic_id if n else np.zeros(1, np.uint32)),
                                        _p(sequence if n else np.zeros(1, np.uint64)), n, template_id,
                                        _p(out), _p(out_off), _p(status), nthreads)
    assert rc == 0
    return out[: int(out_off[n])], out_off, status[:n]


def oracle_reassemble(data, frag_off, flags):
    """LocalFragmentReassembler restated → (messages list of bytes, carry bytes)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    frag_off = np.ascontiguousarray(frag_off, dtype=np.uint64)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    n = flags.size
    tot = max(int(frag_off[-1]) if n else 0, 1)
    out = np.zeros(tot, np.uint8)
    acc = np.zeros(tot, np.uint8)
    msg_off = np.zeros(n + 1, np.uint64)
    counts = np.zeros(2, np.uint64)
    oracle().orc_reassemble(_p(data if data.size else np.zeros(1, np.uint8)), _p(frag_off),
                            _p(flags if n else np.zeros(1, np.uint8)), n, _p(out), _p(msg_off), _p(counts), _p(acc))
    m = int(counts[0])
    msgs = [bytes(out[int(msg_off[j]):int(msg_off[j + 1])]) for j in range(m)]
    carry = bytes(out[int(msg_off[m]):int(msg_off[m]) + int(counts[1])])
    return msgs, carry


def fragment_stream(n, seed, p_single=0.6, maxlen=300, p_group=None, p_inner=0.1):
    """Random Aeron fragment stream: lengths 0..maxlen, flags drawn from whole messages
    (BEGIN|END, probability p_single), BEGIN … END sequences of 2-5 fragments (p_group, default
    0.9 - p_single; a middle fragment is a whole message with probability p_inner), and stray
    middle / END / BEGIN fragments (the rest)."""
    rng = np.random.default_rng(seed)
    flags = np.zeros(n, np.uint8)
    p_grp_end = p_single + (0.9 - p_single if p_group is None else p_group)
    i = 0
    while i < n:
        r = rng.random()
        if r < p_single:
            flags[i] = 0xC0
            i += 1
        elif r < p_grp_end:
            k = int(rng.integers(2, 6))
            for t in range(k):
                if i >= n:
                    break
                flags[i] = 0x80 if t == 0 else (0x40 if t == k - 1 else 0x00)
                if 0 < t < k - 1 and rng.random() < p_inner:
                    flags[i] = 0xC0  # a whole message inside a group
                i += 1
        else:
            flags[i] = int(rng.choice([0x00, 0x40, 0x80]))
            i += 1
    lens = rng.integers(0, maxlen + 1, n)
    lens[rng.random(n) < 0.05] = 0
    frag_off = np.zeros(n + 1, np.uint64)
    frag_off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, int(frag_off[-1]), dtype=np.uint8)
    return data, frag_off, flags


def oracle_decode(data, rec_off, mode=DEC_PARSE, nthreads=1):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    n = rec_off.size - 1
    m = max(n, 1)
    d = dict(status=np.zeros(m, np.uint8), flags=np.zeros(m, np.uint8), hdr=np.zeros((m, 4), np.uint16),
             ts=np.zeros(m, np.uint64), view_off=np.zeros((m, 5), np.uint32), view_len=np.zeros((m, 5), np.uint32))
    buf = data if data.size else np.zeros(1, np.uint8)
    oracle().orc_decode_batch(_p(buf), _p(rec_off), n, mode, _p(d["status"]), _p(d["flags"]), _p(d["hdr"]),
                              _p(d["ts"]), _p(d["view_off"]), _p(d["view_len"]), nthreads)
    return {k: v[:n] for k, v in d.items()}


def oracle_seq_eval(payload: bytes) -> int:
    """ParseResult.sequence_number of one payload (oracle restatement of jsoncpp 1.9.5; unpinned)."""
    buf = np.frombuffer(payload, np.uint8) if payload else np.zeros(1, np.uint8)
    return int(oracle().orc_seq_eval(_p(np.ascontiguousarray(buf)), len(payload)))


def oracle_seq_batch(data, rec_off, dec, nthreads=1):
    """sbe_eval_sequence_numbers over the oracle's parse-mode descriptors; unwritten slots stay 0."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    n = rec_off.size - 1
    seq = np.zeros(max(n, 1), np.uint64)
    buf = data if data.size else np.zeros(1, np.uint8)
    oracle().orc_seq_batch(_p(buf), _p(rec_off), n, _p(np.ascontiguousarray(dec["status"])),
                           _p(np.ascontiguousarray(dec["flags"])), _p(np.ascontiguousarray(dec["view_off"])),
                           _p(np.ascontiguousarray(dec["view_len"])), _p(seq), nthreads)
    return seq[:n]


# ------------------------------------------------------------------------------------------
# reference flyweight harness (oracle/_ref, only where /root/reference was present to build it)
# ------------------------------------------------------------------------------------------
_ref = None


def ref_available():
    return os.path.exists(REF_LIB)


def ref():
    global _ref
    if _ref is None:
        L = ctypes.CDLL(REF_LIB)
        vp, u64, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.ref_tm_encode.argtypes = [vp, vp, u64, i, vp, u64, vp]
        L.ref_tm_decode_parse.argtypes = [vp, u64, vp, vp, vp, vp, vp]
        L.ref_ack_decode.argtypes = [vp, u64, vp, vp, vp]
        L.ref_egress_tm.argtypes = [vp, u64, vp, vp]
        L.ref_lite_encode.argtypes = [ctypes.c_uint32, vp, vp, ctypes.c_uint32, u64, vp, u64, vp]
        L.ref_lite_decode.argtypes = [vp, u64, vp, vp, vp, vp]
        L.ref_publish_topic.argtypes = [vp, vp, u64, vp, u64, vp]
        L.ref_tm_encode_batch.argtypes = [vp, vp, vp, u64, i, vp, vp, vp, i]
        _ref = L
    return _ref


def ref_encode_batch(arena, str_len, ts, wire=False, nthreads=1):
    """The reference's own flyweight sequence of SBEEncoder::encode_topic_message
    (src/sbe_encoder.cpp:141-164) over a packed batch (oracle/_ref, ref_tm_encode_batch), OpenMP
    over nthreads.  Returns (out bytes, out_off)."""
    run, out, out_off = ref_encode_prepared(arena, str_len, ts, wire)
    run(nthreads)
    return out[: int(out_off[-1])], out_off


def ref_encode_prepared(arena, str_len, ts, wire=False):
    """ref_encode_batch with its arrays made once: returns (run(nthreads), out, out_off), run()
    encoding the batch into out again (timing loops)."""
    L = np.ascontiguousarray(str_len, dtype=np.uint32).reshape(-1, 5)
    n = L.shape[0]
    sizes = L.sum(axis=1, dtype=np.uint64)
    in_off = np.zeros(n + 1, np.uint64)
    np.cumsum(sizes, out=in_off[1:])
    out_off = np.zeros(n + 1, np.uint64)
    np.cumsum(sizes + (34 if wire else 26), out=out_off[1:])
    out = np.zeros(int(out_off[-1]) + 16, np.uint8)
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    ts = np.ascontiguousarray(ts, dtype=np.uint64)
    lib = ref()

    def run(nthreads):
        bad = lib.ref_tm_encode_batch(arena.ctypes.data, L.ctypes.data, ts.ctypes.data, n, 1 if wire else 0,
                                      out.ctypes.data, out_off.ctypes.data, in_off.ctypes.data, int(nthreads))
        if bad:
            raise RuntimeError(f"reference encode failed on {bad} records")

    return run, out, out_off


def ref_encode(fields, ts, wire):
    bufs = [ctypes.create_string_buffer(bytes(f), max(len(f), 1)) for f in fields]
    ptrs = (ctypes.c_void_p * 5)(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_uint32 * 5)(*[len(f) for f in fields])
    cap = 34 + sum(len(f) for f in fields) + 16
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_uint64(0)
    rc = ref().ref_tm_encode(ptrs, lens, ts, 1 if wire else 0, out, cap, ctypes.byref(n))
    return rc, out.raw[: n.value]


def ref_publish(fields, ts):
    """ClusterClient::publish_topic's encoder block (src/cluster_client.cpp:1823-1858) through the
    reference flyweights: fields are (topic, type, uuid, payload, headers) as publish_topic passes
    them to put*(const char*, int)."""
    bufs = [ctypes.create_string_buffer(bytes(f), max(len(f), 1)) for f in fields]
    ptrs = (ctypes.c_void_p * 5)(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_uint32 * 5)(*[len(f) for f in fields])
    cap = 34 + sum(len(f) for f in fields) + 16
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_uint64(0)
    rc = ref().ref_publish_topic(ptrs, lens, ts, out, cap, ctypes.byref(n))
    return rc, out.raw[: n.value]


def ref_lite_encode(template_id, fields, topic_id, sequence):
    nf = LITE_NF[template_id]
    assert len(fields) == nf
    bufs = [ctypes.create_string_buffer(bytes(f), max(len(f), 1)) for f in fields]
    ptrs = (ctypes.c_void_p * nf)(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_uint32 * nf)(*[len(f) for f in fields])
    cap = 20 + 2 * nf + sum(len(f) for f in fields) + 16
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_uint64(0)
    rc = ref().ref_lite_encode(template_id, ptrs, lens, topic_id, sequence, out, cap, ctypes.byref(n))
    return rc, out.raw[: n.value]


def ref_lite_decode(rec: bytes):
    """(rc, topic_id, sequence, fields): rc 0 ok, 1 E100 (header must name a Lite template)."""
    b = _rec_buf(rec)
    tid, seq = ctypes.c_uint32(), ctypes.c_uint64()
    flen = (ctypes.c_uint32 * 3)()
    fbuf = ctypes.create_string_buffer(len(rec) * 3 + 16)
    rc = ref().ref_lite_decode(b, len(rec), ctypes.byref(tid), ctypes.byref(seq), flen, fbuf)
    return rc, tid.value, seq.value, _split(fbuf.raw, flen, 3)


def _rec_buf(rec: bytes):
    # the reference reads only inside the record when it succeeds, but its getXAsString builds
    # the string before the bounds check (TopicMessage.h:539-541): pad the harness input so
    # those discarded reads stay inside our allocation.
    return ctypes.create_string_buffer(bytes(rec) + b"\0" * 65600, len(rec) + 65600)


def ref_tm_decode(rec: bytes):
    b = _rec_buf(rec)
    ts, seq = ctypes.c_uint64(), ctypes.c_uint64()
    flen = (ctypes.c_uint32 * 5)()
    fbuf = ctypes.create_string_buffer(len(rec) * 5 + 16)
    hok = ctypes.c_int(0)
    rc = ref().ref_tm_decode_parse(b, len(rec), ctypes.byref(ts), ctypes.byref(seq), flen, fbuf, ctypes.byref(hok))
    return rc, ts.value, _split(fbuf.raw, flen, 5), hok.value


def ref_ack_decode(rec: bytes):
    b = _rec_buf(rec)
    ts = ctypes.c_uint64()
    flen = (ctypes.c_uint32 * 3)()
    fbuf = ctypes.create_string_buffer(len(rec) * 3 + 16)
    rc = ref().ref_ack_decode(b, len(rec), ctypes.byref(ts), flen, fbuf)
    return rc, ts.value, _split(fbuf.raw, flen, 3)


def ref_egress_tm(rec: bytes):
    b = _rec_buf(rec)
    flen = (ctypes.c_uint32 * 5)()
    fbuf = ctypes.create_string_buffer(len(rec) * 5 + 16)
    rc = ref().ref_egress_tm(b, len(rec), flen, fbuf)
    return rc, _split(fbuf.raw, flen, 5)


def _split(raw, flen, k):
    out, at = [], 0
    for i in range(k):
        out.append(raw[at: at + flen[i]])
        at += flen[i]
    return out


# ------------------------------------------------------------------------------------------
# materialisers: descriptor → reference result objects
# ------------------------------------------------------------------------------------------
def _i64(u):
    u = int(u) & (2**64 - 1)
    return u - 2**64 if u >= 2**63 else u


def _view(rec, d, k):
    o, n = int(d["view_off"][k]), int(d["view_len"][k])
    return bytes(rec[o: o + n])


def materialize_parse(rec: bytes, d) -> dict:
    """ParseResult (sbe_messages.hpp:306-328) from one record's descriptor d (dict of scalars/rows)."""
    r = dict(success=False, error_message=b"", message_type=b"", message_id=b"", payload=b"", headers=b"",
             timestamp=0, sequence_number=0, template_id=0, schema_id=0, version=0, block_length=0,
             correlation_id=0, session_id=0, leader_member_id=0, event_code=0, leadership_term_id=0)
    st, fl = int(d["status"]), int(d["flags"])
    hdr = [int(x) for x in d["hdr"]]
    param = int(d["view_off"][0])

    def take_hdr():
        r.update(block_length=hdr[0], template_id=hdr[1], schema_id=hdr[2], version=hdr[3])

    if st == ST_TM:
        r.update(success=True, message_type=_view(rec, d, 1), message_id=_view(rec, d, 2),
                 payload=_view(rec, d, 3), headers=_view(rec, d, 4), timestamp=_i64(d["ts"]))
        take_hdr()
    elif st == ST_ACK:
        ts = int(d["ts"])
        r.update(success=True, message_type=b"Acknowledgment", timestamp=_i64(ts),
                 message_id=(b"ack_" + str(ts).encode()) if fl & FL_ID_DEFAULT else _view(rec, d, 0),
                 payload=b"SUCCESS" if fl & FL_PAYLOAD_DEFAULT else _view(rec, d, 1),
                 headers=_view(rec, d, 2))
        take_hdr()
    elif st == ST_SESSION_EVENT:
        q = lambda o, f: struct.unpack_from(f, rec, o)[0]  # noqa: E731
        r.update(success=True, message_type=b"SessionEvent", correlation_id=q(8, "<q"), session_id=q(16, "<q"),
                 leadership_term_id=q(24, "<q"), leader_member_id=q(32, "<i"), event_code=q(36, "<i"),
                 payload=_view(rec, d, 3), timestamp=0)
        take_hdr()
    else:
        msg = {
            ST_ERR_NULL_EMPTY: b"Null or empty data",
            ST_ERR_HEADER: b"Failed to decode message header",
            ST_ERR_UNKNOWN_TYPE: b"Unknown message type: template=%d, schema=%d" % (hdr[1], hdr[2]),
            ST_ERR_SESSION_EVENT: b"Failed to decode SessionEvent",
            ST_ERR_SESSION_SHORT: b"Session message too short to contain embedded message",
            ST_ERR_EMBEDDED_SHORT: b"Embedded message too short",
            ST_ERR_EMBEDDED_TEMPLATE: b"Unknown embedded message template_id: %d" % param,
            ST_ERR_EMBEDDED_SCHEMA: b"Unknown embedded message schema_id: %d" % param,
            ST_ERR_DIRECT_TEMPLATE: b"Unknown direct message template_id: %d" % param,
            ST_ERR_TM_E100: b"SBE TopicMessage decoding failed: buffer too short [E100]",
            ST_ERR_ACK_SHORT: b"Buffer too short for Acknowledgment message. Need at least 16 bytes, got %d" % param,
        }[st]
        r["error_message"] = msg
        if st == ST_ERR_UNKNOWN_TYPE:
            take_hdr()
    return r


def materialize_egress(rec: bytes, d):
    """Outcome of MessageHandler::on_egress: ('ack', AckInfo dict) | ('tm', 5 fields) | ('none',) |
    ('throw', b'buffer too short [E100]')."""
    st = int(d["status"])
    if st == ST_EG_ACK_SIMPLE:
        return ("ack", dict(timestamp_nanos=int(d["ts"]), message_id=b"", topic=b"", correlation_id=b"",
                            simple_control_ack=True))
    if st == ST_EG_ACK:
        return ("ack", dict(timestamp_nanos=int(d["ts"]), message_id=_view(rec, d, 0), topic=_view(rec, d, 1),
                            correlation_id=_view(rec, d, 2), simple_control_ack=False))
    if st == ST_EG_TM:
        return ("tm", tuple(_view(rec, d, k) for k in range(5)))
    if st == ST_EG_THROW_E100:
        return ("throw", b"buffer too short [E100]")
    assert st == ST_EG_NONE, st
    return ("none",)


def row(dec, i):
    return {k: v[i] for k, v in dec.items()}


# ------------------------------------------------------------------------------------------
# wire builders (tests construct records the way the server / reference would)
# ------------------------------------------------------------------------------------------
def hdr_bytes(blk, tmpl, schema, ver):
    return struct.pack("<HHHH", blk, tmpl, schema, ver)


def tm_wire(fields, ts, blk=16, ver=1, seq=0):
    b = hdr_bytes(blk, 1, 1, ver) + struct.pack("<QQ", ts & (2**64 - 1), seq)
    for f in fields:
        b += struct.pack("<H", len(f)) + bytes(f)
    return b


def ack_wire(msg_id, topic, corr, ts, blk=8, ver=1):
    b = hdr_bytes(blk, 2, 1, ver) + struct.pack("<Q", ts)
    for f in (msg_id, topic, corr):
        b += struct.pack("<H", len(f)) + bytes(f)
    return b


def simple_ack(ts, ver=1):
    return hdr_bytes(8, 2, 1, ver) + struct.pack("<Q", ts)


def session_wrap(rec, term=7, session=9, blk=24):
    return hdr_bytes(blk, 1, 111, 8) + struct.pack("<qqq", term, session, 0) + b"\0" * max(0, blk - 24) + rec


def session_event(corr, sess, term, leader, code, detail=b"", blk=32):
    b = hdr_bytes(blk, 2, 111, 8) + struct.pack("<qqqii", corr, sess, term, leader, code)
    if detail is not None:
        b += struct.pack("<I", len(detail)) + detail
    return b


def pack_records(recs):
    off = np.zeros(len(recs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in recs], dtype=np.uint64) if recs else []
    data = np.frombuffer(b"".join(bytes(r) for r in recs), dtype=np.uint8).copy() if recs else np.zeros(0, np.uint8)
    return data, off


# ------------------------------------------------------------------------------------------
# seeded synthetic workloads; splitmix64 so every component sees the same bytes
# ------------------------------------------------------------------------------------------
def splitmix64(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = (U64(seed) + U64(0x9E3779B97F4A7C15) * (np.arange(1, n + 1, dtype=U64)))
        z = x
        z = (z ^ (z >> U64(30))) * U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> U64(27))) * U64(0x94D049BB133111EB)
        return z ^ (z >> U64(31))


def _digits(v: np.ndarray, width: int) -> np.ndarray:
    """uint64[n] → uint8[n,width] zero-padded decimal of v mod 10**width."""
    v = v.copy()
    out = np.empty((v.size, width), dtype=np.uint8)
    for k in range(width - 1, -1, -1):
        out[:, k] = (v % U64(10)).astype(np.uint8) + ord("0")
        v //= U64(10)
    return out


# payload template (143 B) and headers template (32 B): fixed-256 Order records
_PAYLOAD_T = (b'{"side":"BUY","symbol":"BTC-USD","qty":"#########","price":"#########.##",'
              b'"client_order_id":"cid_#################","type":"LIMIT","tif":"GTC"}')
_HEADERS_T = b'{"messageType":"CREATE_ORDER"}  '


def fixed256_orders(n: int, seed: int = 0x5EED0002):
    """topic "orders", type "CREATE_ORDER", uuid msg_<19d>_<5d>,
    payload 143 B, headers 32 B: Σlen = 222, wire record 256 B.  Packed SoA."""
    assert len(_PAYLOAD_T) == 143 and len(_HEADERS_T) == 32, (len(_PAYLOAD_T), len(_HEADERS_T))
    r = splitmix64(seed, 4 * n).reshape(n, 4)
    ts = (U64(1_760_000_000_000_000_000) + np.arange(n, dtype=U64))
    uuid = np.empty((n, 29), np.uint8)
    uuid[:, :4] = np.frombuffer(b"msg_", np.uint8)
    uuid[:, 4:23] = _digits(ts, 19)
    uuid[:, 23] = ord("_")
    uuid[:, 24:29] = _digits(r[:, 0], 5)
    pay = np.tile(np.frombuffer(_PAYLOAD_T, np.uint8), (n, 1))
    hol = [i for i, c in enumerate(_PAYLOAD_T) if c == ord("#")]
    qty, price, cid = hol[:9], hol[9:20], hol[20:]
    pay[:, qty] = _digits(r[:, 1], 9)
    pay[:, price] = _digits(r[:, 2], 11)
    pay[:, cid] = _digits(r[:, 3], 17)
    rec = np.concatenate([np.tile(np.frombuffer(b"orders", np.uint8), (n, 1)),
                          np.tile(np.frombuffer(b"CREATE_ORDER", np.uint8), (n, 1)),
                          uuid, pay, np.tile(np.frombuffer(_HEADERS_T, np.uint8), (n, 1))], axis=1)
    str_len = np.tile(np.array([6, 12, 29, 143, 32], np.uint32), (n, 1))
    return rec.reshape(-1), str_len, ts


CONFIG5_RECORDS = 134_217_728  # 128 M fixed-256 records (32 GiB encoded)
CONFIG5_SEED = 0x5EED0005


def _h31(i, k: int, seed: int):
    """31-bit hash of record index i (int64 tensor) and field k, in int64 arithmetic that never
    overflows (products of < 2^31 values by < 2^31 constants)."""
    import torch
    m = 0x7FFFFFFF
    x = (i * 0x9E3779B1 + (k + 1) * 0x85EBCA77 + seed) & m
    x = ((x ^ (x >> 15)) * 0x2C1B3C6D) & m
    x = ((x ^ (x >> 12)) * 0x297A2D39) & m
    return x ^ (x >> 15)


def _digits_t(v, width: int):
    import torch
    p = torch.tensor([10 ** (width - 1 - k) for k in range(width)], dtype=torch.int64, device=v.device)
    return ((v[:, None] // p[None, :]) % 10 + 48).to(torch.uint8)


def config5_shard(lo: int, hi: int, device, seed: int = CONFIG5_SEED, chunk: int = 1 << 22):
    """Records [lo, hi) of the config-5 batch, generated on `device` (torch ops, chunked): the
    config-2 record shape (topic "orders", type "CREATE_ORDER", uuid msg_<19d ts>_<5d>, the
    143-B order payload with qty / price / client_order_id digits, 32-B headers; Σlen = 222, wire
    record 256 B), every byte a function of the GLOBAL record index, so any split into shards
    concatenates to the same batch.  Returns packed SoA (arena uint8 [222 m], str_len int32 [m,5],
    timestamp int64 [m])."""
    import torch
    m = hi - lo
    arena = torch.empty((m, 222), dtype=torch.uint8, device=device)
    tmpl = np.concatenate([np.frombuffer(b"orders", np.uint8), np.frombuffer(b"CREATE_ORDER", np.uint8),
                           np.frombuffer(b"msg_" + b"0" * 19 + b"_" + b"0" * 5, np.uint8),
                           np.frombuffer(_PAYLOAD_T, np.uint8), np.frombuffer(_HEADERS_T, np.uint8)])
    tmpl_t = torch.from_numpy(tmpl.copy()).to(device)
    hol = [47 + i for i, c in enumerate(_PAYLOAD_T) if c == ord("#")]
    qty, price, cid = hol[:9], hol[9:20], hol[20:]
    ts = torch.arange(lo, hi, dtype=torch.int64, device=device) + 1_760_000_000_000_000_000
    for a in range(0, m, chunk):
        b = min(m, a + chunk)
        i = torch.arange(lo + a, lo + b, dtype=torch.int64, device=device)
        blk = arena[a:b]
        blk.copy_(tmpl_t.expand(b - a, 222))
        blk[:, 22:41] = _digits_t(ts[a:b], 19)
        blk[:, 42:47] = _digits_t(_h31(i, 0, seed) % 100_000, 5)
        blk[:, qty[0]:qty[-1] + 1] = _digits_t(_h31(i, 1, seed) % 1_000_000_000, 9)
        pv = (_h31(i, 2, seed) * 37 + _h31(i, 3, seed)) % 100_000_000_000
        pd = _digits_t(pv, 11)
        blk[:, price[0]:price[8] + 1] = pd[:, :9]
        blk[:, price[9]:price[10] + 1] = pd[:, 9:]
        blk[:, cid[0]:cid[-1] + 1] = _digits_t((_h31(i, 4, seed) * 0x80000000 + _h31(i, 5, seed)) % 10 ** 17, 17)
    L = torch.tensor([6, 12, 29, 143, 32], dtype=torch.int32, device=device).expand(m, 5).contiguous()
    return arena.reshape(-1), L, ts


_TOPICS = [b"orders", b"order_request_topic", b"order_notification_topic"]
_TYPES = [b"CREATE_ORDER", b"UPDATE_ORDER"]


# printable filler byte for each random byte: (b % 94) + 32, with "_" → "-" (keeps
# "_sequence_number" out of synthetic payloads) and "\\" → "/" (JSON order payloads carry no escapes)
_FILL_LUT = (np.arange(256) % 94 + 32).astype(np.uint8)
_FILL_LUT[_FILL_LUT == ord("_")] = ord("-")
_FILL_LUT[_FILL_LUT == ord("\\")] = ord("/")


def var_orders(n: int, seed: int = 0x5EED0004):
    """SURVEY §8(d) config 4 (variable length): topic ∈ 3 names, type ∈ 2, uuid 29 B, payload
    uniform [32,480] with a 3–10 B symbol, headers uniform [16,64].  Packed SoA."""
    r = splitmix64(seed, 6 * n).reshape(n, 6)
    ti = (r[:, 0] % U64(3)).astype(np.int64)
    yi = (r[:, 1] % U64(2)).astype(np.int64)
    plen = (U64(32) + r[:, 2] % U64(449)).astype(np.int64)
    hlen = (U64(16) + r[:, 3] % U64(49)).astype(np.int64)
    slen = (U64(3) + r[:, 4] % U64(8)).astype(np.int64)
    tlen = np.array([len(t) for t in _TOPICS])[ti]
    ylen = np.array([len(t) for t in _TYPES])[yi]
    str_len = np.stack([tlen, ylen, np.full(n, 29), plen, hlen], axis=1).astype(np.uint32)
    ts = (U64(1_760_000_000_000_000_000) + np.arange(n, dtype=U64))
    tot = str_len.astype(np.int64).sum(1)
    starts = np.zeros(n + 1, np.int64)
    starts[1:] = np.cumsum(tot)
    arena = np.empty(int(starts[-1]), np.uint8)
    # fill with printable filler derived from the random stream, then lay the fixed pieces
    fill = splitmix64(seed ^ 0xABCDEF, (arena.size + 7) // 8).view(np.uint8)[: arena.size]
    arena[:] = _FILL_LUT[fill]
    base = starts[:-1]
    for k, t in enumerate(_TOPICS):
        idx = base[ti == k]
        arena[idx[:, None] + np.arange(len(t))] = np.frombuffer(t, np.uint8)
    tb = base + tlen
    for k, t in enumerate(_TYPES):
        idx = tb[yi == k]
        arena[idx[:, None] + np.arange(len(t))] = np.frombuffer(t, np.uint8)
    ub = tb + ylen
    arena[ub[:, None] + np.arange(4)] = np.frombuffer(b"msg_", np.uint8)
    arena[ub[:, None] + 4 + np.arange(19)] = _digits(ts, 19)
    arena[ub + 23] = ord("-")
    arena[ub[:, None] + 24 + np.arange(5)] = _digits(r[:, 5], 5)
    pb = ub + 29
    arena[pb[:, None] + np.arange(10)] = np.frombuffer(b'{"symbol":', np.uint8)
    return arena, str_len, ts


def vt_mixed(n: int, pattern: str, seed: int = 21):
    """Batches the pack kernel runs on its virtual-tile loop (first superblock averages ~265 B
    records, so a 32-record tile's output ends just past one 8 KiB window) with the records that change
    window arithmetic mixed in: E109 records (no output bytes), 65534-byte and 70000-byte fields,
    empty records, timestamp 0.  pattern: "sprinkled" (1% edge records at random), "zero_run" (a
    run of 700 E109/empty records in the second superblock: tiles with no output), "long_run" (16
    records of ~64 KB in a row, each spanning several windows)."""
    rng = np.random.default_rng(seed)
    L = np.zeros((n, 5), np.uint32)
    L[:, 0] = rng.integers(3, 12, n)
    L[:, 1] = rng.integers(8, 14, n)
    L[:, 2] = 29
    L[:, 3] = rng.integers(140, 171, n)
    L[:, 4] = rng.integers(20, 40, n)
    edges = np.array([[65535, 0, 0, 0, 0], [0, 0, 0, 65535, 0], [0, 0, 0, 0, 0], [65534, 3, 29, 1, 0],
                      [70000, 1, 1, 1, 1], [1, 2, 3, 4, 5], [0, 0, 0, 65534, 65534]], np.uint32)
    if pattern == "sprinkled":
        idx = rng.choice(n, n // 100, replace=False)
        L[idx] = edges[rng.integers(0, len(edges), idx.size)]
    elif pattern == "zero_run":
        lo = 4096 + 300
        L[lo: lo + 700] = np.where((np.arange(700) % 3 == 0)[:, None], edges[2], edges[0])
    elif pattern == "long_run":
        lo = 4096 + 1000
        L[lo: lo + 16, 3] = 65534
        L[lo: lo + 16, 4] = rng.integers(0, 65535, 16)
    else:
        raise ValueError(pattern)
    arena = rng.integers(0, 256, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    ts = rng.integers(1, 2**63, n, dtype=np.uint64)
    ts[::11] = 0
    return arena, L, ts


def _s64(c: int) -> int:
    return c - (1 << 64) if c >= 1 << 63 else c


def _lsr(z, k: int):
    """logical right shift of an int64 tensor holding uint64 bits"""
    return (z >> k) & ((1 << (64 - k)) - 1)


def _umod(z, m: int):
    """uint64 value of int64 tensor z, mod m (m < 2^31)"""
    return ((_lsr(z, 1) % m) * 2 + (z & 1)) % m


def _splitmix64_t(seed: int, lo: int, count: int, device):
    """splitmix64(seed, .)[lo:lo+count] as int64 tensors (two's-complement wrap == uint64 math)."""
    import torch
    z = torch.arange(lo + 1, lo + 1 + count, dtype=torch.int64, device=device)
    z = z * _s64(0x9E3779B97F4A7C15) + _s64(seed & ((1 << 64) - 1))
    z = (z ^ _lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _lsr(z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _lsr(z, 31)


def var_orders_t(n: int, device, seed: int = 0x5EED0004, chunk: int = 1 << 22):
    """var_orders(n, seed) generated with torch ops on `device` (chunked), byte-identical to the
    numpy generator (the 16 M-record config-4 batch takes ~1.5 min on the host in numpy).  Returns
    (arena uint8 [Σlen], str_len int32 [n,5], ts int64 [n])."""
    import torch
    r = _splitmix64_t(seed, 0, 6 * n, device).view(n, 6)
    ti, yi = _umod(r[:, 0], 3), _umod(r[:, 1], 2)
    plen, hlen = 32 + _umod(r[:, 2], 449), 16 + _umod(r[:, 3], 49)
    tl = torch.tensor([len(t) for t in _TOPICS], dtype=torch.int64, device=device)[ti]
    yl = torch.tensor([len(t) for t in _TYPES], dtype=torch.int64, device=device)[yi]
    str_len = torch.stack([tl, yl, torch.full_like(tl, 29), plen, hlen], dim=1)
    ts = torch.arange(n, dtype=torch.int64, device=device) + 1_760_000_000_000_000_000
    base = torch.cumsum(str_len.sum(1), 0) - str_len.sum(1)
    total = int(str_len.sum())
    arena = torch.empty(total, dtype=torch.uint8, device=device)
    lut = torch.from_numpy(_FILL_LUT).to(device)
    words = (total + 7) // 8
    for a in range(0, words, 8 * chunk):
        b = min(words, a + 8 * chunk)
        f = _splitmix64_t(seed ^ 0xABCDEF, a, b - a, device).view(torch.uint8)
        e = min(total, 8 * b)
        arena[8 * a:e] = lut[f[: e - 8 * a].to(torch.int64)]
    del r
    u8 = lambda bs: torch.tensor(list(bs), dtype=torch.uint8, device=device)  # noqa: E731
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        bb, tib, yib = base[a:b], ti[a:b], yi[a:b]
        for k, t in enumerate(_TOPICS):
            idx = bb[tib == k]
            arena[(idx[:, None] + torch.arange(len(t), device=device)).reshape(-1)] = u8(t).repeat(idx.numel())
        tb = bb + tl[a:b]
        for k, t in enumerate(_TYPES):
            idx = tb[yib == k]
            arena[(idx[:, None] + torch.arange(len(t), device=device)).reshape(-1)] = u8(t).repeat(idx.numel())
        ub = tb + yl[a:b]
        m = b - a
        uu = torch.empty((m, 29), dtype=torch.uint8, device=device)
        uu[:, :4] = u8(b"msg_")
        uu[:, 4:23] = _digits_t(ts[a:b], 19)
        uu[:, 23] = ord("-")
        r5 = _splitmix64_t(seed, 6 * a, 6 * m, device).view(m, 6)[:, 5]
        uu[:, 24:29] = _digits_t(_umod(r5, 100_000), 5)
        arena[(ub[:, None] + torch.arange(29, device=device)).reshape(-1)] = uu.reshape(-1)
        pb = ub + 29
        arena[(pb[:, None] + torch.arange(10, device=device)).reshape(-1)] = u8(b'{"symbol":').repeat(m)
    return arena, str_len.to(torch.int32), ts


def lite_records(n: int, template_id: int, seed: int = 0x5EED0301):
    """Lite records in packed SoA form: 301 CommitOffsetLite (messageId = uuid 29 B,
    messageIdentifier 8–40 B); 201 / 202 (uuid 29 B, messageIdentifier 8–40 B, payload 32–480 B).
    Returns (arena, str_len [n, nf], topic_id [n], sequence [n])."""
    nf = LITE_NF[template_id]
    r = splitmix64(seed ^ template_id, 4 * n).reshape(n, 4)
    lens = [np.full(n, 29, np.int64), (U64(8) + r[:, 0] % U64(33)).astype(np.int64)]
    if nf == 3:
        lens.append((U64(32) + r[:, 1] % U64(449)).astype(np.int64))
    str_len = np.stack(lens, axis=1).astype(np.uint32)
    tot = str_len.astype(np.int64).sum(1)
    starts = np.zeros(n + 1, np.int64)
    starts[1:] = np.cumsum(tot)
    fill = splitmix64(seed ^ 0x5151, (int(starts[-1]) + 7) // 8 + 1).view(np.uint8)[: int(starts[-1])]
    arena = ((fill % 94) + 32).astype(np.uint8)
    seq = U64(1_000_000) + np.arange(n, dtype=U64)
    ub = starts[:-1]
    arena[ub[:, None] + np.arange(4)] = np.frombuffer(b"msg_", np.uint8)
    arena[ub[:, None] + 4 + np.arange(19)] = _digits(U64(1_760_000_000_000_000_000) + np.arange(n, dtype=U64), 19)
    topic_id = (U64(1) + r[:, 2] % U64(3)).astype(np.uint32)
    return arena, str_len, topic_id, seq


def mixed_records(n: int, seed: int = 0x5EED0003):
    """69 % TM-256, 15 % Ack-73 (exact), 15 % Ack-81 (+8 B slack),
    1 % simple 16-B ack, randomly interleaved; returns (data, rec_off)."""
    arena, str_len, ts = fixed256_orders(n, seed)
    recs_tm = arena.reshape(n, 222)
    kind = (splitmix64(seed ^ 0x77, n) % U64(100)).astype(np.int64)
    kind = np.where(kind < 69, 0, np.where(kind < 84, 1, np.where(kind < 99, 2, 3)))
    sizes = np.array([256, 73, 81, 16])[kind]
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    data = np.zeros(int(off[-1]), np.uint8)
    ts_ms = U64(1_760_000_000_000) + np.arange(n, dtype=U64)
    tsb = ts.view(np.uint8).reshape(n, 8)
    tsm = ts_ms.view(np.uint8).reshape(n, 8)
    # TopicMessage
    i = np.nonzero(kind == 0)[0]
    b = off[i]
    data[b[:, None] + np.arange(8)] = np.frombuffer(hdr_bytes(16, 1, 1, 1), np.uint8)
    data[b[:, None] + 8 + np.arange(8)] = tsb[i]
    pos = 24
    col = 0
    for L in (6, 12, 29, 143, 32):
        data[b[:, None] + pos + np.arange(2)] = np.frombuffer(struct.pack("<H", L), np.uint8)
        data[b[:, None] + pos + 2 + np.arange(L)] = recs_tm[i, col: col + L]
        pos += 2 + L
        col += L
    # full acks (exact and +8 slack): messageId = uuid (29), topic "orders", corr 16 digits
    for k in (1, 2):
        i = np.nonzero(kind == k)[0]
        b = off[i]
        data[b[:, None] + np.arange(8)] = np.frombuffer(hdr_bytes(8, 2, 1, 1), np.uint8)
        data[b[:, None] + 8 + np.arange(8)] = tsm[i]
        data[b[:, None] + 16 + np.arange(2)] = np.frombuffer(struct.pack("<H", 29), np.uint8)
        data[b[:, None] + 18 + np.arange(29)] = recs_tm[i, 18:47]
        data[b[:, None] + 47 + np.arange(2)] = np.frombuffer(struct.pack("<H", 6), np.uint8)
        data[b[:, None] + 49 + np.arange(6)] = np.frombuffer(b"orders", np.uint8)
        data[b[:, None] + 55 + np.arange(2)] = np.frombuffer(struct.pack("<H", 16), np.uint8)
        data[b[:, None] + 57 + np.arange(16)] = recs_tm[i, 18 + 4: 18 + 20]
    i = np.nonzero(kind == 3)[0]
    b = off[i]
    data[b[:, None] + np.arange(8)] = np.frombuffer(hdr_bytes(8, 2, 1, 1), np.uint8)
    data[b[:, None] + 8 + np.arange(8)] = tsm[i]
    return data, off.astype(np.uint64)


# ------------------------------------------------------------------------------------------
# edge-case records (decode): every status of both modes, ragged lengths, all prefixes
# ------------------------------------------------------------------------------------------
def edge_records():
    """[(name, bytes)] covering the reference's branches."""
    f5 = [b"orders", b"CREATE_ORDER", b"msg_1", b'{"a":1}', b'{"h":2}']
    tm = tm_wire(f5, 0x1122334455667788)
    ack = ack_wire(b"msg_42", b"orders", b"corr-1", 1_700_000_000_000)
    out = [
        ("tm_wire", tm),
        ("tm_ref_trunc", tm[:-8]),
        ("tm_slack8", tm + b"\0" * 8),
        ("tm_slack3", tm + b"\0" * 3),
        ("tm_slack8_empty_type", tm_wire([b"t", b"", b"u", b"p", b"h"], 4) + b"\0" * 8),
        ("tm_slack8_blk0", tm_wire(f5, 5, blk=0) + b"\0" * 8),
        ("tm_cut_in_payload", tm[:50]),
        ("tm_blk8", tm_wire(f5, 5, blk=8)),
        ("tm_blk0", tm_wire(f5, 5, blk=0)),
        ("tm_blk40", tm_wire(f5, 5, blk=40)),
        ("tm_blk_huge", tm_wire(f5, 5, blk=60000)),
        ("tm_all_empty", tm_wire([b""] * 5, 9)),
        ("tm_empty_topic", tm_wire([b"", b"T", b"u", b"p", b"h"], 9)),
        ("tm_empty_headers", tm_wire(f5[:4] + [b""], 9)),
        ("tm_seq_key", tm_wire(f5[:3] + [b'{"_sequence_number":17}', b"{}"], 3)),
        ("tm_seq_key_nested", tm_wire(f5[:3] + [b'{"message":{"_sequence_number":"4"}}', b"{}"], 3)),
        ("tm_ver7", tm_wire(f5, 1, ver=7)),
        ("tm_nonprintable", tm_wire([b"\x00\x01", b"\xff" * 3, b"\x7f", b"\x80abc", b"\n"], 2**64 - 1)),
        ("wrapped_tm", session_wrap(tm)),
        ("wrapped_tm_blk32", session_wrap(tm, blk=32)),
        ("wrapped_ack", session_wrap(ack)),
        ("wrapped_simple_ack", session_wrap(simple_ack(1000))),
        ("wrapped_short_ack", session_wrap(simple_ack(1000)[:12])),
        ("wrapped_only_header", session_wrap(b"")),
        ("wrapped_emb_short", session_wrap(b"\x01\x02\x03")),
        ("wrapped_emb_tmpl9", session_wrap(hdr_bytes(16, 9, 1, 1) + b"x" * 20)),
        ("wrapped_emb_schema5", session_wrap(hdr_bytes(16, 1, 5, 1) + b"x" * 20)),
        ("wrapped_tm_trunc", session_wrap(tm[:-8])),
        ("wrapped_tm_cut", session_wrap(tm[:40])),
        ("unknown_tmpl9", hdr_bytes(16, 9, 1, 1) + b"\0" * 30),
        ("unknown_schema7", hdr_bytes(16, 1, 7, 1) + b"\0" * 30),
        ("unknown_111_tmpl5", hdr_bytes(16, 5, 111, 8) + b"\0" * 30),
        ("simple_ack_ms", simple_ack(1_000_000_000_000)),
        ("simple_ack_ns", simple_ack(1_760_000_000_123_456_789)),
        ("simple_ack_blk16", hdr_bytes(16, 2, 1, 1) + struct.pack("<Q", 12345)),
        ("ack_exact", ack),
        ("ack_slack8", ack + b"\0" * 8),
        ("ack_slack7", ack + b"\0" * 7),
        ("ack_zero_msgid", ack_wire(b"", b"orders", b"corr-1", 77) + b"\0" * 8),
        ("ack_zero_topic", ack_wire(b"m1", b"", b"corr-1", 77) + b"\0" * 8),
        ("ack_glue", ack_wire(b"A" * 0x41, b"orders", b"B" * 0x2041, 123) + b"\0" * 8),
        ("ack_no_runs", hdr_bytes(8, 2, 1, 1) + struct.pack("<Q", 5) + bytes([1, 2, 0, 200, 31, 127, 10])),
        ("ack_runs_2char", hdr_bytes(8, 2, 1, 1) + struct.pack("<Q", 5) + b"ab\0cd\0xyz"),
        ("ack_4runs", hdr_bytes(8, 2, 1, 1) + struct.pack("<Q", 6) + b"one\0two\0three\0four"),
        ("ack_blk0", ack_wire(b"id", b"t", b"c", 8, blk=0) + b"\0" * 8),
        ("ack_blk40", ack_wire(b"id", b"t", b"c", 8, blk=40) + b"\0" * 60),
        ("ack_len8", hdr_bytes(8, 2, 1, 1)),
        ("ack_len15", hdr_bytes(8, 2, 1, 1) + b"1234567"),
        ("session_event_min", session_event(1, 2, 3, 4, 0, detail=None)),
        ("session_event_detail", session_event(-1, 2**40, 3, 1, 2, detail=b"redirect:host:1234")),
        ("session_event_detail_empty", session_event(1, 2, 3, 4, 1, detail=b"")),
        ("session_event_detail_long", session_event(1, 2, 3, 4, 1, detail=b"abc")[:-1]),
        ("session_event_short", session_event(1, 2, 3, 4, 0, detail=None)[:39]),
        ("session_event_3b_tail", session_event(1, 2, 3, 4, 0, detail=None) + b"\x01\x00\x00"),
        ("empty", b""),
    ]
    for k in range(1, 8):
        out.append((f"len{k}", tm[:k]))
    for k in range(0, len(tm) + 1, 3):
        out.append((f"tm_prefix{k}", tm[:k]))
    w = session_wrap(tm)
    for k in range(30, len(w) + 1, 5):
        out.append((f"wrapped_prefix{k}", w[:k]))
    for k in range(8, len(ack) + 9):
        out.append((f"ack_prefix{k}", (ack + b"\0" * 8)[:k]))
    rng = np.random.default_rng(1234)
    for k in range(40):
        hdrs = [(16, 1, 1, 1), (8, 2, 1, 1), (24, 1, 111, 8), (32, 2, 111, 8), (0, 1, 1, 0), (200, 1, 1, 1)]
        h = hdrs[k % len(hdrs)]
        body = rng.integers(0, 256, size=int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        if k % 3 == 0:  # mostly-printable bodies with small length prefixes
            body = bytes((b % 6) if i % 9 == 0 else (32 + b % 95) for i, b in enumerate(body))
        out.append((f"random{k}", hdr_bytes(*h) + body))
    return out


# ------------------------------------------------------------------------------------------
# Order JSON (Order::to_json, publish_order headers)
# ------------------------------------------------------------------------------------------
ORDER_FIELDS = 8  # client_order_uuid, identifier, base_token, quote_token, side, id, message_id, status


def oracle_order_json_one(fields, customer_id, timestamp, quantity, what=0) -> bytes:
    bufs = [ctypes.create_string_buffer(bytes(f), max(len(f), 1)) for f in fields]
    ptrs = (ctypes.c_void_p * 8)(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
    lens = (ctypes.c_uint32 * 8)(*[len(f) for f in fields])
    L = oracle()
    n = L.orc_order_json_one(ptrs, lens, int(customer_id), int(timestamp), float(quantity), what, None)
    out = ctypes.create_string_buffer(max(n, 1))
    L.orc_order_json_one(ptrs, lens, int(customer_id), int(timestamp), float(quantity), what, out)
    return out.raw[:n]


def oracle_order_json(arena, str_len, customer_id, timestamp, quantity, what=0, str_off=None, nthreads=1):
    """Batch Order JSON over host arrays → (text bytes, out_off uint64[n+1])."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    str_len = np.ascontiguousarray(str_len, dtype=np.uint32).reshape(-1, 8)
    customer_id = np.ascontiguousarray(customer_id, dtype=np.int64)
    timestamp = np.ascontiguousarray(timestamp, dtype=np.int64)
    quantity = np.ascontiguousarray(quantity, dtype=np.float64)
    n = customer_id.size
    if str_off is not None:
        str_off = np.ascontiguousarray(str_off, dtype=np.uint32).reshape(-1, 8)
    cap = 700 * n + 12 * int(str_len.sum(dtype=np.uint64)) + 16
    out = np.zeros(cap, dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    oracle().orc_order_json_batch(_p(arena if arena.size else np.zeros(1, np.uint8)), _p(str_off), _p(str_len),
                                  _p(customer_id), _p(timestamp), _p(quantity), n, what, _p(out), _p(out_off),
                                  nthreads)
    return out[: int(out_off[n])].tobytes(), out_off


EDGE_DOUBLES = [0.0, -0.0, 1.0, -1.0, 0.1, 0.5, 1.5, 100.0, 1e16, 1e17, 123456789012345680.0, 2.0 ** 60,
                1 + 2.0 ** -17, 0.0078125, 9.9999995, 0.0000005, 1e-5, 1e-4, 9.99999999999999e-5, 1e21, 1e22,
                5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, 0.30000000000000004, 999999.9999995,
                123.456, 2.5, 0.125, 1e-300, 3.0e100, float("inf"), float("-inf"), float("nan"), -float("nan"),
                9007199254740993.0, 4503599627370495.5, 0.000001, 0.0000015, 99999999999999999.0, 1e15 + 0.3]


def order_batch(n: int, seed: int, hard: bool = True):
    """Seeded Orders: (fields [n][8] list of bytes, customer_id, timestamp, quantity).  With hard,
    strings carry quotes, backslashes, controls, NULs, UTF-8 (valid and not) and doubles span the
    whole binary range."""
    rng = np.random.default_rng(seed)
    alpha = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
    specials = [b'"', b"\\", b"\n", b"\t", b"\x00", b"\x01", b"\x1f", b"\x7f", b"\xc3\xa9", b"\xe2\x82\xac",
                b"\xf0\x9f\x98\x80", b"\xff", b"\xc3", b"\xe2\x82", b"\xed\xa0\x80", b"\xc0\xaf", b"\xf8", b"/",
                b"\xf4\x90\x80\x80", b"\x80"]

    def rstr(lo, hi):
        k = int(rng.integers(lo, hi + 1))
        b = bytearray(rng.choice(np.frombuffer(alpha, np.uint8), k).tobytes())
        if hard and k and rng.random() < 0.3:
            for _ in range(int(rng.integers(1, 4))):
                at = int(rng.integers(0, len(b) + 1))
                b[at:at] = specials[int(rng.integers(0, len(specials)))]
        return bytes(b)

    statuses = [b"CREATED", b"UPDATED", b"CANCELLED", b"UPDATE", b"", b"CANCELLED\x00"]
    fields = []
    for _ in range(n):
        fields.append([rstr(0, 40), rstr(0, 12), rstr(0, 6), rstr(0, 6), rstr(0, 5), rstr(0, 20), rstr(0, 30),
                       statuses[int(rng.integers(0, len(statuses)))]])
    customer_id = rng.integers(-(2 ** 63), 2 ** 63 - 1, n, dtype=np.int64, endpoint=True)
    timestamp = rng.integers(-(2 ** 63), 2 ** 63 - 1, n, dtype=np.int64, endpoint=True)
    small = rng.random(n) < 0.5
    customer_id[small] = rng.integers(0, 10 ** 6, int(small.sum()))
    timestamp[small] = 1_760_000_000_000_000_000 + rng.integers(0, 10 ** 12, int(small.sum()))
    kind = rng.integers(0, 4, n)
    q = np.empty(n, dtype=np.float64)
    # prices / quantities with few decimals, random bit patterns, edge values, round-ish values
    k0 = int((kind == 0).sum())
    scale = 10.0 ** rng.integers(0, 9, k0)
    q[kind == 0] = np.round(rng.random(k0) * 10.0 ** rng.integers(0, 7, k0) * scale) / scale
    q[kind == 1] = rng.integers(0, 2 ** 64, int((kind == 1).sum()), dtype=np.uint64).view(np.float64)
    q[kind == 2] = np.array(EDGE_DOUBLES)[rng.integers(0, len(EDGE_DOUBLES), int((kind == 2).sum()))]
    q[kind == 3] = rng.integers(1, 10 ** 9, int((kind == 3).sum())) / 2.0 ** rng.integers(0, 30, int((kind == 3).sum()))
    if not hard:
        q = np.abs(np.nan_to_num(q, nan=1.0, posinf=1.0, neginf=1.0))
    return fields, customer_id, timestamp, q


def pack_order_fields(fields):
    """[n][8] bytes → (packed arena uint8, str_len uint32[n,8])."""
    flat = [f for rec in fields for f in rec]
    arena = np.frombuffer(b"".join(flat), dtype=np.uint8) if flat else np.zeros(0, np.uint8)
    str_len = np.array([len(f) for f in flat], dtype=np.uint32).reshape(-1, 8)
    return arena, str_len


def realistic_orders(n: int, seed: int = 0x5EED00F3):
    """Order-shaped batch for the bench row: uuid 36 B, identifier 8 B, BTC/USDC-like tokens,
    BUY/SELL, id 20 B, message id 29 B, status; quantities with <= 4 decimals below 1e4."""
    rng = np.random.default_rng(seed)
    hexd = np.frombuffer(b"0123456789abcdef", np.uint8)
    uu = rng.choice(hexd, (n, 36))
    uu[:, [8, 13, 18, 23]] = ord("-")
    ident = rng.choice(np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ", np.uint8), (n, 8))
    oid = rng.choice(hexd, (n, 20))
    mid = np.concatenate([np.tile(np.frombuffer(b"msg_", np.uint8), (n, 1)),
                          (48 + rng.integers(0, 10, (n, 19))).astype(np.uint8),
                          np.full((n, 1), ord("_"), np.uint8), (48 + rng.integers(0, 10, (n, 5))).astype(np.uint8)], 1)
    bases, quotes, sides = [b"BTC", b"ETH", b"SOL"], [b"USDC", b"USDT"], [b"BUY", b"SELL"]
    bi, qi, si = rng.integers(0, 3, n), rng.integers(0, 2, n), rng.integers(0, 2, n)
    fields = [[uu[i].tobytes(), ident[i].tobytes(), bases[bi[i]], quotes[qi[i]], sides[si[i]], oid[i].tobytes(),
               mid[i].tobytes(), b"CREATED"] for i in range(n)]
    cid = rng.integers(1, 10 ** 7, n).astype(np.int64)
    ts = (1_760_000_000_000_000_000 + rng.integers(0, 10 ** 12, n)).astype(np.int64)
    q = np.round(rng.random(n) * 10 ** 4, 4)
    return fields, cid, ts, q


def oracle_materialize(data, rec_off, dec):
    """MATERIALIZE's expected output from oracle descriptors (oracle_decode): every record's five
    views data[rec_off[i] + view_off[i][k] :][: view_len[i][k]] back to back in record / view
    order (what the reference's ParseResult strings hold, include/aeron_cluster/sbe_messages.hpp:
    306-328), and arena_off [5n+1] (the last entry the total)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    rec_off = np.asarray(rec_off, dtype=np.uint64)
    n = rec_off.size - 1
    vl = dec["view_len"][:n].astype(np.uint64).reshape(-1)
    vo = dec["view_off"][:n].astype(np.uint64).reshape(-1)
    off = np.zeros(5 * n + 1, np.uint64)
    off[1:] = np.cumsum(vl)
    src = np.repeat(rec_off[:n], 5) + vo
    total = int(off[-1])
    if total == 0:
        return np.zeros(0, np.uint8), off
    # byte j of the arena comes from src[v] + (j - off[v]) for the view v holding it
    v = np.repeat(np.arange(5 * n), vl.astype(np.int64))
    j = np.arange(total, dtype=np.uint64)
    return data[(src[v] + j - off[:-1][v]).astype(np.int64)], off
