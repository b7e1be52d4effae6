"""Order JSON oracle (Order::to_json, src/order_types.cpp:122-181; publish_order headers JSON,
src/cluster_client.cpp:308-323).

jsoncpp is absent, so the oracle restates its compact StreamWriter (PARITY UNPINNED against
jsoncpp itself).  What pins it here:
  * a hand-derived known answer for one Order (member order = std::map order at every level);
  * Python's json module (sort_keys, compact separators, ensure_ascii: lower-case \\uXXXX and
    surrogate pairs, the escapes jsoncpp uses) as an independent writer of the same object for
    valid UTF-8 strings without DEL, with the two number slots substituted;
  * Python's correctly rounded '%.17g' / '%f' (the glibc semantics jsoncpp valueToString and
    std::to_string rely on) for the number text over edge and random bit-pattern doubles.
"""
import json
import math
import struct

import numpy as np
import pytest

import sbe_testlib as T

F = [b"cli-uuid-1", b"FIXID", b"BTC", b"USDC", b"BUY", b"ord-7", b"msg_1760000000000000000_00042", b"CREATED"]

KNOWN = (b'{"message":{"headers":{"auth_token":"Bearer xxx","connection_uuid":"130032","create_ts":"1760000000123",'
         b'"customer_id":"42","ip_address":"10.37.62.251","origin":"fix","origin_id":"FIXID",'
         b'"origin_name":"FIX_GATEWAY"},"message":{"action":"CREATE","order_details":{"client_order_id":"cli-uuid-1",'
         b'"order_type":"market","quantity":{"token":"BTC","value":0.10000000000000001},"quantity_value_str":"0.100000",'
         b'"side":"BUY","token_pair":{"base_token":"BTC","quote_token":"USDC"}}}},"msg_type":"D","uuid":"cli-uuid-1"}')


def test_known_answer_payload():
    assert T.oracle_order_json_one(F, 42, 1760000000123456789, 0.1) == KNOWN


def test_known_answer_headers():
    assert T.oracle_order_json_one(F, 0, 0, 0.0, 1) == \
        b'{"messageId":"msg_1760000000000000000_00042","messageType":"CREATE_ORDER","orderId":"ord-7"}'
    for st, mt in [(b"UPDATED", b"UPDATE_ORDER"), (b"CANCELLED", b"UPDATE_ORDER"), (b"UPDATE", b"CREATE_ORDER"),
                   (b"CANCELLED\x00", b"CREATE_ORDER")]:
        assert mt in T.oracle_order_json_one(F[:7] + [st], 0, 0, 0.0, 1)


def g17(v):
    if math.isnan(v):
        return "null"
    if math.isinf(v):
        return "-1e+9999" if v < 0 else "1e+9999"
    s = "%.17g" % v
    return s if ("." in s or "e" in s) else s + ".0"


def fixed6(v):
    if math.isnan(v):
        return "-nan" if math.copysign(1.0, v) < 0 else "nan"
    return "%f" % v


def python_writer(f, cid, ts, q):
    """The same object through Python's json module (independent writer)."""
    d = lambda b: b.decode("utf-8")
    obj = {"uuid": d(f[0]), "msg_type": "D", "message": {
        "headers": {"origin": "fix", "origin_name": "FIX_GATEWAY", "origin_id": d(f[1].split(b"\x00")[0]),
                    "connection_uuid": "130032", "customer_id": str(cid),
                    "ip_address": "10.37.62.251", "create_ts": str(_cdiv(ts)),
                    "auth_token": "Bearer xxx"},
        "message": {"action": "CREATE", "order_details": {
            "token_pair": {"base_token": d(f[2]), "quote_token": d(f[3])},
            "quantity": {"token": d(f[2]), "value": "@@Q@@"},
            "side": d(f[4]), "order_type": "market", "quantity_value_str": fixed6(q),
            "client_order_id": d(f[0])}}}}
    s = json.dumps(obj, sort_keys=True, separators=(",", ":"), ensure_ascii=True)
    return s.replace('"@@Q@@"', g17(q)).encode()


def _cdiv(ts):  # C++ int64 division truncates toward zero
    q = abs(ts) // 1000000
    return q if ts >= 0 else -q


@pytest.mark.parametrize("seed", range(6))
def test_python_json_writer_agrees(seed):
    rng = np.random.default_rng(seed)
    pool = ["a", "Z", "0", '"', "\\", "\n", "\t", "\b", "\f", "\r", "\x00", "\x01", "\x1f", " ", "/", "é", "€",
            "😀", "߿", "￿", "\U0010ffff", "~"]
    for _ in range(300):
        f = ["".join(pool[int(rng.integers(0, len(pool)))] for _ in range(int(rng.integers(0, 12)))).encode()
             for _ in range(8)]
        cid = int(rng.integers(-(2 ** 63), 2 ** 63 - 1))
        ts = int(rng.integers(-(2 ** 63), 2 ** 63 - 1))
        q = struct.unpack("<d", struct.pack("<Q", int(rng.integers(0, 2 ** 64, dtype=np.uint64))))[0] \
            if rng.random() < 0.5 else float(rng.choice(T.EDGE_DOUBLES))
        assert T.oracle_order_json_one(f, cid, ts, q) == python_writer(f, cid, ts, q)


def test_number_text_matches_correct_rounding():
    rng = np.random.default_rng(7)
    vals = list(T.EDGE_DOUBLES) + list(rng.integers(0, 2 ** 64, 3000, dtype=np.uint64).view(np.float64)) + \
        list(rng.integers(1, 10 ** 9, 1000) / 2.0 ** rng.integers(0, 40, 1000))
    for v in vals:
        v = float(v)
        out = T.oracle_order_json_one(F, 0, 0, v).decode()
        assert '"value":%s}' % g17(v) in out
        if not math.isnan(v):
            assert '"quantity_value_str":"%s"' % fixed6(v) in out


def test_identifier_cut_at_nul_and_invalid_utf8():
    f = list(F)
    f[1] = b"ab\x00cd"
    f[0] = b"\xff\xc3\xe2\x82\xed\xa0\x80\xf4\x90\x80\x80\x7f"
    out = T.oracle_order_json_one(f, 0, 0, 1.0)
    assert b'"origin_id":"ab"' in out
    # utf8ToCodepoint never checks continuation bytes: FF → U+FFFD (1 byte); C3 E2 → U+00E2;
    # 82 ED → U+00AD; A0 80 → 0 < 0x80, overlong → U+FFFD (2 bytes); F4 90 80 80 → 0x110000,
    # written as the pair (0x100000 >> 10) & 0x3FF = 0 → D800, DC00; DEL passes through
    assert b'"uuid":"\\ufffd\\u00e2\\u00ad\\ufffd\\ud800\\udc00\x7f"}' in out


def test_batch_matches_one_by_one():
    fields, cid, ts, q = T.order_batch(500, 11)
    arena, str_len = T.pack_order_fields(fields)
    for what in (0, 1):
        text, off = T.oracle_order_json(arena, str_len, cid, ts, q, what)
        for i in range(0, 500, 7):
            assert text[int(off[i]):int(off[i + 1])] == T.oracle_order_json_one(fields[i], cid[i], ts[i], q[i], what)
