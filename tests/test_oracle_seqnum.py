"""CPU: the oracle's ParseResult.sequence_number restatement (oracle/sbe_oracle.c orc_seq_eval,
src/sbe_encoder.cpp:1031-1125 over jsoncpp 1.9.5's CharReaderBuilder defaults).

jsoncpp is absent from this image, so this is PARITY UNPINNED against the real library: the hand
cases below spell out jsoncpp 1.9.5's documented/implemented behaviour (OurReader), and the random
cases check the restatement against an independent model built on Python's json module (standard
JSON only) with the same extractSequence and x86-64 double→u64 rules."""
import ctypes
import json
import os
import random
import subprocess

import numpy as np
import pytest

import sbe_testlib as T

U64 = (1 << 64) - 1
MIN64 = 1 << 63


def seq(doc) -> int:
    return T.oracle_seq_eval(doc.encode() if isinstance(doc, str) else doc)


HAND_CASES = [
    ('{"_sequence_number": 42}', 42),
    ('{"_sequence_number": 007}', 7),                     # jsoncpp accepts leading zeros
    ('{"_sequence_number": 0, "message": {"_sequence_number": 7}}', 7),
    ('{"message": {"message": {"_sequence_number": 8}}, "_sequence_number": 0}', 8),
    ('{"message": {"message": {"message": {"_sequence_number": "123"}}}}', 123),
    ('{"message": {"message": {"message": {"message": {"_sequence_number": 5}}}}}', 0),  # depth 4: not looked at
    ('{"message": [{"_sequence_number": 5}]}', 0),
    ('{"x": {"_sequence_number": 5}}', 0),
    ('{"_sequence_number": 3, "message": {"_sequence_number": 9}}', 3),                   # first non-zero wins
    # comments, trailing commas, extra content, BOM, NUL ending the stream
    ('/* c */ {"_sequence_number": 5 // x\n}', 5),
    ('{"_sequence_number": 5 /* c */ , "a": [1, 2,], }', 5),
    ('{"_sequence_number": 5} trailing garbage', 5),
    ('﻿{"_sequence_number": 3}', 3),
    (b'{"_sequence_number": 5}\x00{', 5),
    (b'{"_sequence_number": \x00 5}', 0),
    ('{"_sequence_number": 5', 0),                       # missing '}'
    ('{"_sequence_number": 5,, "a": 1}', 0),
    ('{"_sequence_number" 5}', 0),
    ("{'_sequence_number': 5}", 0),                      # no single quotes
    ('{"_sequence_number": 5} /* unterminated', 5),      # after the root: ignored
    ('{"_sequence_number": 5 /* unterminated', 0),
    ('{"_sequence_number": 5 /*/', 0),
    # numbers
    ('{"_sequence_number": -1}', U64),
    ('{"_sequence_number": -}', 0),
    ('{"_sequence_number": -5, "x": -}', U64 - 4),
    ('{"_sequence_number": 18446744073709551615}', U64),
    ('{"_sequence_number": 18446744073709551616}', 0),   # double 2^64 → cast gives 0
    ('{"_sequence_number": 18446744073709551615.5}', 0),
    ('{"_sequence_number": -9223372036854775808}', MIN64),
    ('{"_sequence_number": -9223372036854775809}', MIN64),
    ('{"_sequence_number": 1.9}', 1),
    ('{"_sequence_number": -1.9}', U64),
    ('{"_sequence_number": 1e3}', 1000),
    ('{"_sequence_number": 1.}', 1),
    ('{"_sequence_number": 1e}', 0),                     # not a number: parse fails
    ('{"_sequence_number": 1e+}', 0),
    ('{"_sequence_number": 1.8446744073709552e19}', 0),
    ('{"_sequence_number": -1e19}', MIN64),
    ('{"_sequence_number": 1e400}', 0),
    ('{"_sequence_number": -1e400}', MIN64),
    ('{"_sequence_number": 9007199254740993.0}', 9007199254740992),   # tie → even
    ('{"_sequence_number": 9007199254740995.0}', 9007199254740996),
    ('{"_sequence_number": 4503599627370495.5}', 4503599627370495),   # representable
    ('{"_sequence_number": 4503599627370496.5}', 4503599627370496),   # q = 1 tie, I even
    ('{"_sequence_number": 4503599627370497.5}', 4503599627370498),   # q = 1 tie, I odd
    ('{"_sequence_number": 0.99999999999999999}', 1),
    ('{"_sequence_number": 0.9999999999999999}', 0),
    ('{"_sequence_number": 7.99999999999999999999e0}', 8),
    ('{"_sequence_number": 123456789012345678901234e-4}', 12345678901234567168),
    ('{"_sequence_number": -0.5}', 0),
    ('{"_sequence_number": -Infinity}', 0),
    ('{"_sequence_number": NaN}', 0),
    ('{"_sequence_number": 0x10}', 0),
    # strings (std::stoull)
    ('{"_sequence_number": " 12"}', 12),
    ('{"_sequence_number": "12abc"}', 12),
    ('{"_sequence_number": "+7"}', 7),
    ('{"_sequence_number": "-1"}', U64),
    ('{"_sequence_number": "- 1"}', 0),
    ('{"_sequence_number": "abc"}', 0),
    ('{"_sequence_number": ""}', 0),
    ('{"_sequence_number": "99999999999999999999"}', 0),
    ('{"_sequence_number": "18446744073709551615"}', U64),
    ('{"_sequence_number": "\\u0031\\u0032"}', 12),
    ('{"_sequence_number": "1\\u00002"}', 1),
    ('{"_sequence_number": "\\t\\n 9"}', 9),
    ('{"_sequence_number": "0x1f"}', 0),
    ('{"_sequence_number": "1\\q"}', 0),                  # bad escape: the parse fails
    # other value types
    ('{"_sequence_number": true}', 0),
    ('{"_sequence_number": null}', 0),
    ('{"_sequence_number": {}}', 0),
    ('{"_sequence_number": [5]}', 0),
    # keys
    ('{"\\u005fsequence_number": 9}', 9),
    ('{"_sequence_numbe\\u0072": 9}', 9),
    ('{"_sequence_number\\u0000": 9}', 0),
    ('{"_sequence_number": 5, "_sequence_number": 6}', 6),
    ('{"_sequence_number": 5, "_sequence_number": "x"}', 0),
    ('{"message": {"_sequence_number": 5}, "message": 1}', 0),
    ('{"message": 1, "message": {"_sequence_number": 5}}', 5),
    ('{"m\\u0065ssage": {"_sequence_number": 4}}', 4),
    # roots
    ('[{"_sequence_number": 5}]', 0),
    ('5', 0),
    ('', 0),
    ('   ', 0),
    ('{}', 0),
]


@pytest.mark.parametrize("doc,exp", HAND_CASES)
def test_hand_cases(doc, exp):
    assert seq(doc) == exp


def test_stack_limit():
    ok = '{"_sequence_number": 1, "a": ' + "[" * 999 + "]" * 999 + "}"
    deep = '{"_sequence_number": 1, "a": ' + "[" * 1000 + "]" * 1000 + "}"
    assert seq(ok) == 1
    assert seq(deep) == 0


def test_surrogates_and_utf8_in_strings():
    assert seq('{"s": "\\ud83d\\ude00", "_sequence_number": 2}') == 2
    assert seq('{"s": "\\ud83d", "_sequence_number": 2}') == 0       # half a pair: error
    assert seq('{"s": "\\ude00", "_sequence_number": 2}') == 2       # lone low surrogate: accepted
    assert seq('{"s": "\\u12", "_sequence_number": 2}') == 0


# ------------------------------------------------------------------------------------------
# independent model over Python's json (standard JSON: the grammar both parsers accept)
# ------------------------------------------------------------------------------------------
def _real_to_u64(tok: str) -> int:
    d = float(tok)  # correctly rounded, like strtod
    if d != d:
        return MIN64
    if d >= 2.0 ** 64:
        return 0
    if d >= 2.0 ** 63:
        return int(d)
    if d < -(2.0 ** 63):
        return MIN64
    return int(d) & U64  # truncation toward zero


def _stoull(s: str) -> int:
    b = s.encode("utf-8", "surrogatepass").split(b"\0")[0]
    i = 0
    while i < len(b) and b[i] in b" \t\n\v\f\r":
        i += 1
    neg = False
    if i < len(b) and b[i] in b"+-":
        neg = b[i] == ord("-")
        i += 1
    j = i
    while j < len(b) and 48 <= b[j] <= 57:
        j += 1
    if j == i:
        return 0
    v = int(b[i:j])
    if v > U64:
        return 0
    return (-v) & U64 if neg else v


class _Num(str):
    pass


def _extract(v) -> int:
    if isinstance(v, bool) or v is None:
        return 0
    if isinstance(v, _Num):
        t = str(v)
        if all(c in "-0123456789" for c in t):
            x = int(t)
            if -(1 << 63) <= x <= U64:
                return x & U64
        return _real_to_u64(t)
    if isinstance(v, str):
        return _stoull(v)
    return 0


def model(doc: str) -> int:
    try:
        root = json.loads(doc, parse_int=_Num, parse_float=_Num, parse_constant=lambda c: 1 / 0)
    except Exception:
        return 0
    if not isinstance(root, dict):
        return 0
    node = root
    for level in range(4):
        if level:
            node = node.get("message")
            if not isinstance(node, dict):
                break
        if "_sequence_number" in node:
            s = _extract(node["_sequence_number"])
            if s:
                return s
    return 0


def _rand_number(r: random.Random) -> str:
    k = r.randrange(8)
    if k == 0:
        return str(r.randrange(0, 1 << 64))
    if k == 1:
        return str(-r.randrange(0, 1 << 63))
    if k == 2:
        return str(r.choice([1 << 64, (1 << 64) - 1, 1 << 63, -(1 << 63), -(1 << 63) - 1, 10 ** 20, -10 ** 19]))
    if k == 3:  # decimals near integers / binade edges
        base = r.choice([0, 1, 2 ** 52, 2 ** 53, 2 ** 63, 2 ** 64, r.randrange(1 << 60)])
        frac = "".join(r.choice("09") for _ in range(r.randrange(1, 30)))
        return f"{'-' if r.random() < 0.3 else ''}{base}.{frac}"
    if k == 4:
        return f"{r.uniform(-1e6, 1e6):.{r.randrange(0, 25)}f}"
    if k == 5:
        m = "".join(r.choice("0123456789") for _ in range(r.randrange(1, 40))).lstrip("0") or "0"
        return f"{m}e{r.randrange(-45, 25)}"  # standard JSON: no leading zeros
    if k == 6:
        return repr(r.uniform(-2e19, 2e19))
    return f"{r.randrange(10 ** 6)}.{r.randrange(10 ** 6)}E+{r.randrange(0, 15)}"


def _rand_value(r: random.Random):
    k = r.randrange(6)
    if k == 0:
        return _Num(_rand_number(r))
    if k == 1:
        return r.choice([" 12", "7x", "-3", "abc", "", "184467440737095516150", "19", "1\u00002"])
    if k == 2:
        return r.choice([True, False, None])
    if k == 3:
        return {"a": 1}
    if k == 4:
        return [1, 2]
    return _Num(str(r.randrange(1, 1 << 32)))


def _dumps(v) -> str:
    if isinstance(v, _Num):
        return str(v)
    if isinstance(v, dict):
        return "{" + ", ".join(json.dumps(k) + ": " + _dumps(x) for k, x in v.items()) + "}"
    if isinstance(v, list):
        return "[" + ", ".join(_dumps(x) for x in v) + "]"
    return json.dumps(v)


def _rand_doc(r: random.Random) -> str:
    def obj(level):
        d = {}
        for _ in range(r.randrange(0, 4)):
            d[r.choice(["qty", "side", "sym", "_seq", "message_"])] = _rand_value(r)
        if r.random() < 0.6:
            d["_sequence_number"] = _rand_value(r)
        if level < 4 and r.random() < 0.6:
            d["message"] = obj(level + 1) if r.random() < 0.85 else _rand_value(r)
        return d
    return _dumps(obj(0))


def test_oracle_matches_json_model():
    r = random.Random(0x5E0)
    for _ in range(4000):
        doc = _rand_doc(r)
        assert seq(doc) == model(doc), doc


def test_numbers_match_strtod_model():
    r = random.Random(0x5E1)
    for _ in range(4000):
        tok = _rand_number(r)
        doc = '{"_sequence_number": ' + tok + "}"
        assert seq(doc) == model(doc), tok


# ------------------------------------------------------------------------------------------
# the device evaluator's logic (csrc/seqnum.hpp, compiled for the host by tests/cpp) against the
# oracle; the GPU tests (test_gpu_seqnum.py) check the kernel itself
# ------------------------------------------------------------------------------------------
_HOSTCHK = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "seqnum_host_check.so")


@pytest.fixture(scope="module")
def dev_logic():
    subprocess.run(["make", "-s", "-C", os.path.dirname(_HOSTCHK), "seqnum_host_check.so"], check=True)
    L = ctypes.CDLL(_HOSTCHK)
    L.seqnum_host_eval.restype = ctypes.c_uint64
    L.seqnum_host_eval.argtypes = [ctypes.c_void_p, ctypes.c_uint32]

    def ev(b: bytes) -> int:
        buf = np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)
        return int(L.seqnum_host_eval(buf.ctypes.data_as(ctypes.c_void_p), len(b)))
    return ev


def _docs(seed, n):
    r = random.Random(seed)
    out = [(d.encode() if isinstance(d, str) else d) for d, _ in HAND_CASES]
    for i in range(n):
        k = i % 5
        if k == 0:
            out.append(_rand_doc(r).encode())
        elif k == 1:
            out.append(b'{"_sequence_number": ' + _rand_number(r).encode() + b"}")
        elif k == 2:  # jsoncpp-only syntax
            d = _rand_doc(r).encode()
            j = r.randrange(len(d) + 1)
            out.append(d[:j] + r.choice([b"/* c */", b"// x\n", b",", b"\\u005f", b"\\", b"\0", b"\xef\xbb\xbf"]) + d[j:])
        elif k == 3:  # byte soup
            out.append(bytes(r.choice(b'q_sequnbr\\"{}[]:,/*\n -+.eE0123456789tfnul') for _ in range(r.randrange(0, 120))))
        else:  # digit-heavy numbers
            m = "".join(r.choice("0123456789") for _ in range(r.randrange(1, 70)))
            f = "".join(r.choice("09") for _ in range(r.randrange(0, 60)))
            e = r.choice(["", f"e{r.randrange(-60, 60)}", f"E+{r.randrange(0, 30)}"])
            s = r.choice(["", "-"])
            out.append(f'{{"_sequence_number": {s}{m}{"." + f if f or r.random() < 0.2 else ""}{e}}}'.encode())
    return out


def test_device_logic_matches_oracle(dev_logic):
    for doc in _docs(0xD0C, 30000):
        assert dev_logic(doc) == T.oracle_seq_eval(doc), doc


def test_device_logic_number_edges(dev_logic):
    """Decimals around every binade edge and integer that the x86 cast can see."""
    r = random.Random(5)
    for p2 in range(0, 65):
        for base in {(1 << p2) - 1, 1 << p2, (1 << p2) + 1}:
            for frac in ("5", "49999999999999999999", "50000000000000000001", "9999999999999999999999",
                         "0000000000000000001", "25", "75", r.choice(["1", "3", "7"]) * r.randrange(1, 40)):
                for sg in ("", "-"):
                    doc = f'{{"_sequence_number": {sg}{base}.{frac}}}'.encode()
                    assert dev_logic(doc) == T.oracle_seq_eval(doc), doc
