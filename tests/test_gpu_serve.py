"""GPU parity of the small-batch serve kernel (sbe_server_* / sbecodec.Server): the resident wave
must return exactly what the batch entry points return for the same inputs, checked against the
oracle (encode: bytes, offsets, status; decode: every descriptor array and sequence numbers),
across record shapes that take each path of the shared device code (single window, records
longer than a window, E109, PUBLISH_TOPIC wrap, edge records at every alignment), plus the
server's own behaviour: argument errors, idle exit and relaunch, interleaving with batch calls.
"""
import time

import numpy as np
import pytest
import torch

import sbe_testlib as T
from test_gpu_parity import assert_same_decode, to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def server(codec):
    s = codec.Server()
    yield s
    s.close()


def host(enc, n):
    off = enc.out_off.cpu().numpy().view(np.uint64)
    return enc.out[: int(off[n])].cpu().numpy(), off, enc.status.cpu().numpy()


def check_same(got, exp):
    go, goff, gst = got
    eo, eoff, est = exp
    np.testing.assert_array_equal(goff, eoff)
    np.testing.assert_array_equal(gst, est)
    np.testing.assert_array_equal(go, eo)


def tm_inputs(arena, L, ts):
    a = to_dev(arena if arena.size else np.zeros(16, np.uint8), torch.uint8)
    return a, to_dev(np.asarray(L, np.uint32).reshape(-1, 5), torch.int32), to_dev(np.asarray(ts, np.uint64), torch.int64)


def long_records(n, seed):
    """Payloads up to 40 KB (records longer than the pack and decode windows) among short ones."""
    rng = np.random.default_rng(seed)
    L = np.stack([rng.integers(0, 20, n), rng.integers(0, 14, n), np.full(n, 29),
                  np.where(rng.random(n) < 0.3, rng.integers(9000, 40000, n), rng.integers(0, 500, n)),
                  rng.integers(0, 64, n)], 1).astype(np.uint32)
    arena = rng.integers(32, 127, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    ts = rng.integers(0, 2**63, n, dtype=np.uint64)
    return arena, L, ts


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8, T.ENC_PUBLISH_TOPIC])
@pytest.mark.parametrize("n", [1, 2, 31, 32, 33, 100, 1000])
def test_serve_encode_topic_fixed(codec, server, n, flags):
    arena, L, ts = T.fixed256_orders(n)
    got = host(server.encode_topic(*tm_inputs(arena, L, ts), flags=flags), n)
    check_same(got, T.oracle_encode(arena, L, ts, flags=flags))


@pytest.mark.parametrize("n", [1, 7, 64, 513])
def test_serve_encode_topic_var(codec, server, n):
    arena, L, ts = T.var_orders(n, seed=0x5E + n)
    got = host(server.encode_topic(*tm_inputs(arena, L, ts), ts_default=77), n)
    check_same(got, T.oracle_encode(arena, L, ts, ts_default=77))


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
def test_serve_encode_long_and_e109(codec, server, flags):
    arena, L, ts = long_records(90, 5)
    L[3, 3] = 70000  # E109 on payload (a 65535-B field is the first failing length)
    L[10, 0] = 65535
    arena = np.concatenate([arena, np.full(70000 + 65535, 65, np.uint8)])
    got = host(server.encode_topic(*tm_inputs(arena, L, ts), flags=flags), 90)
    exp = T.oracle_encode(arena, L, ts, flags=flags)
    assert exp[2][3] != 0 and exp[2][10] != 0
    check_same(got, exp)


def test_serve_encode_publish_wrap(codec, server):
    rng = np.random.default_rng(21)
    L = np.array([[3, 4, 29, 65536 + 17, 2], [0, 0, 0, 0, 0], [70000, 1, 2, 3, 4]], np.uint32)
    arena = rng.integers(0, 256, int(L.sum(dtype=np.int64)), dtype=np.uint8)
    ts = np.array([1, 2, 3], np.uint64)
    got = host(server.encode_topic(*tm_inputs(arena, L, ts), flags=T.ENC_PUBLISH_TOPIC), 3)
    check_same(got, T.oracle_encode(arena, L, ts, flags=T.ENC_PUBLISH_TOPIC))


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8])
@pytest.mark.parametrize("n", [1, 64, 300])
def test_serve_encode_session(codec, server, n, flags):
    arena, L, ts = T.var_orders(n, seed=0x77 + n)
    got = host(server.encode_session(*tm_inputs(arena, L, ts), -3, 1 << 40, flags=flags), n)
    check_same(got, T.oracle_encode_session(arena, L, ts, -3, 1 << 40, flags=flags))


@pytest.mark.parametrize("template_id", [301, 201, 202])
@pytest.mark.parametrize("n", [1, 65, 700])
def test_serve_encode_lite(codec, server, template_id, n):
    arena, L, tid, seq = T.lite_records(n, template_id)
    got = server.encode_lite(template_id, to_dev(arena, torch.uint8), to_dev(L, torch.int32),
                             to_dev(tid, torch.int32), to_dev(seq, torch.int64))
    check_same(host(got, n), T.oracle_encode_lite(template_id, arena, L, tid, seq))


def test_serve_encode_empty(codec, server):
    e = np.zeros(0, np.uint8)
    got = server.encode_topic(*tm_inputs(e, np.zeros((0, 5), np.uint32), np.zeros(0, np.uint64)))
    assert got.out_off.cpu().tolist() == [0]


def serve_decode(server, data, off, mode, seq=None):
    d = to_dev(data if data.size else np.zeros(16, np.uint8), torch.uint8)
    r = to_dev(np.asarray(off, np.uint64), torch.int64)
    dec = server.decode(d, r, mode=mode, seq=seq)
    return dec


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS, T.DEC_LITE])
def test_serve_decode_edges_every_alignment(codec, server, mode):
    recs = [r for _, r in T.edge_records()]
    for lead in range(16):
        data, off = T.pack_records([b"\0" * lead] + recs)
        assert_same_decode(serve_decode(server, data, off, mode).numpy(), T.oracle_decode(data, off, mode))


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS])
@pytest.mark.parametrize("n", [1, 2, 64, 65, 1000, 4096])
def test_serve_decode_mixed(codec, server, mode, n):
    data, off = T.mixed_records(n, seed=0x31 + n)
    assert_same_decode(serve_decode(server, data, off, mode).numpy(), T.oracle_decode(data, off, mode))


def test_serve_decode_long_records(codec, server):
    arena, L, ts = long_records(150, 9)
    out, off, _ = T.oracle_encode(arena, L, ts)
    for mode in (T.DEC_PARSE, T.DEC_EGRESS):
        assert_same_decode(serve_decode(server, out, off, mode).numpy(), T.oracle_decode(out, off, mode))


def test_serve_decode_lite(codec, server):
    arena, L, tid, seq = T.lite_records(300, 201)
    out, off, _ = T.oracle_encode_lite(201, arena, L, tid, seq)
    assert_same_decode(serve_decode(server, out, off, T.DEC_LITE).numpy(), T.oracle_decode(out, off, T.DEC_LITE))


def test_serve_decode_sequence_numbers(codec, server):
    key = b"_sequence_number"
    recs = [T.tm_wire([b"t", b"y", b"u", b'{"' + key + b'":%d}' % (i * 977 + 1), b"{}"], i) for i in range(40)]
    recs += [T.tm_wire([b"t", b"y", b"u", b'{"message":{"' + key + b'":"12"}}', b"{}"], 5)]
    data, off = T.pack_records(recs)
    dec = serve_decode(server, data, off, T.DEC_PARSE, seq=True)
    exp = T.oracle_decode(data, off, T.DEC_PARSE)
    assert_same_decode(dec.numpy(), exp)
    seq = dec.seq.cpu().numpy().view(np.uint64)
    assert seq[:40].tolist() == [i * 977 + 1 for i in range(40)] and int(seq[40]) == 12


def test_serve_matches_batch_path(codec, server):
    """Same inputs through the batch kernels and the server, interleaved in one process."""
    arena, L, ts = T.var_orders(800, seed=99)
    a, Ld, t = tm_inputs(arena, L, ts)
    for _ in range(3):
        b = codec.encode_topic_batch(a, Ld, t)
        torch.cuda.synchronize()
        s = server.encode_topic(a, Ld, t)
        check_same(host(s, 800), host(b, 800))
        bo = b.out_off.cpu().numpy().view(np.uint64)
        d_b = codec.decode_batch(b.out, b.out_off, mode=T.DEC_PARSE)
        torch.cuda.synchronize()
        d_s = server.decode(b.out, b.out_off, mode=T.DEC_PARSE)
        assert_same_decode(d_s.numpy(), d_b.numpy())
        assert int(bo[-1]) > 0


def test_serve_argument_errors(codec, server):
    arena, L, ts = T.fixed256_orders(4)
    a, Ld, t = tm_inputs(arena, L, ts)
    with pytest.raises(codec.SbeError):
        server.encode_topic(a, Ld, t, flags=T.ENC_PUBLISH_TOPIC | T.ENC_REF_TRUNCATE8)
    with pytest.raises(codec.SbeError):
        server.encode_session(a, Ld, t, 1, 2, flags=T.ENC_PUBLISH_TOPIC)
    big = codec.SERVE_MAX_RECORDS + 1
    arena, L, ts = T.fixed256_orders(big)
    with pytest.raises(codec.SbeError):
        server.encode_topic(*tm_inputs(arena, L, ts))
    data, off = T.mixed_records(big)
    with pytest.raises(codec.SbeError):
        serve_decode(server, data, off, T.DEC_PARSE)
    with pytest.raises(codec.SbeError):
        serve_decode(server, data[:64], np.array([1, 17], np.uint64), T.DEC_PARSE + 7)
    # still serving after the refusals
    arena, L, ts = T.fixed256_orders(3)
    check_same(host(server.encode_topic(*tm_inputs(arena, L, ts)), 3), T.oracle_encode(arena, L, ts))


def test_serve_idle_exit_and_relaunch(codec):
    s = codec.Server(idle_us=2000)
    try:
        arena, L, ts = T.fixed256_orders(5)
        exp = T.oracle_encode(arena, L, ts)
        for k in range(4):
            check_same(host(s.encode_topic(*tm_inputs(arena, L, ts)), 5), exp)
            time.sleep(0.03)  # past the idle time: the kernel exits, the next request relaunches it
        req, launches = s.stats()
        assert req == 4 and launches >= 2
    finally:
        s.close()
    # back-to-back requests (well inside a 20 ms idle time) reuse the running kernel
    s = codec.Server(idle_us=20000)
    try:
        a, Ld, t = tm_inputs(arena, L, ts)
        for k in range(20):
            check_same(host(s.encode_topic(a, Ld, t), 5), exp)
        req, launches = s.stats()
        assert req == 20 and launches <= 3
    finally:
        s.close()


def test_device_sync_after_a_served_call(codec):
    """A resident server holds up device-wide synchronisation until it goes idle (sbecodec.h,
    sbe_server_quiesce): torch.cuda.synchronize() after a served call returns within the idle time,
    and at once after quiesce(), which leaves the server usable (the next request relaunches it)."""
    arena, L, ts = T.fixed256_orders(5)
    exp = T.oracle_encode(arena, L, ts)
    idle_s = 0.05
    s = codec.Server(idle_us=int(idle_s * 1e6))
    try:
        a, Ld, t = tm_inputs(arena, L, ts)
        s.encode_topic(a, Ld, t)
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        waited = time.perf_counter() - t0
        assert waited < idle_s + 0.5, waited  # bounded by the idle exit (plus scheduling slack)
        got = s.encode_topic(a, Ld, t)
        s.quiesce()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        after_quiesce = time.perf_counter() - t0
        assert after_quiesce < idle_s / 2, after_quiesce  # the kernel has already left
        check_same(host(got, 5), exp)
        check_same(host(s.encode_topic(a, Ld, t), 5), exp)  # relaunched by the next request
        req, launches = s.stats()
        assert req == 3 + 1 and launches >= 2  # the quiesce's shutdown counts as a request
        print(f"device sync after a served call: {waited * 1e3:.2f} ms (idle {idle_s * 1e3:.0f} ms); "
              f"after quiesce {after_quiesce * 1e3:.3f} ms")
    finally:
        s.close()


# ---- host-memory inputs (sbe_serve_*_host: inputs copied into the request slot) ----------------
@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8, T.ENC_PUBLISH_TOPIC])
@pytest.mark.parametrize("n", [1, 2, 33, 36])
def test_serve_host_encode_topic(codec, server, n, flags):
    arena, L, ts = T.var_orders(n, seed=0x90 + n)  # n = 36: 14 KB of inputs, near the 16 KiB inline area
    got = host(server.encode_topic_host(arena, L, ts, flags=flags, ts_default=5), n)
    check_same(got, T.oracle_encode(arena, L, ts, flags=flags, ts_default=5))


def test_serve_host_encode_session_and_lite(codec, server):
    arena, L, ts = T.var_orders(20, seed=0x91)
    got = host(server.encode_topic_host(arena, L, ts, flags=T.ENC_REF_TRUNCATE8, session=(4, -9)), 20)
    check_same(got, T.oracle_encode_session(arena, L, ts, 4, -9, flags=T.ENC_REF_TRUNCATE8))
    for tid in (301, 201):
        a, Ll, t, q = T.lite_records(30, tid)
        check_same(host(server.encode_lite_host(tid, a, Ll, t, q), 30), T.oracle_encode_lite(tid, a, Ll, t, q))


def test_serve_host_encode_limits(codec, server):
    arena, L, ts = T.fixed256_orders(80)  # 80 x 250 B of inputs: past the 16 KiB inline area
    with pytest.raises(codec.SbeError):
        server.encode_topic_host(arena, L, ts)
    e = np.zeros(0, np.uint8)
    got = server.encode_topic_host(e, np.zeros((0, 5), np.uint32), np.zeros(0, np.uint64))
    assert got.out_off[:1].cpu().tolist() == [0]
    # E109 lengths count against the inline area too (their strings are part of the packed input)
    L2 = np.array([[70000, 0, 0, 0, 0]], np.uint32)
    with pytest.raises(codec.SbeError):
        server.encode_topic_host(np.zeros(70000, np.uint8), L2, np.ones(1, np.uint64))


@pytest.mark.parametrize("mode", [T.DEC_PARSE, T.DEC_EGRESS, T.DEC_LITE])
def test_serve_host_decode_edges_any_base(codec, server, mode):
    recs = [r for _, r in T.edge_records()]
    for lead in (0, 1, 7, 13):
        data, off = T.pack_records([b"\0" * lead] + recs)
        # the records after the lead-in, offsets not starting at 0: the host entry point rebases
        sub = off[1:]
        exp = T.oracle_decode(data, sub, mode)
        for a in range(0, len(sub) - 1, 50):
            b = min(a + 50, len(sub) - 1)
            got = server.decode_host(data, sub[a: b + 1], mode=mode).numpy()
            assert_same_decode(got, {k: v[a:b] for k, v in exp.items()})


def test_serve_host_decode_mixed_and_seq(codec, server):
    data, off = T.mixed_records(60, seed=0x92)
    for mode in (T.DEC_PARSE, T.DEC_EGRESS):
        assert_same_decode(server.decode_host(data, off, mode=mode).numpy(), T.oracle_decode(data, off, mode))
    key = b"_sequence_number"
    recs = [T.tm_wire([b"t", b"y", b"u", b'{"' + key + b'":%d}' % (i + 7), b"{}"], i) for i in range(10)]
    d2, o2 = T.pack_records(recs)
    dec = server.decode_host(d2, o2, seq=True)
    assert dec.seq.cpu().numpy().view(np.uint64).tolist() == [i + 7 for i in range(10)]
    with pytest.raises(codec.SbeError):  # past the inline area
        big, boff = T.mixed_records(200, seed=1)
        server.decode_host(big, boff)


# ---- several workgroups (sbe_server_create_wide): decode tiles and planned encodes ------------
def sizes_tm(L, flags=0, session=False):
    """Output / input bytes per record as sbe_enc_sums counts them (E109: no output)."""
    L = np.asarray(L, np.uint64).reshape(-1, 5)
    if flags & T.ENC_PUBLISH_TOPIC:
        out = (L & np.uint64(0xFFFF)).sum(1) + np.uint64(34)
    else:
        ovh = 26 if flags & T.ENC_REF_TRUNCATE8 else 34
        out = L.sum(1) + np.uint64(ovh + (32 if session else 0))
        out[(L > 65534).any(1)] = 0
    return out.astype(np.uint64), L.sum(1).astype(np.uint64)


@pytest.fixture(scope="module")
def wide(codec):
    s = codec.Server(workgroups=codec.SERVE_MAX_WORKGROUPS)
    yield s
    s.close()


@pytest.mark.parametrize("n", [1, 65, 1000, 4096])
def test_wide_decode_mixed(codec, wide, n):
    data, off = T.mixed_records(n, seed=0x51 + n)
    for mode in (T.DEC_PARSE, T.DEC_EGRESS):
        assert_same_decode(serve_decode(wide, data, off, mode).numpy(), T.oracle_decode(data, off, mode))


def test_wide_decode_long_and_host(codec, wide):
    arena, L, ts = long_records(300, 19)
    out, off, _ = T.oracle_encode(arena, L, ts)
    assert_same_decode(serve_decode(wide, out, off, T.DEC_PARSE).numpy(), T.oracle_decode(out, off, T.DEC_PARSE))
    data, off = T.mixed_records(60, seed=0x52)  # inline inputs, 1 tile: the leader alone
    assert_same_decode(wide.decode_host(data, off).numpy(), T.oracle_decode(data, off, T.DEC_PARSE))


@pytest.mark.parametrize("flags", [0, T.ENC_REF_TRUNCATE8, T.ENC_PUBLISH_TOPIC])
@pytest.mark.parametrize("n", [33, 1000, 4096])
def test_wide_planned_topic(codec, wide, n, flags):
    arena, L, ts = T.var_orders(n, seed=0x53 + n)
    ob, ib = sizes_tm(L, flags)
    tsum, bsum = codec.Server.tile_sums(codec.LAYOUT_TOPIC, ob, ib)
    got = wide.encode_planned(codec.LAYOUT_TOPIC, *tm_inputs(arena, L, ts), tsum, bsum, flags=flags, ts_default=3)
    check_same(host(got, n), T.oracle_encode(arena, L, ts, flags=flags, ts_default=3))


def test_wide_planned_e109_and_session(codec, wide):
    arena, L, ts = long_records(500, 23)
    L[7, 3] = 70000
    L[300, 1] = 65535
    arena = np.concatenate([arena, np.full(70000 + 65535, 66, np.uint8)])
    ob, ib = sizes_tm(L)
    tsum, bsum = codec.Server.tile_sums(codec.LAYOUT_TOPIC, ob, ib)
    got = wide.encode_planned(codec.LAYOUT_TOPIC, *tm_inputs(arena, L, ts), tsum, bsum)
    check_same(host(got, 500), T.oracle_encode(arena, L, ts))
    arena, L, ts = T.var_orders(2000, seed=0x54)
    ob, ib = sizes_tm(L, T.ENC_REF_TRUNCATE8, session=True)
    tsum, bsum = codec.Server.tile_sums(codec.LAYOUT_SESSION, ob, ib)
    got = wide.encode_planned(codec.LAYOUT_SESSION, *tm_inputs(arena, L, ts), tsum, bsum, flags=T.ENC_REF_TRUNCATE8,
                              session=(2, 5))
    check_same(host(got, 2000), T.oracle_encode_session(arena, L, ts, 2, 5, flags=T.ENC_REF_TRUNCATE8))


@pytest.mark.parametrize("template_id", [301, 201])
def test_wide_planned_lite(codec, wide, template_id):
    n = 3000
    arena, L, tid, seq = T.lite_records(n, template_id)
    nf = T.LITE_NF[template_id]
    Lu = np.asarray(L, np.uint64).reshape(-1, nf)
    ob = Lu.sum(1) + np.uint64(20 + 2 * nf)
    ob[(Lu > 65534).any(1)] = 0
    tsum, bsum = codec.Server.tile_sums(codec.LAYOUT_LITE, ob, Lu.sum(1))
    got = wide.encode_planned(codec.LAYOUT_LITE, to_dev(arena, torch.uint8), to_dev(L, torch.int32),
                              to_dev(seq, torch.int64), tsum, bsum, template_id=template_id,
                              topic_id=to_dev(tid, torch.int32))
    check_same(host(got, n), T.oracle_encode_lite(template_id, arena, L, tid, seq))


def test_wide_alternating_and_relaunch(codec):
    """One-tile requests (the leader alone, not republished) between wide ones, then idle exits:
    the followers' view of the sequence numbers and the exit count stay right."""
    s = codec.Server(idle_us=3000, workgroups=16)
    try:
        d1, o1 = T.mixed_records(1, seed=0x61)
        d2, o2 = T.mixed_records(900, seed=0x62)
        e1, e2 = T.oracle_decode(d1, o1, T.DEC_PARSE), T.oracle_decode(d2, o2, T.DEC_PARSE)
        for k in range(12):
            assert_same_decode(serve_decode(s, d2, o2, T.DEC_PARSE).numpy(), e2)
            for _ in range(k % 3):
                assert_same_decode(serve_decode(s, d1, o1, T.DEC_PARSE).numpy(), e1)
            if k % 4 == 3:
                time.sleep(0.02)  # past the idle time: all workgroups leave, the next request relaunches
        req, launches = s.stats()
        assert launches >= 3
    finally:
        s.close()
