"""CPU: libsbecodec.so loads and exports every entry point include/sbecodec.h declares; the
argument checks that need no device behave (no compute is launched here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "sbecodec.h")
LIB = os.path.join(ROOT, "aeron-cluster-client-cpp_amd", "libsbecodec.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.dirname(LIB), "libsbecodec.so"], check=True)
    return ctypes.CDLL(LIB)


def declared():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sbe_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared()
    for n in ("sbe_encode_topic_batch", "sbe_decode_batch", "sbe_encode_workspace_size", "sbe_abi_version"):
        assert n in names


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_host_side_entry_points(lib):
    lib.sbe_abi_version.restype = ctypes.c_int
    assert lib.sbe_abi_version() == 8
    lib.sbe_encode_workspace_size.restype = ctypes.c_size_t
    lib.sbe_encode_workspace_size.argtypes = [ctypes.c_uint64]
    assert lib.sbe_encode_workspace_size(1_000_000) >= 16 * (1_000_000 // 256)
    lib.sbe_encode_output_bound.restype = ctypes.c_uint64
    lib.sbe_encode_output_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    assert lib.sbe_encode_output_bound(10, 222 * 10, 0) == 2220 + (34 + 32) * 10  # covers session framing
    lib.sbe_lite_fields.restype = ctypes.c_uint32
    lib.sbe_lite_fields.argtypes = [ctypes.c_uint32]
    assert [lib.sbe_lite_fields(t) for t in (301, 201, 202, 1, 0)] == [2, 3, 3, 0, 0]
    lib.sbe_lite_output_bound.restype = ctypes.c_uint64
    lib.sbe_lite_output_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    assert lib.sbe_lite_output_bound(10, 500, 301) == 500 + 24 * 10
    assert lib.sbe_lite_output_bound(10, 500, 201) == 500 + 26 * 10
    lib.sbe_order_json_workspace_size.restype = ctypes.c_size_t
    lib.sbe_order_json_workspace_size.argtypes = [ctypes.c_uint64]
    assert lib.sbe_order_json_workspace_size(1000) >= 2 * 8 * 1000 + 2 * 8 * 4  # sizes, bases, block sums
    lib.sbe_last_error.restype = ctypes.c_char_p
    assert lib.sbe_last_error() == b""
    # the RCCL gather's argument checks (no communicator is created without a device)
    vp = ctypes.c_void_p
    lib.sbe_comm_init.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, vp]
    h = vp()
    uid = ctypes.create_string_buffer(128)
    assert lib.sbe_comm_init(ctypes.byref(h), 0, 0, uid) == -1
    assert lib.sbe_comm_init(ctypes.byref(h), 2, 2, uid) == -1
    assert lib.sbe_comm_init(None, 1, 0, uid) == -1
    lib.sbe_gather_encoded.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64, vp,
                                       ctypes.c_uint64, vp, vp]
    assert lib.sbe_gather_encoded(None, 0, None, None, 0, None, 0, None, 0, None, None) == -1
    lib.sbe_gather_encoded_sized.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp,
                                             ctypes.c_uint64, vp, vp]
    assert lib.sbe_gather_encoded_sized(None, 0, None, None, None, None, 0, None, 0, None, None) == -1
    lib.sbe_comm_destroy.argtypes = [vp]
    assert lib.sbe_comm_destroy(None) == 0


def test_invalid_arguments_are_rejected_before_any_launch(lib):
    vp = ctypes.c_void_p
    lib.sbe_order_to_json_batch.restype = ctypes.c_int
    lib.sbe_order_to_json_batch.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint64, vp, vp, vp,
                                            ctypes.c_size_t, vp]
    assert lib.sbe_order_to_json_batch(None, 1, 0, None, 0, None, None, None, 0, None) == -1
    lib.sbe_encode_topic_batch.restype = ctypes.c_int
    lib.sbe_encode_topic_batch.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, vp,
                                           ctypes.c_uint64, vp, vp, vp, ctypes.c_size_t, vp]
    assert lib.sbe_encode_topic_batch(None, 1, 0, 0, None, 0, None, None, None, 0, None) == -1
    lib.sbe_encode_lite_batch.restype = ctypes.c_int
    lib.sbe_encode_lite_batch.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_uint64, vp, vp, vp,
                                          ctypes.c_size_t, vp]
    dummy = (ctypes.c_uint64 * 8)()
    assert lib.sbe_encode_lite_batch(ctypes.addressof(dummy), 1, 7, None, 0, None, None, None, 0, None) == -1
    lib.sbe_encode_session_batch.restype = ctypes.c_int
    lib.sbe_encode_session_batch.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64,
                                             ctypes.c_int64, vp, ctypes.c_uint64, vp, vp, vp, ctypes.c_size_t, vp]
    assert lib.sbe_encode_session_batch(None, 1, 0, 0, 1, 2, None, 0, None, None, None, 0, None) == -1
    assert lib.sbe_encode_session_batch(ctypes.addressof(dummy), 1, 0, 0x80, 1, 2, None, 0,
                                        ctypes.addressof(dummy), None, None, 0, None) == -1  # unknown flag
    lib.sbe_decode_batch.restype = ctypes.c_int
    lib.sbe_decode_batch.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp, vp]
    assert lib.sbe_decode_batch(None, None, 5, 7, None, None) == -1      # unknown mode
    assert lib.sbe_decode_batch(None, None, 5, 0, None, None) == -1      # null buffers
    assert lib.sbe_decode_batch(None, None, 0, 0, None, None) == 0       # empty batch: nothing to do


def test_profiling_ring_without_launches(lib):
    lib.sbe_profile_enable.restype = ctypes.c_int
    lib.sbe_profile_enable.argtypes = [ctypes.c_int]
    lib.sbe_profile_read.restype = ctypes.c_int
    lib.sbe_profile_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    buf = (ctypes.c_float * 4)()
    # enabling creates the ring's HIP events up front: SBE_EHIP where no device is present
    assert lib.sbe_profile_enable(1) in (0, -2)
    assert lib.sbe_profile_read(0, buf, 4) == 0       # nothing launched yet
    assert lib.sbe_profile_read(2, buf, 4) == -1      # unknown kernel
    assert lib.sbe_profile_enable(0) == 0


def test_codec_library_does_not_link_rccl():
    """RCCL is dlopen-ed by the first sbe_comm_* call: the codec loads without it."""
    out = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"\(NEEDED\).*\[(.+?)\]", out)
    assert needed and not any("rccl" in n for n in needed), needed


def test_serve_entry_points_without_a_server(lib):
    """The serve API's host-side checks: a NULL server or out-of-range arguments are refused before
    anything touches a device (sbe_server_create itself needs one)."""
    EINVAL = -1
    for name, nargs in (("sbe_serve_encode_topic", 9), ("sbe_serve_encode_topic_host", 9),
                        ("sbe_serve_encode_session", 11), ("sbe_serve_encode_session_host", 11),
                        ("sbe_serve_encode_lite", 8), ("sbe_serve_encode_lite_host", 8),
                        ("sbe_serve_decode", 6), ("sbe_serve_decode_host", 6)):
        f = getattr(lib, name)
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * nargs
        assert f(*([None] * nargs)) == EINVAL, name
    lib.sbe_server_destroy.restype = ctypes.c_int
    lib.sbe_server_destroy.argtypes = [ctypes.c_void_p]
    assert lib.sbe_server_destroy(None) == 0
    lib.sbe_server_stats.restype = ctypes.c_int
    lib.sbe_server_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    assert lib.sbe_server_stats(None, None, None) == EINVAL
    lib.sbe_server_create.restype = ctypes.c_int
    lib.sbe_server_create.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    assert lib.sbe_server_create(None, 0) == EINVAL
