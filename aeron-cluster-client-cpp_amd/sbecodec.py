"""Python binding of the MI355X SBE codec C ABI (include/sbecodec.h) over ctypes.

PyTorch is plumbing here: it owns device memory and the current HIP stream; every byte of the
codec is produced by the HIP kernels in libsbecodec.so.  There is no CPU fallback: importing this
module without the built library, or calling it without a gfx950 device, raises.

Reference surface mirrored (paths relative to the reference tree):
  encode_topic_batch  ~ SBEEncoder::encode_topic_message   src/sbe_encoder.cpp:131-167
  encode_session_batch~ SessionManager create_topic_message + send_combined_message framing
                        src/session_manager.cpp:936-967, :1050-1144
  encode_lite_batch   ~ CommitManager::build_commit_offset_message (CommitOffsetLite)
                        src/commit_manager.cpp:107-132; OrderRequestLite / OrderNotificationLite
  decode_batch(LITE)  ~ the Lite templates' generated decode flyweights
  reassemble          ~ LocalFragmentReassembler::onFragment  src/cluster_client.cpp:39-82
  decode_batch(PARSE) ~ MessageParser::parse_message        src/sbe_encoder.cpp:513-551
  decode_batch(EGRESS)~ decode_ack + MessageHandler::on_egress
                        src/ack_decoder.cpp:29-105, include/aeron_cluster/message_handler.hpp:35-68
  order_to_json_batch ~ Order::to_json src/order_types.cpp:122-181 and publish_order's headers JSON
                        src/cluster_client.cpp:308-323
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SBECODEC_LIB") or os.path.join(_HERE, "libsbecodec.so")

# ---- constants mirrored from include/sbecodec.h ----
ABI_VERSION = 8
ENC_REF_TRUNCATE8 = 0x1
ENC_PUBLISH_TOPIC = 0x2
ENC_OK, ENC_OVERFLOW = 0, 6
DEC_PARSE_MESSAGE, DEC_ON_EGRESS, DEC_LITE = 0, 1, 2
TM_WIRE_OVERHEAD, TM_REF_OVERHEAD = 34, 26
SESSION_HDR_LEN = 32
COMMIT_OFFSET_LITE, ORDER_REQUEST_LITE, ORDER_NOTIFICATION_LITE = 301, 201, 202
LITE_FIELDS = {COMMIT_OFFSET_LITE: 2, ORDER_REQUEST_LITE: 3, ORDER_NOTIFICATION_LITE: 3}
ST_LITE, ST_LITE_E100, ST_LITE_NOT_LITE = 48, 49, 50
FRAG_BEGIN, FRAG_END = 0x80, 0x40
ORDER_FIELDS = 8  # client_order_uuid, identifier, base_token, quote_token, side, id, message_id, status
JSON_ORDER_PAYLOAD, JSON_PUBLISH_HEADERS = 0, 1
JSON_OK, JSON_OVERFLOW = 0, 6

ST_TM, ST_ACK, ST_SESSION_EVENT = 0, 1, 2
ST_ERR_NULL_EMPTY, ST_ERR_HEADER, ST_ERR_UNKNOWN_TYPE = 16, 17, 18
ST_ERR_SESSION_EVENT, ST_ERR_SESSION_SHORT, ST_ERR_EMBEDDED_SHORT = 19, 20, 21
ST_ERR_EMBEDDED_TEMPLATE, ST_ERR_EMBEDDED_SCHEMA, ST_ERR_DIRECT_TEMPLATE = 22, 23, 24
ST_ERR_TM_E100, ST_ERR_ACK_SHORT = 25, 26
ST_EG_ACK_SIMPLE, ST_EG_ACK, ST_EG_TM, ST_EG_NONE, ST_EG_THROW_E100 = 32, 33, 34, 35, 36
FL_ID_DEFAULT, FL_PAYLOAD_DEFAULT, FL_HEADERS_E100, FL_SEQ_KEY, FL_WRAPPED, FL_SEQ_ESC = 1, 2, 4, 8, 16, 32

_ERRORS = {0: "ok", -1: "EINVAL", -2: "EHIP", -3: "ENOSPC", -4: "ENODEV", -5: "ECOMM"}
COMM_ID_BYTES = 128


class SbeError(RuntimeError):
    pass


class _TmBatch(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("str_off", ctypes.c_void_p),
                ("str_len", ctypes.c_void_p), ("timestamp", ctypes.c_void_p)]


class _LiteBatch(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("str_off", ctypes.c_void_p), ("str_len", ctypes.c_void_p),
                ("topic_id", ctypes.c_void_p), ("sequence", ctypes.c_void_p)]


class _OrderBatch(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("str_off", ctypes.c_void_p), ("str_len", ctypes.c_void_p),
                ("customer_id", ctypes.c_void_p), ("timestamp", ctypes.c_void_p), ("quantity", ctypes.c_void_p)]


class _Decoded(ctypes.Structure):
    _fields_ = [("status", ctypes.c_void_p), ("flags", ctypes.c_void_p), ("hdr", ctypes.c_void_p),
                ("ts", ctypes.c_void_p), ("view_off", ctypes.c_void_p), ("view_len", ctypes.c_void_p),
                ("seq", ctypes.c_void_p)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise SbeError(f"{LIB_PATH} is missing: build it with `make -C aeron-cluster-client-cpp_amd` "
                       "(there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    lib.sbe_abi_version.restype = ctypes.c_int
    lib.sbe_device_ready.restype = ctypes.c_int
    lib.sbe_last_error.restype = ctypes.c_char_p
    lib.sbe_encode_workspace_size.restype = ctypes.c_size_t
    lib.sbe_encode_workspace_size.argtypes = [ctypes.c_uint64]
    lib.sbe_encode_workspace_init.restype = ctypes.c_int
    lib.sbe_encode_workspace_init.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.sbe_encode_output_bound.restype = ctypes.c_uint64
    lib.sbe_encode_output_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    lib.sbe_encode_topic_batch.restype = ctypes.c_int
    lib.sbe_encode_topic_batch.argtypes = [
        ctypes.POINTER(_TmBatch), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    if not hasattr(lib, "sbe_encode_session_batch"):  # an older build loaded for A/B timing only
        return lib if lib.sbe_abi_version() == ABI_VERSION else _abi_mismatch()
    lib.sbe_encode_session_batch.restype = ctypes.c_int
    lib.sbe_encode_session_batch.argtypes = [
        ctypes.POINTER(_TmBatch), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64,
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.sbe_lite_fields.restype = ctypes.c_uint32
    lib.sbe_lite_fields.argtypes = [ctypes.c_uint32]
    lib.sbe_lite_output_bound.restype = ctypes.c_uint64
    lib.sbe_lite_output_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    lib.sbe_encode_lite_batch.restype = ctypes.c_int
    lib.sbe_encode_lite_batch.argtypes = [
        ctypes.POINTER(_LiteBatch), ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.sbe_reassemble_workspace_size.restype = ctypes.c_size_t
    lib.sbe_reassemble_workspace_size.argtypes = [ctypes.c_uint64]
    lib.sbe_reassemble_fragments.restype = ctypes.c_int
    lib.sbe_reassemble_fragments.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.c_void_p]
    lib.sbe_decode_batch.restype = ctypes.c_int
    lib.sbe_decode_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.POINTER(_Decoded), ctypes.c_void_p]
    if hasattr(lib, "sbe_decode_batch_sized"):
        lib.sbe_decode_batch_sized.restype = ctypes.c_int
        lib.sbe_decode_batch_sized.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_uint32, ctypes.POINTER(_Decoded), ctypes.c_void_p]
    if hasattr(lib, "sbe_materialize_views"):
        lib.sbe_materialize_workspace_size.restype = ctypes.c_size_t
        lib.sbe_materialize_workspace_size.argtypes = [ctypes.c_uint64]
        lib.sbe_materialize_views.restype = ctypes.c_int
        lib.sbe_materialize_views.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.POINTER(_Decoded), ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.sbe_eval_sequence_numbers.restype = ctypes.c_int
    lib.sbe_eval_sequence_numbers.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.POINTER(_Decoded), ctypes.c_void_p, ctypes.c_void_p]
    lib.sbe_profile_enable.restype = ctypes.c_int
    lib.sbe_order_json_workspace_size.argtypes = [ctypes.c_uint64]
    lib.sbe_order_json_workspace_size.restype = ctypes.c_size_t
    lib.sbe_order_to_json_batch.argtypes = [ctypes.POINTER(_OrderBatch), ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.sbe_order_to_json_batch.restype = ctypes.c_int
    lib.sbe_profile_enable.argtypes = [ctypes.c_int]
    lib.sbe_profile_read.restype = ctypes.c_int
    lib.sbe_profile_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    lib.sbe_comm_unique_id.restype = ctypes.c_int
    lib.sbe_comm_unique_id.argtypes = [ctypes.c_void_p]
    lib.sbe_comm_init.restype = ctypes.c_int
    lib.sbe_comm_init.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.sbe_comm_destroy.restype = ctypes.c_int
    lib.sbe_comm_destroy.argtypes = [ctypes.c_void_p]
    lib.sbe_gather_encoded.restype = ctypes.c_int
    lib.sbe_gather_encoded.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    lib.sbe_gather_encoded_sized.restype = ctypes.c_int
    lib.sbe_gather_encoded_sized.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.c_void_p]
    lib.sbe_gather_plan.restype = ctypes.c_int
    lib.sbe_gather_plan.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_uint64)]
    lib.sbe_server_create.restype = ctypes.c_int
    lib.sbe_server_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32]
    lib.sbe_server_destroy.restype = ctypes.c_int
    lib.sbe_server_destroy.argtypes = [ctypes.c_void_p]
    lib.sbe_server_quiesce.restype = ctypes.c_int
    lib.sbe_server_quiesce.argtypes = [ctypes.c_void_p]
    lib.sbe_server_stats.restype = ctypes.c_int
    lib.sbe_server_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.sbe_serve_encode_topic.restype = ctypes.c_int
    lib.sbe_serve_encode_topic.argtypes = [ctypes.c_void_p, ctypes.POINTER(_TmBatch), ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_void_p]
    lib.sbe_serve_encode_session.restype = ctypes.c_int
    lib.sbe_serve_encode_session.argtypes = [ctypes.c_void_p, ctypes.POINTER(_TmBatch), ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    lib.sbe_serve_encode_lite.restype = ctypes.c_int
    lib.sbe_serve_encode_lite.argtypes = [ctypes.c_void_p, ctypes.POINTER(_LiteBatch), ctypes.c_uint64,
                                          ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_void_p]
    lib.sbe_serve_encode_topic_host.restype = ctypes.c_int
    lib.sbe_serve_encode_topic_host.argtypes = lib.sbe_serve_encode_topic.argtypes
    lib.sbe_serve_encode_session_host.restype = ctypes.c_int
    lib.sbe_serve_encode_session_host.argtypes = lib.sbe_serve_encode_session.argtypes
    lib.sbe_serve_encode_lite_host.restype = ctypes.c_int
    lib.sbe_serve_encode_lite_host.argtypes = lib.sbe_serve_encode_lite.argtypes
    lib.sbe_serve_decode_host.restype = ctypes.c_int
    lib.sbe_serve_decode_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_uint32, ctypes.POINTER(_Decoded)]
    lib.sbe_server_create_wide.restype = ctypes.c_int
    lib.sbe_server_create_wide.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.c_uint32]
    lib.sbe_encode_tile_records.restype = ctypes.c_uint32
    lib.sbe_encode_tile_records.argtypes = [ctypes.c_uint32]
    for name, base in (("sbe_serve_encode_topic_planned", lib.sbe_serve_encode_topic.argtypes),
                       ("sbe_serve_encode_session_planned", lib.sbe_serve_encode_session.argtypes),
                       ("sbe_serve_encode_lite_planned", lib.sbe_serve_encode_lite.argtypes)):
        f = getattr(lib, name)
        f.restype = ctypes.c_int
        f.argtypes = list(base) + [ctypes.c_void_p, ctypes.c_void_p]
    lib.sbe_serve_decode.restype = ctypes.c_int
    lib.sbe_serve_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_uint32, ctypes.POINTER(_Decoded)]
    if lib.sbe_abi_version() != ABI_VERSION:
        _abi_mismatch()
    return lib


def _abi_mismatch():
    raise SbeError("libsbecodec.so ABI version mismatch")


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def use_library(path: str):
    """Bind this module to another build of the codec (A/B timing of kernel variants)."""
    global _lib, LIB_PATH
    LIB_PATH = path
    _lib = _load()


def _check(rc: int, what: str):
    if rc != 0:
        raise SbeError(f"{what} failed: {_ERRORS.get(rc, rc)} {lib().sbe_last_error().decode()}")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _dev(t, dtype, name):
    if t is None:
        return None
    if not (t.is_cuda and t.dtype == dtype and t.is_contiguous()):
        raise SbeError(f"{name}: expected a contiguous {dtype} device tensor")
    return t


def require_device():
    if not torch.cuda.is_available() or lib().sbe_device_ready() != 1:
        raise SbeError("no gfx950 device visible: the SBE codec runs only on MI355X")


PROF_PACK, PROF_DECODE = 0, 1


def profile_enable(every: int = 1):
    """HIP events on the pack / decode kernel dispatch of every `every`-th call (0: off)."""
    _check(lib().sbe_profile_enable(int(every)), "sbe_profile_enable")


def profile_read(kernel: int, max_n: int = 256) -> list:
    """Elapsed ms of the recorded launches of `kernel` (oldest first); synchronise first."""
    buf = (ctypes.c_float * max_n)()
    n = lib().sbe_profile_read(kernel, buf, max_n)
    if n < 0:
        _check(n, "sbe_profile_read")
    return [float(buf[i]) for i in range(n)]


def output_bound(n: int, string_bytes: int, flags: int = 0) -> int:
    return int(lib().sbe_encode_output_bound(n, string_bytes, flags))


def workspace_size(n: int) -> int:
    return int(lib().sbe_encode_workspace_size(n))


def alloc_workspace(n: int, device, stream=None) -> torch.Tensor:
    """Workspace for encoding up to n records, zeroed and registered once."""
    ws = torch.empty(max(workspace_size(n), 16), dtype=torch.uint8, device=device)
    _check(lib().sbe_encode_workspace_init(_ptr(ws), ws.numel(), _stream(stream)), "sbe_encode_workspace_init")
    return ws


@dataclass
class Encoded:
    out: torch.Tensor       # uint8 [capacity]; record i = out[out_off[i]:out_off[i+1]]
    out_off: torch.Tensor   # int64 [n+1]
    status: torch.Tensor    # uint8 [n]
    workspace: torch.Tensor | None = None


def encode_topic_batch(arena, str_len, timestamp, str_off=None, flags=0, ts_default=0,
                       out=None, out_off=None, status=None, workspace=None, stream=None) -> Encoded:
    """Batch TopicMessage encode.  arena uint8, str_len int32 [n,5] (u32), timestamp int64 [n] (u64),
    str_off int32 [n,5] or None (packed).  Output buffers are allocated when not given."""
    arena = _dev(arena, torch.uint8, "arena")
    str_len = _dev(str_len, torch.int32, "str_len")
    timestamp = _dev(timestamp, torch.int64, "timestamp")
    str_off = _dev(str_off, torch.int32, "str_off")
    n = int(timestamp.numel())
    if str_len.numel() != 5 * n:
        raise SbeError("str_len must have 5 entries per record")
    dev = arena.device
    if out is None:
        cap = output_bound(n, int(arena.numel()), flags)
        out = torch.empty(max(cap, 16), dtype=torch.uint8, device=dev)
    if out_off is None:
        out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    elif status is False:
        status = None
    if workspace is None:
        workspace = alloc_workspace(n, dev, stream)
    elif workspace.numel() < workspace_size(n):
        raise SbeError("workspace too small")
    batch = _TmBatch(arena.data_ptr(), None if str_off is None else str_off.data_ptr(),
                     str_len.data_ptr(), timestamp.data_ptr())
    rc = lib().sbe_encode_topic_batch(ctypes.byref(batch), n, ts_default & (2**64 - 1), flags,
                                      _ptr(out), out.numel(), _ptr(out_off), _ptr(status),
                                      _ptr(workspace), workspace.numel(), _stream(stream))
    _check(rc, "sbe_encode_topic_batch")
    return Encoded(out, out_off, None if status is None else status[:n], workspace)


def _enc_outputs(n, cap, dev, out, out_off, status, workspace, stream):
    if out is None:
        out = torch.empty(max(cap, 16), dtype=torch.uint8, device=dev)
    if out_off is None:
        out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    elif status is False:
        status = None
    if workspace is None:
        workspace = alloc_workspace(n, dev, stream)
    elif workspace.numel() < workspace_size(n):
        raise SbeError("workspace too small")
    return out, out_off, status, workspace


def encode_session_batch(arena, str_len, timestamp, leadership_term_id, cluster_session_id, str_off=None,
                         flags=ENC_REF_TRUNCATE8, ts_default=0, out=None, out_off=None, status=None,
                         workspace=None, stream=None) -> Encoded:
    """Session-framed TopicMessages: each record is the 32-B SessionMessageHeader followed by the
    TopicMessage (26+Σlen bytes with ENC_REF_TRUNCATE8, as the live publish path sends it)."""
    arena = _dev(arena, torch.uint8, "arena")
    str_len = _dev(str_len, torch.int32, "str_len")
    timestamp = _dev(timestamp, torch.int64, "timestamp")
    str_off = _dev(str_off, torch.int32, "str_off")
    n = int(timestamp.numel())
    if str_len.numel() != 5 * n:
        raise SbeError("str_len must have 5 entries per record")
    out, out_off, status, workspace = _enc_outputs(n, output_bound(n, int(arena.numel()), flags), arena.device,
                                                   out, out_off, status, workspace, stream)
    batch = _TmBatch(arena.data_ptr(), None if str_off is None else str_off.data_ptr(),
                     str_len.data_ptr(), timestamp.data_ptr())
    rc = lib().sbe_encode_session_batch(ctypes.byref(batch), n, ts_default & (2**64 - 1), flags,
                                        int(leadership_term_id), int(cluster_session_id),
                                        _ptr(out), out.numel(), _ptr(out_off), _ptr(status),
                                        _ptr(workspace), workspace.numel(), _stream(stream))
    _check(rc, "sbe_encode_session_batch")
    return Encoded(out, out_off, None if status is None else status[:n], workspace)


def encode_lite_batch(template_id, arena, str_len, topic_id, sequence, str_off=None, out=None, out_off=None,
                      status=None, workspace=None, stream=None) -> Encoded:
    """Lite records (301 CommitOffsetLite, 201 OrderRequestLite, 202 OrderNotificationLite):
    str_len int32 [n, nf] (u32), topic_id int32 [n] (u32), sequence int64 [n] (u64)."""
    nf = LITE_FIELDS.get(int(template_id))
    if nf is None:
        raise SbeError(f"not a Lite template: {template_id}")
    arena = _dev(arena, torch.uint8, "arena")
    str_len = _dev(str_len, torch.int32, "str_len")
    topic_id = _dev(topic_id, torch.int32, "topic_id")
    sequence = _dev(sequence, torch.int64, "sequence")
    str_off = _dev(str_off, torch.int32, "str_off")
    n = int(sequence.numel())
    if str_len.numel() != nf * n or topic_id.numel() != n:
        raise SbeError(f"str_len must have {nf} entries and topic_id one per record")
    cap = int(lib().sbe_lite_output_bound(n, int(arena.numel()), int(template_id)))
    out, out_off, status, workspace = _enc_outputs(n, cap, arena.device, out, out_off, status, workspace, stream)
    batch = _LiteBatch(arena.data_ptr(), None if str_off is None else str_off.data_ptr(), str_len.data_ptr(),
                       topic_id.data_ptr(), sequence.data_ptr())
    rc = lib().sbe_encode_lite_batch(ctypes.byref(batch), n, int(template_id), _ptr(out), out.numel(),
                                     _ptr(out_off), _ptr(status), _ptr(workspace), workspace.numel(),
                                     _stream(stream))
    _check(rc, "sbe_encode_lite_batch")
    return Encoded(out, out_off, None if status is None else status[:n], workspace)


@dataclass
class Decoded:
    status: torch.Tensor    # uint8 [n]
    flags: torch.Tensor     # uint8 [n]
    hdr: torch.Tensor       # int16 [n,4]  (u16 block_length, template_id, schema_id, version)
    ts: torch.Tensor        # int64 [n]    (u64)
    view_off: torch.Tensor  # int32 [n,5]  (u32, relative to the record start)
    view_len: torch.Tensor  # int32 [n,5]  (u32)
    seq: torch.Tensor | None = None  # int64 [n] (u64): sequence_number of flagged records (parse mode)

    def numpy(self):
        import numpy as np
        return {k: getattr(self, k).cpu().numpy().view(t) for k, t in
                (("status", np.uint8), ("flags", np.uint8), ("hdr", np.uint16), ("ts", np.uint64),
                 ("view_off", np.uint32), ("view_len", np.uint32))}


def alloc_decoded(n: int, device) -> Decoded:
    m = max(n, 1)
    return Decoded(torch.empty(m, dtype=torch.uint8, device=device),
                   torch.empty(m, dtype=torch.uint8, device=device),
                   torch.empty((m, 4), dtype=torch.int16, device=device),
                   torch.empty(m, dtype=torch.int64, device=device),
                   torch.empty((m, 5), dtype=torch.int32, device=device),
                   torch.empty((m, 5), dtype=torch.int32, device=device))


def decode_batch(data, rec_off, mode=DEC_PARSE_MESSAGE, out: Decoded | None = None, stream=None,
                 seq=None, in_bytes: int = 0) -> Decoded:
    """Batch decode of the records data[rec_off[i]:rec_off[i+1]] (rec_off int64 [n+1]).
    Parse mode with seq (int64 [n]): the same launch writes ParseResult.sequence_number of the
    records flagged FL_SEQ_KEY / FL_SEQ_ESC (others are not written; seq=True allocates it zeroed).
    in_bytes: the records' total bytes when the caller knows them (rec_off[n] - rec_off[0]); only
    picks the kernel shape (sbe_decode_batch_sized), results are the same."""
    data = _dev(data, torch.uint8, "data")
    rec_off = _dev(rec_off, torch.int64, "rec_off")
    n = int(rec_off.numel()) - 1
    if out is None:
        out = alloc_decoded(n, data.device)
    if seq is True:
        seq = torch.zeros(max(n, 1), dtype=torch.int64, device=data.device)
    if seq is not None:
        seq = _dev(seq, torch.int64, "seq")
    d = _Decoded(*(getattr(out, k).data_ptr() for k in ("status", "flags", "hdr", "ts", "view_off", "view_len")),
                 None if seq is None else seq.data_ptr())
    if in_bytes and hasattr(lib(), "sbe_decode_batch_sized"):
        rc = lib().sbe_decode_batch_sized(_ptr(data), _ptr(rec_off), n, int(in_bytes), mode, ctypes.byref(d),
                                          _stream(stream))
    else:
        rc = lib().sbe_decode_batch(_ptr(data), _ptr(rec_off), n, mode, ctypes.byref(d), _stream(stream))
    _check(rc, "sbe_decode_batch")
    keys = ("status", "flags", "hdr", "ts", "view_off", "view_len")
    if n < out.status.numel():
        out = Decoded(*(getattr(out, k)[:n] for k in keys))
    else:
        out = Decoded(*(getattr(out, k) for k in keys))
    out.seq = None if seq is None else seq[:n]
    return out


def eval_sequence_numbers(data, rec_off, dec: Decoded, seq=None, stream=None) -> torch.Tensor:
    """ParseResult.sequence_number (src/sbe_encoder.cpp:1031-1125) of the records a parse-mode
    decode_batch flagged (FL_SEQ_KEY / FL_SEQ_ESC on a TopicMessage); the JSON evaluation runs on the
    device.  seq (int64 [n], u64 values) is allocated zeroed when not given; entries of unflagged
    records are not written (their sequence_number is 0)."""
    data = _dev(data, torch.uint8, "data")
    rec_off = _dev(rec_off, torch.int64, "rec_off")
    n = int(rec_off.numel()) - 1
    if seq is None:
        seq = torch.zeros(max(n, 1), dtype=torch.int64, device=data.device)
    d = _Decoded(*(getattr(dec, k).data_ptr() for k in ("status", "flags", "hdr", "ts", "view_off", "view_len")))
    rc = lib().sbe_eval_sequence_numbers(_ptr(data), _ptr(rec_off), n, ctypes.byref(d), _ptr(seq), _stream(stream))
    _check(rc, "sbe_eval_sequence_numbers")
    return seq[:n]


@dataclass
class Materialized:
    arena: torch.Tensor      # uint8: every record's five views back to back
    arena_off: torch.Tensor  # int64 [5n+1]: view k of record i = arena[arena_off[5i+k]:][:view_len[i][k]]


def materialize_views(data, rec_off, dec: Decoded, arena=None, arena_capacity=None, arena_off=None,
                      workspace=None, stream=None) -> Materialized:
    """MATERIALIZE (sbe_materialize_views): the five views of every record that decode_batch
    described, copied out of `data` into one arena, so the strings outlive the input (the
    reference's ParseResult owns its strings, include/aeron_cluster/sbe_messages.hpp:306-328).
    With no arena given, it is sized exactly: one synchronisation of `stream` reads the total."""
    data = _dev(data, torch.uint8, "data")
    rec_off = _dev(rec_off, torch.int64, "rec_off")
    n = int(rec_off.numel()) - 1
    dev = data.device
    if arena_off is None:
        arena_off = torch.empty(5 * n + 1, dtype=torch.int64, device=dev)
    arena_off = _dev(arena_off, torch.int64, "arena_off")
    if arena_off.numel() < 5 * n + 1:
        raise SbeError(f"arena_off holds {arena_off.numel()} entries, 5 n + 1 = {5 * n + 1} needed")
    need = int(lib().sbe_materialize_workspace_size(max(n, 1)))
    if workspace is None:
        workspace = torch.empty(need + 16, dtype=torch.uint8, device=dev)
    workspace = _dev(workspace, torch.uint8, "workspace")
    d = _Decoded(*(getattr(dec, k).data_ptr() for k in ("status", "flags", "hdr", "ts", "view_off", "view_len")))
    sized = arena is None and arena_capacity is None
    if sized:  # views can only be as long as the records: the input bytes bound the arena
        total = int(dec.view_len[:n].to(torch.int64).sum().item()) if n else 0
        arena = torch.empty(max(total, 16), dtype=torch.uint8, device=dev)
    arena = _dev(arena, torch.uint8, "arena")
    cap = int(arena.numel()) if arena_capacity is None else int(arena_capacity)
    if cap > arena.numel():
        raise SbeError(f"arena_capacity {cap} exceeds the arena tensor ({arena.numel()} bytes)")
    rc = lib().sbe_materialize_views(_ptr(data), _ptr(rec_off), n, ctypes.byref(d), _ptr(arena), cap,
                                     _ptr(arena_off), _ptr(workspace), int(workspace.numel()), _stream(stream))
    _check(rc, "sbe_materialize_views")
    return Materialized(arena, arena_off[: 5 * n + 1])


@dataclass
class Reassembled:
    out: torch.Tensor      # uint8: messages back to back, then the carry
    msg_off: torch.Tensor  # int64 [n+1]: message j = out[msg_off[j]:msg_off[j+1]] for j < m
    counts: torch.Tensor   # int64 [2]: m, carry bytes (carry = out[msg_off[m]:msg_off[m]+carry])


def reassemble(data, frag_off, flags, out=None, msg_off=None, workspace=None, stream=None) -> Reassembled:
    """Aeron BEGIN/END fragment reassembly of data[frag_off[i]:frag_off[i+1]] with flags[i]."""
    data = _dev(data, torch.uint8, "data")
    frag_off = _dev(frag_off, torch.int64, "frag_off")
    flags = _dev(flags, torch.uint8, "flags")
    n = int(flags.numel())
    if frag_off.numel() != n + 1:
        raise SbeError("frag_off must have n + 1 entries")
    dev = data.device
    if out is None:
        out = torch.empty(max(int(data.numel()), 16), dtype=torch.uint8, device=dev)
    if msg_off is None:
        msg_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    counts = torch.empty(2, dtype=torch.int64, device=dev)
    need = int(lib().sbe_reassemble_workspace_size(n))
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(max(need, 16), dtype=torch.uint8, device=dev)
    rc = lib().sbe_reassemble_fragments(_ptr(data), _ptr(frag_off), _ptr(flags), n, _ptr(out), _ptr(msg_off),
                                        _ptr(counts), _ptr(workspace), workspace.numel(), _stream(stream))
    _check(rc, "sbe_reassemble_fragments")
    return Reassembled(out, msg_off, counts)


# bytes per order of the default output bound (a record is at most ~800 B plus its escaped strings:
# 428 fixed, 316 for a "%f" quantity near DBL_MAX, 24 for "%.17g", 34 for the two integers)
ORDER_JSON_BOUND = 900


@dataclass
class OrderJson:
    out: torch.Tensor      # u8 text, record i = out[out_off[i]:out_off[i+1]]
    out_off: torch.Tensor  # i64 [n+1]
    status: torch.Tensor   # u8 [n]


def order_json_workspace_size(n: int) -> int:
    return int(lib().sbe_order_json_workspace_size(n))


def order_to_json_batch(arena, str_len, customer_id, timestamp, quantity, what=JSON_ORDER_PAYLOAD,
                        str_off=None, out=None, out_capacity=None, out_off=None, status=None, workspace=None,
                        stream=None) -> OrderJson:
    """Order::to_json (what=JSON_ORDER_PAYLOAD) or publish_order's headers JSON
    (what=JSON_PUBLISH_HEADERS) of n Orders, str_len [n][8] (ORDER_FIELDS order).
    Asynchronous on `stream` when the caller passes `out` or `out_capacity`; when this call sizes
    the output itself it synchronises `stream` once to read the total (out_off[n]) and reruns the
    launches at that size if the default bound was short."""
    arena = _dev(arena, torch.uint8, "arena")
    str_len = _dev(str_len, torch.int32, "str_len")
    customer_id = _dev(customer_id, torch.int64, "customer_id")
    timestamp = _dev(timestamp, torch.int64, "timestamp")
    quantity = _dev(quantity, torch.float64, "quantity")
    n = int(customer_id.numel())
    if str_len.numel() != ORDER_FIELDS * n or timestamp.numel() != n or quantity.numel() != n:
        raise SbeError("order batch arrays disagree on n")
    if str_off is not None:
        str_off = _dev(str_off, torch.int32, "str_off")
        if str_off.numel() != ORDER_FIELDS * n:
            raise SbeError("str_off must be [n][8]")
    dev = arena.device
    grow = out is None and out_capacity is None  # a buffer this call sizes itself is regrown if short
    if out is None:
        cap = out_capacity if out_capacity is not None else ORDER_JSON_BOUND * n + 6 * 3 * int(arena.numel()) + 64
        out = torch.empty(max(int(cap), 16), dtype=torch.uint8, device=dev)
    cap = int(out.numel()) if out_capacity is None else int(out_capacity)
    if cap > out.numel():
        raise SbeError(f"out_capacity {cap} exceeds the out tensor ({out.numel()} bytes)")
    if out_off is None:
        out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    need = order_json_workspace_size(n)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(max(need, 16), dtype=torch.uint8, device=dev)
    b = _OrderBatch(_ptr(arena), _ptr(str_off) if str_off is not None else None, _ptr(str_len),
                    _ptr(customer_id), _ptr(timestamp), _ptr(quantity))

    def run(o, c):
        rc = lib().sbe_order_to_json_batch(ctypes.byref(b), n, what, _ptr(o), c, _ptr(out_off), _ptr(status),
                                           _ptr(workspace), workspace.numel(), _stream(stream))
        _check(rc, "sbe_order_to_json_batch")

    run(out, cap)
    if grow and n:  # out_off always holds the full sizes: one rerun at the measured size
        s = stream if stream is not None else torch.cuda.current_stream()
        s.synchronize()  # the launches ran on `stream`, which need not be torch's current stream
        total = int(out_off[n].item())
        if total > cap:
            out = torch.empty(total, dtype=torch.uint8, device=dev)
            run(out, total)
    return OrderJson(out, out_off, status)


# ---------------------------------------------------------------------------------------------
# multi-GPU gather of encoded shards over RCCL (sbe_gather_encoded)
# ---------------------------------------------------------------------------------------------
def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id, made on one rank and handed to every rank out of band."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _check(lib().sbe_comm_unique_id(buf), "sbe_comm_unique_id")
    return buf.raw


class Comm:
    """One rank's communicator for sbe_gather_encoded (collective creation on the current device)."""

    def __init__(self, world: int, rank: int, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise SbeError("communicator id must be 128 bytes")
        self.world, self.rank = int(world), int(rank)
        self._h = ctypes.c_void_p()
        idbuf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        _check(lib().sbe_comm_init(ctypes.byref(self._h), self.world, self.rank, idbuf), "sbe_comm_init")

    def close(self):
        if self._h:
            _check(lib().sbe_comm_destroy(self._h), "sbe_comm_destroy")
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gather_plan(ranks, root: int = 0):
    """sbe_gather_plan on the host: ranks = [(bytes, records, dst_capacity, dst_off_capacity)] per
    rank (capacities read from the root's entry).  Returns (rc, byte_base, rec_base, totals) with
    the bases as lists of world + 1 prefix sums; rc is 0 or ENOSPC (-3)."""
    world = len(ranks)
    flat = (ctypes.c_uint64 * (4 * max(world, 1)))(*[int(v) & (2**64 - 1) for r in ranks for v in r])
    bb = (ctypes.c_uint64 * (world + 1))()
    rb = (ctypes.c_uint64 * (world + 1))()
    tot = (ctypes.c_uint64 * 2)()
    rc = lib().sbe_gather_plan(flat, world, int(root), bb, rb, tot)
    return rc, list(bb), list(rb), (int(tot[0]), int(tot[1]))


def gather_encoded(comm: Comm, out, out_off, n: int, root: int = 0, dst=None, dst_off=None, stream=None):
    """Collective: every rank's encoded shard (out, out_off [n+1]) back to back on `root`, offsets
    rebased.  The root passes dst (uint8, large enough for every shard) and dst_off (int64, N + 1
    entries); returns (dst[:bytes], dst_off, bytes, N) on the root and (None, None, bytes, N)
    elsewhere.  A short dst / dst_off raises ENOSPC on every rank before any transfer."""
    out = _dev(out, torch.uint8, "out")
    out_off = _dev(out_off, torch.int64, "out_off")
    if out_off.numel() < int(n) + 1:
        raise SbeError(f"out_off holds {out_off.numel()} entries, the shard needs n + 1 = {int(n) + 1}")
    am_root = comm.rank == root
    if am_root:
        dst = _dev(dst, torch.uint8, "dst")
        dst_off = _dev(dst_off, torch.int64, "dst_off")
        if dst is None or dst_off is None:
            raise SbeError("the root passes dst and dst_off")
    totals = (ctypes.c_uint64 * 2)()
    rc = lib().sbe_gather_encoded(comm._h, int(root), _ptr(out), _ptr(out_off), int(n),
                                  _ptr(dst) if am_root else None, int(dst.numel()) if am_root else 0,
                                  _ptr(dst_off) if am_root else None, int(dst_off.numel()) if am_root else 0,
                                  totals, _stream(stream))
    _check(rc, "sbe_gather_encoded")
    nbytes, nrec = int(totals[0]), int(totals[1])
    if am_root:
        return dst[:nbytes], dst_off[: nrec + 1], nbytes, nrec
    return None, None, nbytes, nrec


def gather_encoded_sized(comm: Comm, sizes, out, out_off, root: int = 0, dst=None, dst_off=None,
                         dst_capacity: int = 0, dst_off_capacity: int = 0, stream=None):
    """Collective, for callers that know every shard's size: sizes = [(bytes, records)] per rank,
    identical on every rank.  No size all-gather and no host wait (sbe_gather_encoded_sized): the
    transfers and the root's rebase are enqueued on `stream`.  Every rank passes the ROOT's
    capacities (dst_capacity bytes, dst_off_capacity offsets; both required, on every rank: a rank
    that decided ENOSPC alone would leave the others blocked in their transfers); returns as
    gather_encoded.

    Checked before anything is enqueued: both capacities non-zero; on the root, that
    they do not exceed dst / dst_off; on every rank, that out / out_off hold this rank's
    sizes[rank] bytes / records (RCCL reads and writes exactly the planned counts)."""
    world = comm.world
    if len(sizes) != world:
        raise SbeError(f"sizes has {len(sizes)} entries for a world of {world}")
    dst_capacity, dst_off_capacity = int(dst_capacity), int(dst_off_capacity)
    if dst_capacity <= 0 or dst_off_capacity <= 0:
        raise SbeError("gather_encoded_sized: every rank passes the root's dst_capacity and dst_off_capacity "
                       f"(got {dst_capacity}, {dst_off_capacity})")
    my_bytes, my_recs = (int(v) for v in sizes[comm.rank])
    out = _dev(out, torch.uint8, "out")
    out_off = _dev(out_off, torch.int64, "out_off")
    if out is None or out_off is None:
        raise SbeError("gather_encoded_sized: every rank passes its shard's out and out_off")
    if out.numel() < my_bytes or out_off.numel() < my_recs:
        raise SbeError(f"rank {comm.rank}: shard buffers hold {out.numel()} bytes / {out_off.numel()} offsets, "
                       f"sizes[{comm.rank}] says {my_bytes} / {my_recs}")
    am_root = comm.rank == root
    if am_root:
        dst = _dev(dst, torch.uint8, "dst")
        dst_off = _dev(dst_off, torch.int64, "dst_off")
        if dst is None or dst_off is None:
            raise SbeError("the root passes dst and dst_off")
        if dst_capacity > dst.numel() or dst_off_capacity > dst_off.numel():
            raise SbeError(f"root capacities {dst_capacity} / {dst_off_capacity} exceed dst ({dst.numel()}) / "
                           f"dst_off ({dst_off.numel()})")
    flat = (ctypes.c_uint64 * (2 * world))(*[int(v) for sz in sizes for v in sz])
    totals = (ctypes.c_uint64 * 2)()
    rc = lib().sbe_gather_encoded_sized(comm._h, int(root), flat, _ptr(out), _ptr(out_off),
                                        _ptr(dst) if am_root else None, dst_capacity,
                                        _ptr(dst_off) if am_root else None, dst_off_capacity,
                                        totals, _stream(stream))
    _check(rc, "sbe_gather_encoded_sized")
    nbytes, nrec = int(totals[0]), int(totals[1])
    if am_root:
        return dst[:nbytes], dst_off[: nrec + 1], nbytes, nrec
    return None, None, nbytes, nrec


SERVE_MAX_RECORDS = 4096
SERVE_MAX_WORKGROUPS = 64
LAYOUT_TOPIC, LAYOUT_SESSION, LAYOUT_LITE = 0, 1, 2


class Server:
    """The small-batch serve kernel (sbe_server_* in include/sbecodec.h): one resident wave on its
    own HIP stream that polls a page-locked request slot, so a one-record call costs no kernel
    launch.  Every method is synchronous and returns the batch entry point's outputs for the same
    inputs.  Inputs must be complete when a method is called (it synchronises torch's current
    stream first); encodes take packed input (no str_off); n <= SERVE_MAX_RECORDS."""

    def __init__(self, idle_us: int = 0, workgroups: int = 1):
        require_device()
        h = ctypes.c_void_p()
        _check(lib().sbe_server_create_wide(ctypes.byref(h), int(idle_us), int(workgroups)), "sbe_server_create_wide")
        self._h = h
        self.workgroups = int(workgroups)

    def close(self):
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            _check(lib().sbe_server_destroy(h), "sbe_server_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def quiesce(self):
        """Make the resident kernel exit now (sbe_server_quiesce); the next request relaunches it.
        A resident server holds up device-wide synchronisation (torch.cuda.synchronize()) and
        work on streams that share its hardware queue until it goes idle."""
        _check(lib().sbe_server_quiesce(self._h), "sbe_server_quiesce")

    def stats(self):
        """(requests served, kernel launches) so far."""
        r, l = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().sbe_server_stats(self._h, ctypes.byref(r), ctypes.byref(l)), "sbe_server_stats")
        return int(r.value), int(l.value)

    def encode_topic(self, arena, str_len, timestamp, flags=0, ts_default=0, out=None, out_off=None,
                     status=None) -> Encoded:
        arena = _dev(arena, torch.uint8, "arena")
        str_len = _dev(str_len, torch.int32, "str_len")
        timestamp = _dev(timestamp, torch.int64, "timestamp")
        n = int(timestamp.numel())
        if str_len.numel() != 5 * n:
            raise SbeError("str_len must have 5 entries per record")
        out, out_off, status = self._outputs(n, output_bound(n, int(arena.numel()), flags), arena.device,
                                             out, out_off, status)
        batch = _TmBatch(arena.data_ptr(), None, str_len.data_ptr(), timestamp.data_ptr())
        torch.cuda.current_stream().synchronize()
        rc = lib().sbe_serve_encode_topic(self._h, ctypes.byref(batch), n, ts_default & (2**64 - 1), flags,
                                          _ptr(out), out.numel(), _ptr(out_off), _ptr(status))
        _check(rc, "sbe_serve_encode_topic")
        return Encoded(out, out_off, None if status is None else status[:n])

    def encode_session(self, arena, str_len, timestamp, leadership_term_id, cluster_session_id,
                       flags=ENC_REF_TRUNCATE8, ts_default=0, out=None, out_off=None, status=None) -> Encoded:
        arena = _dev(arena, torch.uint8, "arena")
        str_len = _dev(str_len, torch.int32, "str_len")
        timestamp = _dev(timestamp, torch.int64, "timestamp")
        n = int(timestamp.numel())
        if str_len.numel() != 5 * n:
            raise SbeError("str_len must have 5 entries per record")
        out, out_off, status = self._outputs(n, output_bound(n, int(arena.numel()), flags), arena.device,
                                             out, out_off, status)
        batch = _TmBatch(arena.data_ptr(), None, str_len.data_ptr(), timestamp.data_ptr())
        torch.cuda.current_stream().synchronize()
        rc = lib().sbe_serve_encode_session(self._h, ctypes.byref(batch), n, ts_default & (2**64 - 1), flags,
                                            int(leadership_term_id), int(cluster_session_id), _ptr(out),
                                            out.numel(), _ptr(out_off), _ptr(status))
        _check(rc, "sbe_serve_encode_session")
        return Encoded(out, out_off, None if status is None else status[:n])

    def encode_lite(self, template_id, arena, str_len, topic_id, sequence, out=None, out_off=None,
                    status=None) -> Encoded:
        nf = LITE_FIELDS.get(int(template_id))
        if nf is None:
            raise SbeError(f"not a Lite template: {template_id}")
        arena = _dev(arena, torch.uint8, "arena")
        str_len = _dev(str_len, torch.int32, "str_len")
        topic_id = _dev(topic_id, torch.int32, "topic_id")
        sequence = _dev(sequence, torch.int64, "sequence")
        n = int(sequence.numel())
        if str_len.numel() != nf * n or topic_id.numel() != n:
            raise SbeError(f"str_len must have {nf} entries and topic_id one per record")
        cap = int(lib().sbe_lite_output_bound(n, int(arena.numel()), int(template_id)))
        out, out_off, status = self._outputs(n, cap, arena.device, out, out_off, status)
        batch = _LiteBatch(arena.data_ptr(), None, str_len.data_ptr(), topic_id.data_ptr(), sequence.data_ptr())
        torch.cuda.current_stream().synchronize()
        rc = lib().sbe_serve_encode_lite(self._h, ctypes.byref(batch), n, int(template_id), _ptr(out), out.numel(),
                                         _ptr(out_off), _ptr(status))
        _check(rc, "sbe_serve_encode_lite")
        return Encoded(out, out_off, None if status is None else status[:n])

    def decode(self, data, rec_off, mode=DEC_PARSE_MESSAGE, out: Decoded | None = None, seq=None) -> Decoded:
        data = _dev(data, torch.uint8, "data")
        rec_off = _dev(rec_off, torch.int64, "rec_off")
        n = int(rec_off.numel()) - 1
        if out is None:
            out = alloc_decoded(n, data.device)
        if seq is True:
            seq = torch.zeros(max(n, 1), dtype=torch.int64, device=data.device)
        if seq is not None:
            seq = _dev(seq, torch.int64, "seq")
        d = _Decoded(*(getattr(out, k).data_ptr() for k in ("status", "flags", "hdr", "ts", "view_off", "view_len")),
                     None if seq is None else seq.data_ptr())
        torch.cuda.current_stream().synchronize()
        _check(lib().sbe_serve_decode(self._h, _ptr(data), _ptr(rec_off), n, mode, ctypes.byref(d)),
               "sbe_serve_decode")
        keys = ("status", "flags", "hdr", "ts", "view_off", "view_len")
        out = Decoded(*(getattr(out, k)[:n] for k in keys))
        out.seq = None if seq is None else seq[:n]
        return out

    # host-memory inputs (numpy arrays), copied into the request slot: the *_host entry points
    def encode_topic_host(self, arena, str_len, timestamp, flags=0, ts_default=0, session=None, dev="cuda"):
        """TopicMessage (session=None) or session-framed (session=(term, session_id)) encode of host
        numpy inputs: arena uint8, str_len uint32 [n,5], timestamp uint64 [n]."""
        import numpy as np
        arena = np.ascontiguousarray(arena, np.uint8)
        str_len = np.ascontiguousarray(str_len, np.uint32).reshape(-1, 5)
        timestamp = np.ascontiguousarray(timestamp, np.uint64)
        n = int(timestamp.size)
        out, out_off, status = self._outputs(n, output_bound(n, int(arena.size), flags), torch.device(dev),
                                             None, None, None)
        torch.cuda.current_stream().synchronize()  # the fresh outputs may still be in use on torch's stream
        batch = _TmBatch(arena.ctypes.data if arena.size else None, None, str_len.ctypes.data, timestamp.ctypes.data)
        if session is None:
            rc = lib().sbe_serve_encode_topic_host(self._h, ctypes.byref(batch), n, ts_default & (2**64 - 1), flags,
                                                   _ptr(out), out.numel(), _ptr(out_off), _ptr(status))
        else:
            rc = lib().sbe_serve_encode_session_host(self._h, ctypes.byref(batch), n, ts_default & (2**64 - 1), flags,
                                                     int(session[0]), int(session[1]), _ptr(out), out.numel(),
                                                     _ptr(out_off), _ptr(status))
        _check(rc, "sbe_serve_encode_*_host")
        return Encoded(out, out_off, status[:n])

    def encode_lite_host(self, template_id, arena, str_len, topic_id, sequence, dev="cuda"):
        import numpy as np
        nf = LITE_FIELDS.get(int(template_id))
        if nf is None:
            raise SbeError(f"not a Lite template: {template_id}")
        arena = np.ascontiguousarray(arena, np.uint8)
        str_len = np.ascontiguousarray(str_len, np.uint32).reshape(-1, nf)
        topic_id = np.ascontiguousarray(topic_id, np.uint32)
        sequence = np.ascontiguousarray(sequence, np.uint64)
        n = int(sequence.size)
        cap = int(lib().sbe_lite_output_bound(n, int(arena.size), int(template_id)))
        out, out_off, status = self._outputs(n, cap, torch.device(dev), None, None, None)
        torch.cuda.current_stream().synchronize()  # the fresh outputs may still be in use on torch's stream
        batch = _LiteBatch(arena.ctypes.data if arena.size else None, None, str_len.ctypes.data, topic_id.ctypes.data,
                           sequence.ctypes.data)
        _check(lib().sbe_serve_encode_lite_host(self._h, ctypes.byref(batch), n, int(template_id), _ptr(out),
                                                out.numel(), _ptr(out_off), _ptr(status)), "sbe_serve_encode_lite_host")
        return Encoded(out, out_off, status[:n])

    def decode_host(self, data, rec_off, mode=DEC_PARSE_MESSAGE, seq=None, dev="cuda") -> Decoded:
        """Decode of host numpy inputs: data uint8, rec_off uint64 [n+1] (any base, no alignment)."""
        import numpy as np
        data = np.ascontiguousarray(data, np.uint8)
        rec_off = np.ascontiguousarray(rec_off, np.uint64)
        n = int(rec_off.size) - 1
        out = alloc_decoded(n, torch.device(dev))
        if seq is True:
            seq = torch.zeros(max(n, 1), dtype=torch.int64, device=dev)
        d = _Decoded(*(getattr(out, k).data_ptr() for k in ("status", "flags", "hdr", "ts", "view_off", "view_len")),
                     None if seq is None else seq.data_ptr())
        torch.cuda.current_stream().synchronize()
        _check(lib().sbe_serve_decode_host(self._h, data.ctypes.data if data.size else None, rec_off.ctypes.data, n,
                                           mode, ctypes.byref(d)), "sbe_serve_decode_host")
        keys = ("status", "flags", "hdr", "ts", "view_off", "view_len")
        out = Decoded(*(getattr(out, k)[:n] for k in keys))
        out.seq = None if seq is None else seq[:n]
        return out

    # planned encodes (several workgroups): the tile sums from host-side record sizes
    @staticmethod
    def tile_sums(layout, out_bytes, in_bytes, dev="cuda"):
        """sbe_enc_sums' output for records of the given output / input sizes (numpy u64 [n]):
        (tile_sums [T,2], sb_sums [S,2]) as int64 device tensors."""
        import numpy as np
        R = int(lib().sbe_encode_tile_records(int(layout)))
        SB = 128 * R
        n = int(out_bytes.size)
        po = np.zeros(n + 1, np.uint64)
        pi = np.zeros(n + 1, np.uint64)
        po[1:] = np.cumsum(out_bytes.astype(np.uint64))
        pi[1:] = np.cumsum(in_bytes.astype(np.uint64))
        if n == 0:
            ts = bs = np.zeros((1, 2), np.uint64)
        else:
            t0 = np.arange(0, n, R)
            b0 = (t0 // SB) * SB
            ts = np.stack([po[t0] - po[b0], pi[t0] - pi[b0]], 1)
            s0 = np.arange(0, n, SB)
            s1 = np.minimum(s0 + SB, n)
            bs = np.stack([po[s1] - po[s0], pi[s1] - pi[s0]], 1)
        cv = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
        return cv(ts), cv(bs)

    def encode_planned(self, layout, arena, str_len, timestamp, tile_sums, sb_sums, flags=0, ts_default=0,
                       session=None, template_id=None, topic_id=None) -> Encoded:
        """Planned encode on device tensors (packed input) with host-made tile sums (tile_sums())."""
        arena = _dev(arena, torch.uint8, "arena")
        str_len = _dev(str_len, torch.int32, "str_len")
        timestamp = _dev(timestamp, torch.int64, "timestamp")
        n = int(timestamp.numel())
        if layout == LAYOUT_LITE:
            cap = int(lib().sbe_lite_output_bound(n, int(arena.numel()), int(template_id)))
        else:
            cap = output_bound(n, int(arena.numel()), flags)
        out, out_off, status = self._outputs(n, cap, arena.device, None, None, None)
        torch.cuda.current_stream().synchronize()
        if layout == LAYOUT_LITE:
            batch = _LiteBatch(arena.data_ptr(), None, str_len.data_ptr(), _dev(topic_id, torch.int32, "topic_id").data_ptr(),
                               timestamp.data_ptr())
            rc = lib().sbe_serve_encode_lite_planned(self._h, ctypes.byref(batch), n, int(template_id), _ptr(out),
                                                     out.numel(), _ptr(out_off), _ptr(status), _ptr(tile_sums),
                                                     _ptr(sb_sums))
        elif layout == LAYOUT_SESSION:
            batch = _TmBatch(arena.data_ptr(), None, str_len.data_ptr(), timestamp.data_ptr())
            rc = lib().sbe_serve_encode_session_planned(self._h, ctypes.byref(batch), n, ts_default & (2**64 - 1),
                                                        flags, int(session[0]), int(session[1]), _ptr(out),
                                                        out.numel(), _ptr(out_off), _ptr(status), _ptr(tile_sums),
                                                        _ptr(sb_sums))
        else:
            batch = _TmBatch(arena.data_ptr(), None, str_len.data_ptr(), timestamp.data_ptr())
            rc = lib().sbe_serve_encode_topic_planned(self._h, ctypes.byref(batch), n, ts_default & (2**64 - 1), flags,
                                                      _ptr(out), out.numel(), _ptr(out_off), _ptr(status),
                                                      _ptr(tile_sums), _ptr(sb_sums))
        _check(rc, "sbe_serve_encode_*_planned")
        return Encoded(out, out_off, status[:n])

    @staticmethod
    def _outputs(n, cap, dev, out, out_off, status):
        if out is None:
            out = torch.empty(max(cap, 16), dtype=torch.uint8, device=dev)
        if out_off is None:
            out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        elif status is False:
            status = None
        return out, out_off, status
