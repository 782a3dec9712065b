"""ctypes binding of include/psx.h (libpsx.so, built in-tree for gfx950).

There is no fallback: if libpsx.so is missing or cannot be loaded, importing the
binding raises.  The product path never touches oracle/.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# PSX_LIB: another in-tree build of the library (A/B runs of two builds on one box,
# tools/gpu_run.sh c3lib); default the package's own libpsx.so
LIB_PATH = os.environ.get("PSX_LIB") or os.path.join(_HERE, "libpsx.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "psx.h")

PSX_OK = 0
STATUS_NAMES = {
    0: "PSX_OK", 1: "PSX_ERR_INVALID_ARG", 2: "PSX_ERR_VERSION", 3: "PSX_ERR_UNKNOWN_TABLE",
    4: "PSX_ERR_MALFORMED", 5: "PSX_ERR_ROW_RANGE", 6: "PSX_ERR_CAPACITY", 7: "PSX_ERR_DEVICE",
    8: "PSX_ERR_OOM", 9: "PSX_ERR_BUFFER_TOO_SMALL", 10: "PSX_ERR_UNSUPPORTED",
    11: "PSX_ERR_SENDER", 12: "PSX_ERR_NO_DEVICE", 13: "PSX_ERR_STATE",
}
ROW_DENSE, ROW_SORTED_MAP, ROW_MAP = 0, 1, 2
F32, F64, I32, I64 = 0, 1, 2, 3
MAX_FUSED_STREAMS = 16
MAX_CLIENTS = 64
# TableInfo.row_oplog_type (configs.hpp:35-40)
DENSE_ROW_OPLOG, SPARSE_ROW_OPLOG, SPARSE_VECTOR_ROW_OPLOG, DENSE_ROW_OPLOG_FLOAT16 = 0, 1, 2, 3


class psx_table_config(ctypes.Structure):
    _fields_ = [
        ("table_id", ctypes.c_int32),
        ("row_kind", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("oplog_dense_serialized", ctypes.c_int32),
        ("row_capacity", ctypes.c_int64),
        ("dense_row_oplog_capacity", ctypes.c_int64),
        ("row_offset", ctypes.c_int64),
        ("row_stride", ctypes.c_int64),
        ("max_rows", ctypes.c_int64),
        ("max_entries", ctypes.c_int64),
        ("accum_importance", ctypes.c_int32),
        ("version_maintain", ctypes.c_int32),
        ("server_push_row_upper_bound", ctypes.c_int64),
        ("row_oplog_type", ctypes.c_int32),
        ("row_bytes_f16", ctypes.c_int32),
    ]


class psx_stream(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("size", ctypes.c_size_t),
        ("bg_id", ctypes.c_int32),
        ("version", ctypes.c_uint32),
    ]


class psx_pack_table(ctypes.Structure):
    _fields_ = [
        ("table_id", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("dense_serialized", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("capacity", ctypes.c_int64),
        ("num_rows", ctypes.c_int64),
        ("row_ids", ctypes.c_void_p),
        ("oplogs", ctypes.c_void_p),
    ]


class psx_adarevision_config(ctypes.Structure):
    _fields_ = [
        ("init_step_size", ctypes.c_float),
        ("gaussian_init", ctypes.c_int32),
        ("old_grad_upper_bound", ctypes.c_uint64),
        ("push_clients", ctypes.c_int32),
        ("max_snapshots_per_row", ctypes.c_int32),
    ]


class psx_oplog_msg_header(ctypes.Structure):
    _fields_ = [
        ("seq_num", ctypes.c_uint64),
        ("ack_num", ctypes.c_uint64),
        ("avai_size", ctypes.c_uint64),
        ("is_clock", ctypes.c_int32),
        ("client_id", ctypes.c_int32),
        ("version", ctypes.c_uint32),
        ("bg_clock", ctypes.c_int32),
    ]


class psx_push_msg_header(ctypes.Structure):
    _fields_ = [
        ("seq_num", ctypes.c_uint64),
        ("ack_num", ctypes.c_uint64),
        ("avai_size", ctypes.c_uint64),
        ("clock", ctypes.c_int32),
        ("version", ctypes.c_uint32),
        ("is_clock", ctypes.c_int32),
    ]


OPLOG_MSG_HEADER_BYTES = 41
PUSH_MSG_HEADER_BYTES = 37
COMPAT_INT32_STREAM_OFFSETS = 1


class psx_apply_stats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("messages", ctypes.c_uint64), ("oplog_bytes", ctypes.c_uint64),
                ("apply_sec", ctypes.c_double), ("settled_calls", ctypes.c_uint64)]


class PsxError(RuntimeError):
    def __init__(self, status, msg):
        self.status = status
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")


_lib = None


def header_functions():
    """Names of every function declared in include/*.h."""
    inc = os.path.dirname(HEADER_PATH)
    src = "".join(open(os.path.join(inc, f)).read() for f in sorted(os.listdir(inc)) if f.endswith(".h"))
    return sorted(set(re.findall(r"\b(psx_[a-z_0-9]+)\s*\(", src)))


def load():
    """Load libpsx.so; raises OSError if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built: run `make -C parameter_server_amd/csrc` "
                      "or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32, sz = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                             ctypes.c_uint32, ctypes.c_size_t)
    P = ctypes.POINTER
    sigs = {
        "psx_abi_version": ([], i32),
        "psx_device_count": ([P(i32)], ctypes.c_int),
        "psx_ctx_create": ([i32, i32, P(vp)], ctypes.c_int),
        "psx_ctx_destroy": ([vp], ctypes.c_int),
        "psx_ctx_set_stream": ([vp, vp], ctypes.c_int),
        "psx_ctx_get_stream": ([vp], vp),
        "psx_register_sender": ([vp, i32], ctypes.c_int),
        "psx_sender_version": ([vp, i32, P(i64)], ctypes.c_int),
        "psx_table_create": ([vp, P(psx_table_config)], ctypes.c_int),
        "psx_table_load_rows": ([vp, i32, i64, i64, vp, i32], ctypes.c_int),
        "psx_table_read_rows": ([vp, i32, i64, i64, vp, i32], ctypes.c_int),
        "psx_row_flags": ([vp, i32, i64, i64, vp], ctypes.c_int),
        "psx_clear_dirty": ([vp, i32], ctypes.c_int),
        "psx_apply_stream": ([vp, vp, sz, i32, u32], ctypes.c_int),
        "psx_apply_streams_device": ([vp, P(psx_stream), i32], ctypes.c_int),
        "psx_apply_indexed": ([vp, P(psx_stream), P(vp), i32], ctypes.c_int),
        "psx_apply_indexed_rows": ([vp, P(psx_stream), P(vp), P(vp), i32], ctypes.c_int),
        "psx_sync": ([vp], ctypes.c_int),
        "psx_serialize_rows": ([vp, i32, vp, i32, vp, sz, P(sz)], ctypes.c_int),
        "psx_serialize_dirty": ([vp, vp, sz, P(sz), i32, i32], ctypes.c_int),
        "psx_serialize_partial": ([vp, vp, sz, P(sz), i32, i32], ctypes.c_int),
        "psx_row_importance": ([vp, i32, i64, i64, vp], ctypes.c_int),
        "psx_row_versions": ([vp, i32, i64, i64, vp], ctypes.c_int),
        "psx_table_set_adarevision": ([vp, i32, P(psx_adarevision_config)], ctypes.c_int),
        "psx_row_sent": ([vp, i32, vp, i32, i32], ctypes.c_int),
        "psx_adarevision_state": ([vp, i32, i64, i64, vp, vp, vp, P(ctypes.c_uint64)], ctypes.c_int),
        "psx_pack_stream": ([vp, P(psx_pack_table), i32, vp, sz, P(sz), vp], ctypes.c_int),
        "psx_pack_stream_indexed": ([vp, P(psx_pack_table), i32, vp, sz, P(sz), vp, vp], ctypes.c_int),
        "psx_clock_until": ([vp, i32, i32, P(i32)], ctypes.c_int),
        "psx_min_clock": ([vp, P(i32)], ctypes.c_int),
        "psx_sender_clock": ([vp, i32, P(i32)], ctypes.c_int),
        "psx_set_num_clients": ([vp, i32], ctypes.c_int),
        "psx_row_subscribe": ([vp, i32, vp, i32, i32], ctypes.c_int),
        "psx_row_subscriptions": ([vp, i32, i64, i64, vp], ctypes.c_int),
        "psx_serialize_push": ([vp, vp, vp, vp, i32, i32], ctypes.c_int),
        "psx_apply_push_body": ([vp, vp, sz, i32, i32], ctypes.c_int),
        "psx_encode_oplog_header": ([P(psx_oplog_msg_header), vp], ctypes.c_int),
        "psx_decode_oplog_header": ([vp, sz, P(psx_oplog_msg_header)], ctypes.c_int),
        "psx_encode_push_header": ([P(psx_push_msg_header), vp], ctypes.c_int),
        "psx_decode_push_header": ([vp, sz, P(psx_push_msg_header)], ctypes.c_int),
        "psx_ctx_set_compat": ([vp, i32], ctypes.c_int),
        "psx_ctx_set_pipeline": ([vp, i32], ctypes.c_int),
        "psx_ctx_set_seam": ([vp, i32], ctypes.c_int),
        "psx_handle_oplog_msg": ([vp, vp, sz, i32, P(i32)], ctypes.c_int),
        "psx_last_error": ([vp], ctypes.c_char_p),
        "psx_status_string": ([ctypes.c_int], ctypes.c_char_p),
        "psx_timing_enable": ([vp, i32], ctypes.c_int),
        "psx_timing_read": ([vp, ctypes.c_char_p, P(ctypes.c_double), P(i64)], ctypes.c_int),
        "psx_timing_reset": ([vp], ctypes.c_int),
        "psx_ctx_stats": ([vp, P(psx_apply_stats), i32], ctypes.c_int),
        "psx_split_stream": ([vp, vp, sz, vp, i32, vp, vp, sz, vp], ctypes.c_int),
        "psx_split_stream_formats": ([vp, P(psx_table_config), i32, vp, sz, vp, i32, vp, vp, sz, vp], ctypes.c_int),
        "psx_comm_unique_id": ([vp], ctypes.c_int),
        "psx_comm_create": ([vp, i32, i32, i32, P(vp)], ctypes.c_int),
        "psx_comm_destroy": ([vp], ctypes.c_int),
        "psx_comm_last_error": ([vp], ctypes.c_char_p),
        "psx_exchange_sizes": ([vp, vp, vp, vp], ctypes.c_int),
        "psx_exchange_streams": ([vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "psx_exchange_sizes_async": ([vp, vp, vp, vp], ctypes.c_int),
        "psx_exchange_streams_v": ([vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "psx_comm_info": ([vp, P(i32), P(i32), P(i32), P(i32), ctypes.c_char_p, sz], ctypes.c_int),
        "psx_comm_peer_bytes": ([vp, vp, vp, i32], ctypes.c_int),
        "psx_debug_set_variant": ([i32, i32], i32),
        "psx_debug_get_variant": ([i32], i32),
        "psx_debug_walk_trace": ([vp, vp, ctypes.c_int64], ctypes.c_int64),
        "psx_debug_read_sweep": ([vp, ctypes.c_int64, i32], ctypes.c_double),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L
