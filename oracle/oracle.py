"""ctypes wrapper over oracle/psx_oracle.c — TEST INFRASTRUCTURE ONLY.

This is the parity checker.  It restates Server::ApplyOpLogUpdateVersion
(src/petuum_ps/server/server.cpp:120-179) and the row stores on the CPU.  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libpsx_oracle.so")
_lib = None

DENSE, SORTED_MAP, MAP = 0, 1, 2
F32, F64, I32, I64 = 0, 1, 2, 3
NP_DTYPE = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64}

ST_OK = 0


def build():
    """Compile the oracle with gcc (make)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "psx_oracle.c")
        if (not os.path.exists(_LIB_PATH)
                or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
        L.orc_server_create.restype = vp
        L.orc_server_destroy.argtypes = [vp]
        L.orc_register_sender.argtypes = [vp, i32]
        L.orc_table_create.argtypes = [vp, i32, ctypes.c_int, ctypes.c_int, ctypes.c_int, i64, i64]
        L.orc_apply_stream.argtypes = [vp, vp, sz, i32, ctypes.c_uint32]
        L.orc_apply_stream_once.argtypes = [vp, vp, sz, i32, ctypes.c_uint32]
        L.orc_sender_version.argtypes = [vp, i32]
        L.orc_sender_version.restype = i64
        L.orc_row_exists.argtypes = [vp, i32, i32]
        L.orc_row_dirty.argtypes = [vp, i32, i32]
        L.orc_num_rows.argtypes = [vp, i32]
        L.orc_num_rows.restype = i64
        L.orc_load_dense_rows.argtypes = [vp, i32, i64, i64, i64, vp]
        L.orc_read_dense_rows.argtypes = [vp, i32, i64, i64, i64, vp]
        L.orc_serialize_row.argtypes = [vp, i32, i32, vp, sz]
        L.orc_serialize_row.restype = i64
        L.orc_serialize_records.argtypes = [vp, i32, vp, i32, vp, sz]
        L.orc_serialize_records.restype = i64
        L.orc_get.argtypes = [vp, i32, i32, i32, vp]
        L.orc_row_inc.argtypes = [vp, i32, i32, i32, vp]
        L.orc_pack_stream.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, sz]
        L.orc_pack_stream.restype = sz
        L.orc_serialize_dirty.argtypes = [vp, vp, ctypes.c_int, vp, sz, ctypes.c_int]
        L.orc_serialize_dirty.restype = i64
        L.orc_table_set_importance.argtypes = [vp, i32, ctypes.c_int]
        L.orc_table_set_version_maintain.argtypes = [vp, i32, ctypes.c_int]
        L.orc_table_set_f16_records.argtypes = [vp, i32, ctypes.c_int]
        L.orc_table_set_f16_rows.argtypes = [vp, i32, ctypes.c_int]
        L.orc_float_to_half.argtypes = [ctypes.c_float]
        L.orc_float_to_half.restype = ctypes.c_uint16
        L.orc_floats_to_halves.argtypes = [vp, vp, sz]
        L.orc_half_to_float.argtypes = [ctypes.c_uint16]
        L.orc_half_to_float.restype = ctypes.c_float
        L.orc_row_version.argtypes = [vp, i32, i32, ctypes.POINTER(ctypes.c_uint64)]
        L.orc_table_set_adarevision.argtypes = [vp, i32, ctypes.c_float, ctypes.c_int, ctypes.c_uint64, i32]
        L.orc_row_sent.argtypes = [vp, i32, i32, i32]
        L.orc_ada_state.argtypes = [vp, i32, i32, vp, vp, vp]
        L.orc_ada_num_snapshots.argtypes = [vp, i32]
        L.orc_ada_num_snapshots.restype = i64
        L.orc_rng_normals.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_float, i64, vp]
        L.orc_row_importance.argtypes = [vp, i32, i32, ctypes.POINTER(ctypes.c_double)]
        L.orc_serialize_partial.argtypes = [vp, vp, ctypes.c_int, vp, vp, sz, ctypes.c_int]
        L.orc_serialize_partial.restype = i64
        L.orc_partition_server.argtypes = [i32, i32, i32, i32]
        L.orc_partition_server.restype = i32
        L.orc_clock_until.argtypes = [vp, i32, i32]
        L.orc_clock_until.restype = i32
        L.orc_min_clock.argtypes = [vp]
        L.orc_min_clock.restype = i32
        L.orc_subscribe.argtypes = [vp, i32, i32, i32]
        L.orc_row_subs.argtypes = [vp, i32, i32]
        L.orc_row_subs.restype = ctypes.c_uint64
        L.orc_serialize_push.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_int]
        L.orc_serialize_push.restype = i64
        _lib = L
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class OracleServer:
    """Mirror of petuum::Server (server.hpp) restricted to the apply path."""

    def __init__(self, bg_ids=()):
        self._L = lib()
        self._s = self._L.orc_server_create()
        self.tables = {}
        for bg in bg_ids:
            self.register_sender(bg)

    def close(self):
        if self._s:
            self._L.orc_server_destroy(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def register_sender(self, bg):
        assert self._L.orc_register_sender(self._s, bg) == ST_OK

    def create_table(self, table_id, kind, dtype, row_capacity, oplog_dense_serialized=True,
                     dense_row_oplog_capacity=None, accum_importance=False, version_maintain=False,
                     f16_records=False, f16_rows=False):
        cap = row_capacity if dense_row_oplog_capacity is None else dense_row_oplog_capacity
        st = self._L.orc_table_create(self._s, table_id, kind, dtype,
                                      1 if oplog_dense_serialized else 0, row_capacity, cap)
        assert st == ST_OK, st
        if accum_importance:
            assert self._L.orc_table_set_importance(self._s, table_id, 1) == ST_OK
        if version_maintain:
            assert self._L.orc_table_set_version_maintain(self._s, table_id, 1) == ST_OK
        if f16_records:
            assert self._L.orc_table_set_f16_records(self._s, table_id, 1) == ST_OK
        if f16_rows:
            assert self._L.orc_table_set_f16_rows(self._s, table_id, 1) == ST_OK
        self.tables[table_id] = (kind, dtype, row_capacity)

    def importance(self, table_id, row_id):
        out = ctypes.c_double()
        assert self._L.orc_row_importance(self._s, table_id, row_id, ctypes.byref(out)) == ST_OK
        return out.value

    def row_version(self, table_id, row_id):
        """VersionServerRow::get_version (version_server_row.hpp:66); 0 otherwise."""
        out = ctypes.c_uint64()
        assert self._L.orc_row_version(self._s, table_id, row_id, ctypes.byref(out)) == ST_OK
        return out.value

    def set_adarevision(self, table_id, init_step_size=0.1, gaussian_init=True, old_grad_upper_bound=10000,
                        push_clients=1):
        """AdaRevisionServerTableLogic on a table (adarevision_server_table_logic.cpp); returns the status."""
        return self._L.orc_table_set_adarevision(self._s, table_id, init_step_size, 1 if gaussian_init else 0,
                                                 old_grad_upper_bound, push_clients)

    def row_sent(self, table_id, row_id, num_clients=1):
        """Server::RowSent (server.cpp:436-441)."""
        return self._L.orc_row_sent(self._s, table_id, row_id, num_clients)

    def ada_state(self, table_id, row_id):
        """(accum_gradients_, z_, z_max_) of a row, or None if the row does not exist."""
        cap = self.tables[table_id][2]
        a, z, m = (np.zeros(cap, np.float32) for _ in range(3))
        if self._L.orc_ada_state(self._s, table_id, row_id, _ptr(a), _ptr(z), _ptr(m)) != ST_OK:
            return None
        return a, z, m

    def ada_num_snapshots(self, table_id):
        return self._L.orc_ada_num_snapshots(self._s, table_id)

    def apply_stream(self, data, bg, version):
        """Server::ApplyOpLogUpdateVersion; returns the status code."""
        buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        buf = np.ascontiguousarray(buf)
        return self._L.orc_apply_stream(self._s, _ptr(buf) if buf.size else None,
                                        buf.size, bg, version)

    def apply_stream_once(self, data, bg, version):
        """The reference's one-pass loop shape (orc_apply_stream_once): for timing only —
        a malformed stream is found after the records before it were applied."""
        buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        buf = np.ascontiguousarray(buf)
        return self._L.orc_apply_stream_once(self._s, _ptr(buf) if buf.size else None,
                                             buf.size, bg, version)

    def sender_version(self, bg):
        return self._L.orc_sender_version(self._s, bg)

    def row_exists(self, table_id, row_id):
        return bool(self._L.orc_row_exists(self._s, table_id, row_id))

    def row_dirty(self, table_id, row_id):
        return bool(self._L.orc_row_dirty(self._s, table_id, row_id))

    def num_rows(self, table_id):
        return self._L.orc_num_rows(self._s, table_id)

    def load_dense_rows(self, table_id, first_row, rows, stride=1):
        kind, dt, cap = self.tables[table_id]
        a = np.ascontiguousarray(rows, dtype=NP_DTYPE[dt]).reshape(-1, cap)
        assert self._L.orc_load_dense_rows(self._s, table_id, first_row, stride, a.shape[0], _ptr(a)) == 0

    def read_dense_rows(self, table_id, first_row, n, stride=1):
        kind, dt, cap = self.tables[table_id]
        out = np.zeros((n, cap), dtype=NP_DTYPE[dt])
        assert self._L.orc_read_dense_rows(self._s, table_id, first_row, stride, n, _ptr(out)) == 0
        return out

    def serialize_row(self, table_id, row_id):
        kind, dt, cap = self.tables[table_id]
        nb = max(64, cap * 16)
        while True:
            out = np.zeros(nb, dtype=np.uint8)
            r = self._L.orc_serialize_row(self._s, table_id, row_id, _ptr(out), nb)
            if r == -2:
                nb *= 4
                continue
            return None if r == -1 else out[:r].tobytes()

    def serialize_records(self, table_id, row_ids):
        ids = np.ascontiguousarray(row_ids, dtype=np.int32)
        nb = 1 << 16
        while True:
            out = np.zeros(nb, dtype=np.uint8)
            r = self._L.orc_serialize_records(self._s, table_id, _ptr(ids), ids.size, _ptr(out), nb)
            if r == -2:
                nb *= 4
                continue
            assert r >= 0, r
            return out[:r].tobytes()

    def serialize_dirty(self, table_ids, clear=True):
        """Push-message body for every dirty row (server.cpp:189-309), tables in order."""
        tids = np.ascontiguousarray(table_ids, dtype=np.int32)
        nb = 1 << 16
        while True:
            out = np.zeros(nb, dtype=np.uint8)
            r = self._L.orc_serialize_dirty(self._s, _ptr(tids), tids.size, _ptr(out), nb, 1 if clear else 0)
            if r == -2:
                nb *= 4
                continue
            assert r >= 0, r
            return out[:r].tobytes()

    def serialize_partial(self, table_ids, upper_bounds, clear=True):
        """Partial push body (server.cpp:311-420); b"" when nothing is sent."""
        tids = np.ascontiguousarray(table_ids, dtype=np.int32)
        ub = np.ascontiguousarray(upper_bounds, dtype=np.int64)
        nb = 1 << 16
        while True:
            out = np.zeros(nb, dtype=np.uint8)
            r = self._L.orc_serialize_partial(self._s, _ptr(tids), tids.size, _ptr(ub), _ptr(out), nb,
                                              1 if clear else 0)
            if r == -2:
                nb *= 4
                continue
            assert r >= 0, r
            return out[:r].tobytes()

    def clock_until(self, bg, clock):
        """Server::ClockUntil (server.cpp:62-79): the new min clock if it advanced, else 0."""
        r = self._L.orc_clock_until(self._s, bg, clock)
        assert r >= 0, "unknown sender"
        return r

    def min_clock(self):
        return self._L.orc_min_clock(self._s)

    def subscribe(self, table_id, row_id, client_id):
        """FindCreateRow + RowSubscribe (server_thread.cpp:185-200)."""
        assert self._L.orc_subscribe(self._s, table_id, row_id, client_id) == ST_OK

    def row_subs(self, table_id, row_id):
        return self._L.orc_row_subs(self._s, table_id, row_id)

    def serialize_push(self, table_ids, num_clients, clear=True):
        """Server::CreateSendServerPushRowMsgs with per-client subscriptions
        (server.cpp:189-309, server_table.cpp:197-261): one body per client."""
        tids = np.ascontiguousarray(table_ids, dtype=np.int32)
        nb = 1 << 16
        while True:
            bufs = [np.zeros(nb, dtype=np.uint8) for _ in range(num_clients)]
            ptrs = (ctypes.c_void_p * num_clients)(*[b.ctypes.data for b in bufs])
            caps = np.full(num_clients, nb, dtype=np.uint64)
            used = np.zeros(num_clients, dtype=np.int64)
            r = self._L.orc_serialize_push(self._s, _ptr(tids), tids.size, num_clients,
                                           ctypes.cast(ptrs, ctypes.c_void_p), _ptr(caps), _ptr(used),
                                           1 if clear else 0)
            if r == -2:
                nb = int(max(used.max(), nb)) * 2
                continue
            assert r == 0, r
            return [b[:u].tobytes() for b, u in zip(bufs, used)]

    def get(self, table_id, row_id, col):
        kind, dt, cap = self.tables[table_id]
        out = np.zeros(1, dtype=NP_DTYPE[dt])
        assert self._L.orc_get(self._s, table_id, row_id, col, _ptr(out)) == 0
        return out[0]

    def row_inc(self, table_id, row_id, col, delta):
        kind, dt, cap = self.tables[table_id]
        d = np.array([delta], dtype=NP_DTYPE[dt])
        assert self._L.orc_row_inc(self._s, table_id, row_id, col, _ptr(d)) == 0


def pack_stream(tables):
    """Build one ClientSendOpLogMsg payload with the reference packer's layout.

    tables: list of dicts {table_id, dtype, dense_serialized, row_ids (int32[n]),
    oplogs (V[n, capacity])} — restates RowOpLogSerializer/OpLogSerializer
    (row_oplog_serializer.hpp:139-166, oplog_serializer.hpp:12-37).
    """
    L = lib()
    n = len(tables)
    tid = np.array([t["table_id"] for t in tables], dtype=np.int32)
    dts = np.array([t["dtype"] for t in tables], dtype=np.int32)
    ds = np.array([1 if t["dense_serialized"] else 0 for t in tables], dtype=np.int32)
    ops = [np.ascontiguousarray(t["oplogs"], dtype=NP_DTYPE[t["dtype"]]) for t in tables]
    caps = np.array([o.shape[1] if o.ndim == 2 else 0 for o in ops], dtype=np.int64)
    rids = [np.ascontiguousarray(t["row_ids"], dtype=np.int32) for t in tables]
    nrows = np.array([r.size for r in rids], dtype=np.int64)
    rid_ptrs = (ctypes.c_void_p * max(n, 1))(*[r.ctypes.data for r in rids])
    op_ptrs = (ctypes.c_void_p * max(n, 1))(*[o.ctypes.data for o in ops])
    total = L.orc_pack_stream(n, _ptr(tid), _ptr(dts), _ptr(ds), _ptr(caps), _ptr(nrows),
                              ctypes.cast(rid_ptrs, ctypes.c_void_p),
                              ctypes.cast(op_ptrs, ctypes.c_void_p), None, 0)
    assert total != ctypes.c_size_t(-1).value
    if total == 0:
        return b""
    out = np.zeros(total, dtype=np.uint8)
    w = L.orc_pack_stream(n, _ptr(tid), _ptr(dts), _ptr(ds), _ptr(caps), _ptr(nrows),
                          ctypes.cast(rid_ptrs, ctypes.c_void_p),
                          ctypes.cast(op_ptrs, ctypes.c_void_p), _ptr(out), total)
    assert w == total
    return out.tobytes()


def rng_normals(seed, mean, stddev, n):
    """First n draws of the restated std::normal_distribution<float>(mean, stddev) on
    std::mt19937(seed) (the generator AdaRevisionServerTableLogic uses)."""
    out = np.zeros(n, np.float32)
    lib().orc_rng_normals(seed, mean, stddev, n, _ptr(out))
    return out


def partition_server(row_id, num_channels, num_clients, channel):
    return lib().orc_partition_server(row_id, num_channels, num_clients, channel)
