"""Host-side mirror of the reference's server apply interface, over the C ABI.

Names follow src/petuum_ps/server/server.hpp (Server::Init, CreateTable,
ApplyOpLogUpdateVersion, GetBgVersion) and configs.hpp (TableInfo), so the parity
tests read like the reference's own call sites (server_thread.cpp:224-299).  Errors
that the reference turns into glog CHECK aborts raise PsxError here.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import PsxError, psx_stream, psx_table_config

NP_DTYPE = {_abi.F32: np.float32, _abi.F64: np.float64, _abi.I32: np.int32, _abi.I64: np.int64}


@dataclass
class TableInfo:
    """The TableInfo fields the apply path reads (configs.hpp:170-210) plus shard geometry."""
    row_kind: int = _abi.ROW_DENSE
    dtype: int = _abi.F32
    row_capacity: int = 0
    oplog_dense_serialized: bool = True
    dense_row_oplog_capacity: int = 0   # 0 -> row_capacity
    row_offset: int = 0
    row_stride: int = 1
    max_rows: int = 0
    max_entries: int = 0
    accum_importance: bool = False          # SSPAggr + RelativeMagnitude/FIFO_N_ReMag (server_table.cpp:26-47)
    server_push_row_upper_bound: int = 0    # configs.hpp:181; 0 -> 100
    version_maintain: bool = False          # VersionDenseRowOpLog records + VersionServerRow rows (configs.hpp:207)
    row_oplog_type: int = 0                 # RowOpLogType (configs.hpp:35-40); 3 = float16 dense records
    row_bytes_f16: bool = False             # DenseRowFloat16 rows: served as binary16 (dense_row_float16.hpp:13)


def table_config(table_id, info: TableInfo):
    """The psx_table_config of a TableInfo (psx_table_create / psx_split_stream_formats)."""
    return psx_table_config(
        table_id=table_id, row_kind=info.row_kind, dtype=info.dtype,
        oplog_dense_serialized=1 if info.oplog_dense_serialized else 0,
        row_capacity=info.row_capacity,
        dense_row_oplog_capacity=info.dense_row_oplog_capacity or info.row_capacity,
        row_offset=info.row_offset, row_stride=info.row_stride, max_rows=info.max_rows,
        max_entries=info.max_entries, accum_importance=1 if info.accum_importance else 0,
        server_push_row_upper_bound=info.server_push_row_upper_bound,
        version_maintain=1 if info.version_maintain else 0, row_oplog_type=info.row_oplog_type,
        row_bytes_f16=1 if info.row_bytes_f16 else 0)


def _check(L, ctx, st):
    if st != _abi.PSX_OK:
        msg = L.psx_last_error(ctx).decode() if ctx else ""
        raise PsxError(st, msg)


class Server:
    """One shard (one reference ServerThread's Server) on one GPU."""

    def __init__(self, device=0, server_id=1, bg_ids=()):
        self._L = _abi.load()
        self._ctx = ctypes.c_void_p()
        _check(self._L, None, self._L.psx_ctx_create(device, server_id, ctypes.byref(self._ctx)))
        self.device = device
        self.tables = {}
        for bg in bg_ids:
            self.register_sender(bg)

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if self._ctx:
            self._L.psx_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._ctx

    def register_sender(self, bg_id):
        _check(self._L, self._ctx, self._L.psx_register_sender(self._ctx, bg_id))

    def set_stream(self, hip_stream_handle):
        _check(self._L, self._ctx, self._L.psx_ctx_set_stream(self._ctx, hip_stream_handle))

    def set_seam(self, mode):
        """psx_ctx_set_seam: 0 (default) ApplyOpLogUpdateVersion returns once its bytes are
        copied to HBM and the apply is enqueued (device errors surface at the next sync);
        1 every host call also settles, so its own errors come back from it."""
        _check(self._L, self._ctx, self._L.psx_ctx_set_seam(self._ctx, int(mode)))

    def set_pipeline(self, mode):
        """psx_ctx_set_pipeline: 0 off, 1 calls whose dense tables are all placed from
        record-row lists, 2 every call.  Opt-in: a call's messages must be complete when
        the call is made (its index stage may overlap the previous call's apply)."""
        _check(self._L, self._ctx, self._L.psx_ctx_set_pipeline(self._ctx, int(mode)))

    # -- Server API (server.hpp) ----------------------------------------------
    def CreateTable(self, table_id, info: TableInfo):
        cfg = table_config(table_id, info)
        _check(self._L, self._ctx, self._L.psx_table_create(self._ctx, ctypes.byref(cfg)))
        self.tables[table_id] = info

    def ApplyOpLogUpdateVersion(self, oplog, oplog_size, bg_thread_id, version):
        """Host-bytes apply, as Server::ApplyOpLogUpdateVersion (server.cpp:120-179)."""
        buf = np.frombuffer(oplog, dtype=np.uint8) if isinstance(oplog, (bytes, bytearray)) else oplog
        buf = np.ascontiguousarray(buf)
        ptr = ctypes.c_void_p(buf.ctypes.data) if oplog_size else None
        _check(self._L, self._ctx,
               self._L.psx_apply_stream(self._ctx, ptr, oplog_size, bg_thread_id, version))

    def GetBgVersion(self, bg_thread_id):
        v = ctypes.c_int64()
        _check(self._L, self._ctx, self._L.psx_sender_version(self._ctx, bg_thread_id, ctypes.byref(v)))
        return v.value

    # -- device-resident path -----------------------------------------------------
    def apply_device(self, streams):
        """streams: sequence of (device_ptr, nbytes, bg_id, version); applied in order."""
        n = len(streams)
        arr = (psx_stream * n)()
        for i, (ptr, nbytes, bg, ver) in enumerate(streams):
            arr[i].data = ptr
            arr[i].size = nbytes
            arr[i].bg_id = bg
            arr[i].version = ver
        _check(self._L, self._ctx, self._L.psx_apply_streams_device(self._ctx, arr, n))

    def apply_indexed(self, streams, record_offsets):
        """apply_device with producer record indexes: record_offsets[i] is the device
        pointer of message i's uint64 row-id offsets (psx_pack_stream's), or None."""
        n = len(streams)
        arr = (psx_stream * n)()
        for i, (ptr, nbytes, bg, ver) in enumerate(streams):
            arr[i].data = ptr
            arr[i].size = nbytes
            arr[i].bg_id = bg
            arr[i].version = ver
        offs = (ctypes.c_void_p * n)(*[o or None for o in record_offsets])
        _check(self._L, self._ctx, self._L.psx_apply_indexed(self._ctx, arr, offs, n))

    def apply_indexed_rows(self, streams, record_rows, record_offsets=None):
        """apply_device with producer record-row lists (psx_apply_indexed_rows):
        record_rows[i] is the device pointer of message i's int32 row ids in record order
        (psx_pack_stream_indexed's), or None; record_offsets as in apply_indexed."""
        n = len(streams)
        arr = (psx_stream * n)()
        for i, (ptr, nbytes, bg, ver) in enumerate(streams):
            arr[i].data = ptr
            arr[i].size = nbytes
            arr[i].bg_id = bg
            arr[i].version = ver
        rows = (ctypes.c_void_p * n)(*[r or None for r in record_rows])
        offs = (ctypes.c_void_p * n)(*[o or None for o in record_offsets]) if record_offsets else None
        _check(self._L, self._ctx, self._L.psx_apply_indexed_rows(self._ctx, arr, offs, rows, n))

    def sync(self):
        _check(self._L, self._ctx, self._L.psx_sync(self._ctx))

    # -- rows --------------------------------------------------------------------------
    def _np(self, table_id):
        return NP_DTYPE[self.tables[table_id].dtype]

    def load_rows(self, table_id, first_row, rows, on_device_ptr=None, num_rows=None):
        if on_device_ptr is not None:
            _check(self._L, self._ctx, self._L.psx_table_load_rows(
                self._ctx, table_id, first_row, num_rows, on_device_ptr, 1))
            return
        info = self.tables[table_id]
        a = np.ascontiguousarray(rows, dtype=self._np(table_id)).reshape(-1, info.row_capacity)
        _check(self._L, self._ctx, self._L.psx_table_load_rows(
            self._ctx, table_id, first_row, a.shape[0], ctypes.c_void_p(a.ctypes.data), 0))

    def read_rows_device(self, table_id, first_row, num_rows, out):
        """psx_table_read_rows into a CUDA tensor of num_rows x row_capacity values (absent
        rows read as zero); synchronous."""
        import torch
        info = self.tables[table_id]
        assert out.is_cuda and out.is_contiguous() and out.numel() == num_rows * info.row_capacity
        assert out.element_size() == np.dtype(self._np(table_id)).itemsize
        _check(self._L, self._ctx, self._L.psx_table_read_rows(
            self._ctx, table_id, first_row, num_rows, out.data_ptr(), 1))
        _check(self._L, self._ctx, self._L.psx_sync(self._ctx))
        torch.cuda.synchronize(out.device)
        return out

    def read_rows(self, table_id, first_row, num_rows):
        info = self.tables[table_id]
        out = np.zeros((num_rows, info.row_capacity), dtype=self._np(table_id))
        _check(self._L, self._ctx, self._L.psx_table_read_rows(
            self._ctx, table_id, first_row, num_rows, ctypes.c_void_p(out.ctypes.data), 0))
        return out

    def row_flags(self, table_id, first_row, num_rows):
        out = np.zeros(num_rows, dtype=np.uint8)
        _check(self._L, self._ctx, self._L.psx_row_flags(
            self._ctx, table_id, first_row, num_rows, ctypes.c_void_p(out.ctypes.data)))
        return out

    def row_importance(self, table_id, first_row, num_rows):
        """ServerRow::get_importance for a row range (server_row.hpp:120-122)."""
        out = np.zeros(num_rows, dtype=np.float64)
        _check(self._L, self._ctx, self._L.psx_row_importance(
            self._ctx, table_id, first_row, num_rows, ctypes.c_void_p(out.ctypes.data)))
        return out

    def row_versions(self, table_id, first_row, num_rows):
        """VersionServerRow::get_version for a row range (version_server_row.hpp:66)."""
        out = np.zeros(num_rows, dtype=np.uint64)
        _check(self._L, self._ctx, self._L.psx_row_versions(
            self._ctx, table_id, first_row, num_rows, ctypes.c_void_p(out.ctypes.data)))
        return out

    def set_adarevision(self, table_id, init_step_size=0.1, gaussian_init=True, old_grad_upper_bound=10000,
                        push_clients=1, max_snapshots_per_row=4):
        """Attach AdaRevisionServerTableLogic to a table (adarevision_server_table_logic.cpp:19-36;
        defaults are its gflags, :8-10)."""
        cfg = _abi.psx_adarevision_config(float(init_step_size), int(bool(gaussian_init)),
                                          int(old_grad_upper_bound), int(push_clients),
                                          int(max_snapshots_per_row))
        _check(self._L, self._ctx, self._L.psx_table_set_adarevision(self._ctx, table_id, ctypes.byref(cfg)))

    def row_sent(self, table_id, row_ids, num_clients):
        """Server::RowSent -> ServerRowSent (server.cpp:436-441)."""
        ids = np.ascontiguousarray(row_ids, dtype=np.int32)
        _check(self._L, self._ctx, self._L.psx_row_sent(self._ctx, table_id, ctypes.c_void_p(ids.ctypes.data),
                                                          int(ids.size), int(num_clients)))

    def adarevision_state(self, table_id, first_row, num_rows):
        """(accum_gradients, z, z_max) [num_rows, row_capacity] f32 and the live snapshot count."""
        cap = self.tables[table_id].row_capacity
        acc, z, zm = (np.zeros((num_rows, cap), np.float32) for _ in range(3))
        live = ctypes.c_uint64(0)
        _check(self._L, self._ctx, self._L.psx_adarevision_state(
            self._ctx, table_id, first_row, num_rows, ctypes.c_void_p(acc.ctypes.data),
            ctypes.c_void_p(z.ctypes.data), ctypes.c_void_p(zm.ctypes.data), ctypes.byref(live)))
        return acc, z, zm, int(live.value)

    def clear_dirty(self, table_id):
        _check(self._L, self._ctx, self._L.psx_clear_dirty(self._ctx, table_id))

    def serialize_rows(self, table_id, row_ids):
        ids = np.ascontiguousarray(row_ids, dtype=np.int32)
        cap = 1 << 16
        while True:
            out = np.zeros(cap, dtype=np.uint8)
            used = ctypes.c_size_t()
            st = self._L.psx_serialize_rows(self._ctx, table_id, ctypes.c_void_p(ids.ctypes.data),
                                            ids.size, ctypes.c_void_p(out.ctypes.data), cap,
                                            ctypes.byref(used))
            if st == 9:   # PSX_ERR_BUFFER_TOO_SMALL
                cap *= 4
                continue
            _check(self._L, self._ctx, st)
            return out[:used.value].tobytes()

    def serialize_dirty(self, clear=True, out=None):
        """Push body for every dirty row of every table (server.cpp:189-309).

        Returns a numpy uint8 view of the body.  The body lands in page-locked host
        memory (kept by this object and reused, so the view is valid until the next
        call) unless `out` (a writable numpy uint8 array) is given."""
        return self._serialize(self._L.psx_serialize_dirty, clear, out)

    def serialize_partial(self, clear=True, out=None):
        """Partial push body (Server::CreateSendServerPushRowMsgsPartial, server.cpp:311-420):
        per table the first server_push_row_upper_bound dirty rows in send order.  An
        empty array when no table has a row to send."""
        return self._serialize(self._L.psx_serialize_partial, clear, out)

    def _serialize(self, fn, clear, out):
        used = ctypes.c_size_t()
        st = fn(self._ctx, None, 0, ctypes.byref(used), 0, 0)
        if st not in (_abi.PSX_OK, 9):
            _check(self._L, self._ctx, st)
        need = max(used.value, 1)
        if out is None:
            buf = getattr(self, "_pinned", None)
            if buf is None or buf.numel() < need:
                import torch
                self._pinned = buf = torch.empty(need + need // 4, dtype=torch.uint8, pin_memory=True)
            out = buf.numpy()
        assert out.dtype == np.uint8 and out.size >= need
        _check(self._L, self._ctx, fn(self._ctx, ctypes.c_void_p(out.ctypes.data), out.size,
                                      ctypes.byref(used), 0, 1 if clear else 0))
        return out[:used.value]

    # -- clocks and subscriptions (SSP / SSPPush) -------------------------------------
    def ClockUntil(self, bg_thread_id, clock):
        """Server::ClockUntil (server.cpp:62-79): advance the sender's clock; returns the new
        min clock if it advanced, else 0 (the reference's "clock changed")."""
        out = ctypes.c_int32()
        _check(self._L, self._ctx, self._L.psx_clock_until(self._ctx, bg_thread_id, clock, ctypes.byref(out)))
        return out.value

    def GetMinClock(self):
        out = ctypes.c_int32()
        _check(self._L, self._ctx, self._L.psx_min_clock(self._ctx, ctypes.byref(out)))
        return out.value

    def sender_clock(self, bg_thread_id):
        out = ctypes.c_int32()
        _check(self._L, self._ctx, self._L.psx_sender_clock(self._ctx, bg_thread_id, ctypes.byref(out)))
        return out.value

    def set_num_clients(self, n):
        _check(self._L, self._ctx, self._L.psx_set_num_clients(self._ctx, n))
        self.num_clients = n

    def subscribe(self, table_id, row_ids, client_id):
        """FindCreateRow + RowSubscribe for the listed rows (server_thread.cpp:185-200)."""
        ids = np.ascontiguousarray(row_ids, dtype=np.int32)
        _check(self._L, self._ctx, self._L.psx_row_subscribe(self._ctx, table_id, ctypes.c_void_p(ids.ctypes.data),
                                                               int(ids.size), client_id))

    def row_subscriptions(self, table_id, first_row, num_rows):
        out = np.zeros(num_rows, dtype=np.uint64)
        _check(self._L, self._ctx, self._L.psx_row_subscriptions(self._ctx, table_id, first_row, num_rows,
                                                                   ctypes.c_void_p(out.ctypes.data)))
        return out

    def serialize_push(self, clear=True, as_bytes=True):
        """Server::CreateSendServerPushRowMsgs with subscriptions (server.cpp:189-309): a list
        of num_clients push bodies, one per client.  The bodies land in page-locked host
        buffers kept by this object; as_bytes=False returns numpy views of them (valid
        until the next call) instead of bytes copies."""
        C = getattr(self, "num_clients", 1)
        caps = (ctypes.c_size_t * C)()
        used = (ctypes.c_size_t * C)()
        st = self._L.psx_serialize_push(self._ctx, None, caps, used, 0, 0)
        if st not in (_abi.PSX_OK, 9):
            _check(self._L, self._ctx, st)
        pinned = getattr(self, "_push_pinned", None)
        if pinned is None or len(pinned) != C:
            pinned = self._push_pinned = [None] * C
        import torch
        for k in range(C):
            need = max(used[k], 1)
            if pinned[k] is None or pinned[k].numel() < need:
                pinned[k] = torch.empty(need + need // 4, dtype=torch.uint8, pin_memory=True)
        bufs = [t.numpy() for t in pinned]
        ptrs = (ctypes.c_void_p * C)(*[b.ctypes.data for b in bufs])
        for k in range(C):
            caps[k] = bufs[k].size
        _check(self._L, self._ctx, self._L.psx_serialize_push(self._ctx, ptrs, caps, used, 0, 1 if clear else 0))
        if as_bytes:
            return [bufs[k][:used[k]].tobytes() for k in range(C)]
        return [bufs[k][:used[k]] for k in range(C)]

    # -- client side of serve-back ------------------------------------------------------
    def apply_push_body(self, body, insert_missing=False, device_ptr=None, size=None):
        """SSPPushBgWorker::ApplyServerPushedRow on this context as a client cache
        (ssp_push_bg_worker.cpp:70-122): host bytes, or a device buffer (device_ptr, size)."""
        if device_ptr is not None:
            _check(self._L, self._ctx, self._L.psx_apply_push_body(self._ctx, device_ptr, size, 1,
                                                                     1 if insert_missing else 0))
            return
        buf = np.ascontiguousarray(np.frombuffer(bytes(body), dtype=np.uint8))
        _check(self._L, self._ctx, self._L.psx_apply_push_body(
            self._ctx, ctypes.c_void_p(buf.ctypes.data) if buf.size else None, buf.size, 0,
            1 if insert_missing else 0))

    # -- client-side pack -------------------------------------------------------------
    def pack_stream(self, tables, with_index=False, with_rows=False):
        """Pack per-table oplog rows into one message on the device (psx_pack_stream).

        tables: dicts {table_id, dtype (psx dtype), dense_serialized, row_ids (CUDA int32
        [n]), oplogs (CUDA [n, capacity])}.  Returns a CUDA uint8 tensor holding the
        message (empty for an all-empty pack) and, with with_index, the CUDA int64 tensor
        of record offsets; with with_rows (psx_pack_stream_indexed), also the CUDA int32
        tensor of record rows (appended to the returned tuple)."""
        import torch
        torch.cuda.current_stream(self.device).synchronize()   # inputs come from torch's stream
        n = len(tables)
        arr = (_abi.psx_pack_table * max(n, 1))()
        nrec = 0
        for i, t in enumerate(tables):
            op = t["oplogs"]
            assert op.is_cuda and op.is_contiguous() and op.dim() == 2
            ids = t["row_ids"]
            assert ids.is_cuda and ids.dtype == torch.int32 and ids.is_contiguous()
            arr[i].table_id = t["table_id"]
            arr[i].dtype = t["dtype"]
            arr[i].dense_serialized = 1 if t["dense_serialized"] else 0
            arr[i].capacity = op.shape[1]
            arr[i].num_rows = op.shape[0]
            arr[i].row_ids = ids.data_ptr() if op.shape[0] else None
            arr[i].oplogs = op.data_ptr() if op.shape[0] else None
            nrec += op.shape[0]
        used = ctypes.c_size_t()
        st = self._L.psx_pack_stream(self._ctx, arr, n, None, 0, ctypes.byref(used), None)
        if st not in (_abi.PSX_OK, 9):
            _check(self._L, self._ctx, st)
        dev = torch.device("cuda", self.device)
        out = torch.empty((used.value + 3) // 4, dtype=torch.int32, device=dev).view(torch.uint8)
        idx = torch.empty(max(nrec, 1), dtype=torch.int64, device=dev) if with_index else None
        rws = torch.empty(max(nrec, 1), dtype=torch.int32, device=dev) if with_rows else None
        if used.value:
            _check(self._L, self._ctx, self._L.psx_pack_stream_indexed(
                self._ctx, arr, n, out.data_ptr(), out.numel(), ctypes.byref(used),
                idx.data_ptr() if idx is not None else None, rws.data_ptr() if rws is not None else None))
        out = out[:used.value]
        res = (out,)
        if with_index:
            res += (idx[:nrec],)
        if with_rows:
            res += (rws[:nrec],)
        return res if len(res) > 1 else out

    def split_stream(self, msg, row_begin, record_offsets=None, formats=None, out=None, sync_current=True):
        """psx_split_stream: the per-server split of one device message (CUDA uint8 tensor)
        over row-range owners (row_begin: nowners + 1 ascending row ids).  Returns (out, sizes):
        a CUDA uint8 tensor with the owners' sub-streams back to back and their byte counts.
        formats: {table_id: TableInfo} — split with these record formats
        (psx_split_stream_formats) instead of this context's tables, so a splitter needs no
        table storage.  out: a preallocated CUDA uint8 buffer (4-byte aligned) to split into.
        sync_current: first wait for torch's current stream (the message's producer)."""
        import torch
        if sync_current:
            torch.cuda.current_stream(self.device).synchronize()
        rb = (ctypes.c_int64 * len(row_begin))(*[int(x) for x in row_begin])
        nown = len(row_begin) - 1
        sizes = (ctypes.c_uint64 * nown)()
        n = msg.numel()
        ntab = len(formats) if formats is not None else len(self.tables)
        cap = n + nown * (4 + 16 * max(ntab, 1))
        if out is None:
            out = torch.empty((cap + 3) // 4, dtype=torch.int32, device=msg.device).view(torch.uint8)
        offs = record_offsets.data_ptr() if record_offsets is not None else None
        if formats is not None:
            arr = (psx_table_config * max(len(formats), 1))(*[table_config(t, i) for t, i in formats.items()])
            st = self._L.psx_split_stream_formats(self._ctx, arr, len(formats), msg.data_ptr() if n else None, n,
                                                  offs, nown, rb, out.data_ptr(), out.numel(), sizes)
        else:
            st = self._L.psx_split_stream(self._ctx, msg.data_ptr() if n else None, n, offs, nown, rb,
                                          out.data_ptr(), out.numel(), sizes)
        _check(self._L, self._ctx, st)
        sz = [int(x) for x in sizes]
        return out[:sum(sz)], sz

    # -- timing ------------------------------------------------------------------------
    def timing(self, on=True):
        """on: False/0 off, True/1 every pipeline kernel, 2 the apply kernels only."""
        _check(self._L, self._ctx, self._L.psx_timing_enable(self._ctx, int(on)))

    def timing_read(self, kernel):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        _check(self._L, self._ctx, self._L.psx_timing_read(self._ctx, kernel.encode(),
                                                           ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def stats(self, reset=False):
        """psx_ctx_stats: the STATS_SERVER_ACCUM_APPLY_OPLOG_* counters (server_thread.cpp:240-244)
        as a dict: calls, messages, oplog_bytes, apply_sec, settled_calls (+ oplog_recv_mb)."""
        st = _abi.psx_apply_stats()
        _check(self._L, self._ctx, self._L.psx_ctx_stats(self._ctx, ctypes.byref(st), 1 if reset else 0))
        d = {k: getattr(st, k) for k, _ in st._fields_}
        d["oplog_recv_mb"] = d["oplog_bytes"] / float(1 << 20)
        return d

    def timing_reset(self):
        _check(self._L, self._ctx, self._L.psx_timing_reset(self._ctx))


class ServerThread:
    """The caller of the apply path: ServerThread::HandleOpLogMsg and HandleRowRequest
    (server_thread.cpp:185-299) with SSPPush's push-on-clock-change, over any server
    backend exposing the Server methods below (psx Server; the oracle adapter in tests).

    push(bodies, min_clock): receives one push body per client whenever the server's min
    clock advances (ServerPushRow -> CreateSendServerPushRowMsgs, ssp_push_server_thread.cpp:39-49).
    reply(bg_id, table_id, row_id, server_clock, record): the row-request reply
    (ReplyRowRequest, server_thread.cpp:205-222) with the row as one RecordBuff record.
    """

    def __init__(self, server, push, reply=None):
        self.server = server
        self.push = push
        self.reply = reply
        self.requests = {}   # clock -> [(bg_id, table_id, row_id)] (Server::AddRowRequest, server.cpp:81-98)

    @staticmethod
    def client_of(bg_id):
        """GlobalContext::thread_id_to_client_id: thread ids are client * 1000 + k (context.hpp:410-414)."""
        return bg_id // 1000

    def _reply(self, bg_id, table_id, row_id):
        s = self.server
        s.subscribe(table_id, [row_id], self.client_of(bg_id))           # RowSubscribe
        rec = s.serialize_rows(table_id, [row_id])
        if self.reply:
            self.reply(bg_id, table_id, row_id, s.GetMinClock(), rec)
        s.row_sent(table_id, [row_id], 1)                                # Server::RowSent(.., 1)

    def HandleRowRequest(self, bg_id, table_id, row_id, clock):
        """server_thread.cpp:185-200: answer now, or once the min clock reaches `clock`."""
        if self.server.GetMinClock() < clock:
            self.requests.setdefault(clock, []).append((bg_id, table_id, row_id))
            return False
        self._reply(bg_id, table_id, row_id)
        return True

    def HandleOpLogMsg(self, bg_id, payload, is_clock, bg_clock, version):
        """server_thread.cpp:224-299: apply, advance the sender's clock, and on a new min
        clock fulfil the waiting row requests and push the dirty rows to every client."""
        self.server.ApplyOpLogUpdateVersion(payload, len(payload), bg_id, version)
        changed = False
        if is_clock:
            changed = self.server.ClockUntil(bg_id, bg_clock) != 0
            if changed:   # Server::GetFulfilledRowRequests: the requests of exactly the new min clock
                for req in self.requests.pop(self.server.GetMinClock(), []):
                    self._reply(*req)
        if changed:
            self.push(self.server.serialize_push(clear=True), self.server.GetMinClock())
        return changed
