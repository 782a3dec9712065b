"""Vectorised builders for the reference's oplog stream format (Appendix A of SURVEY.md).

One ClientSendOpLogMsg payload (ps_msgs.hpp:1003-1055, after the 41-byte header):
    int32 num_tables
    per table: int32 table_id; size_t update_size; int32 num_rows; records...
    dense record : int32 row_id; V[dense_row_oplog_capacity]     (dense_row_oplog.hpp:133-136)
    sparse record: int32 row_id; int32 n; int32 cols[n]; V vals[n] (dense_row_oplog.hpp:112-131)
Layout as written by OpLogSerializer + RowOpLogSerializer (oplog_serializer.hpp:12-37,
row_oplog_serializer.hpp:139-166).  These builders are how bench.py and the tests
produce synthetic worker batches; tests cross-check them against the oracle's packer.
"""
import numpy as np

TABLE_HEADER_BYTES = 16   # int32 table_id + size_t update_size + int32 num_rows


def dense_record_bytes(cap, vsize):
    return 4 + cap * vsize


def dense_stream_bytes(num_rows, cap, vsize):
    return 4 + TABLE_HEADER_BYTES + num_rows * dense_record_bytes(cap, vsize)


def dense_stream_np(table_id, row_ids, payload):
    """One single-table dense stream as a numpy uint8 array."""
    payload = np.ascontiguousarray(payload)
    n, cap = payload.shape
    vsize = payload.dtype.itemsize
    words_per_rec = 1 + cap * vsize // 4
    out = np.zeros(dense_stream_bytes(n, cap, vsize), dtype=np.uint8)
    hdr = out[:20].view(np.int32)
    hdr[0] = 1
    hdr[1] = table_id
    out[8:16].view(np.uint64)[0] = vsize
    hdr[4] = n
    recs = out[20:].view(np.int32).reshape(n, words_per_rec)
    recs[:, 0] = np.asarray(row_ids, dtype=np.int32)
    recs[:, 1:] = payload.view(np.int32).reshape(n, words_per_rec - 1)
    return out


def dense_variant_stream_np(table_id, row_ids, payload, versions=None, end_of_version=None, f16=False):
    """One single-table stream of the variant dense record formats (records are only
    byte-aligned here, so they are assembled bytewise):
      versions given : VersionDenseRowOpLog::SerializeDense = V[cap] + uint64 version +
                       bool end_of_version (version_dense_row_oplog.hpp:161-171)
      f16            : DenseRowOpLogFloat16::SerializeDense = uint16[cap] (binary16 bits,
                       dense_row_oplog_float16.hpp:135-142); payload is uint16 bits or
                       float16, and update_size in the table header stays sizeof(float)."""
    payload = np.ascontiguousarray(payload)
    n, cap = payload.shape
    if f16:
        body = payload.view(np.uint16).view(np.uint8).reshape(n, 2 * cap)
        vsize = 4
    else:
        vsize = payload.dtype.itemsize
        body = payload.view(np.uint8).reshape(n, cap * vsize)
    cols = [np.asarray(row_ids, dtype="<i4").view(np.uint8).reshape(n, 4), body]
    if versions is not None:
        cols.append(np.asarray(versions, dtype="<u8").view(np.uint8).reshape(n, 8))
        eov = np.zeros(n, bool) if end_of_version is None else np.asarray(end_of_version, bool)
        cols.append(eov.astype(np.uint8).reshape(n, 1))
    recs = np.concatenate(cols, axis=1)
    hdr = np.zeros(20, np.uint8)
    hdr[:8].view(np.int32)[:] = [1, table_id]
    hdr[8:16].view(np.uint64)[0] = vsize
    hdr[16:20].view(np.int32)[0] = n
    return np.concatenate([hdr, recs.reshape(-1)])


def sparse_stream_np(table_id, vsize, rows):
    """rows: list of (row_id, cols int32[n], vals V[n]); one single-table sparse stream."""
    parts = [np.array([1, table_id], dtype=np.int32).view(np.uint8),
             np.array([vsize], dtype=np.uint64).view(np.uint8),
             np.array([len(rows)], dtype=np.int32).view(np.uint8)]
    for rid, cols, vals in rows:
        parts.append(np.array([rid, len(cols)], dtype=np.int32).view(np.uint8))
        parts.append(np.ascontiguousarray(cols, dtype=np.int32).view(np.uint8))
        parts.append(np.ascontiguousarray(vals).view(np.uint8))
    return np.concatenate(parts)


def stream_record_offsets(stream, tables):
    """tables: {table_id: body_bytes or None}; body_bytes for dense-serialized tables
    (cap * update_size, + 9 for version records), None for sparse tables."""
    b = bytes(np.asarray(stream, dtype=np.uint8))
    ntab = int(np.frombuffer(b[:4], "<i4")[0]) if len(b) >= 4 else 0
    off, out = 4, []
    for _ in range(ntab):
        tid, = np.frombuffer(b[off:off + 4], "<i4")
        usz, = np.frombuffer(b[off + 4:off + 12], "<u8")
        nrows, = np.frombuffer(b[off + 12:off + 16], "<i4")
        off += 16
        body = tables[int(tid)]
        for _ in range(int(nrows)):
            out.append(off)
            if body is None:
                n, = np.frombuffer(b[off + 4:off + 8], "<i4")
                off += 8 + int(n) * (4 + int(usz))
            else:
                off += 4 + body
    return np.array(out, dtype=np.uint64)


def pack_np(tables):
    """One multi-table message, as CreateOpLogMsgs + OpLogSerializer lay it out
    (abstract_bg_worker.cpp:590-649, oplog_serializer.hpp:12-37): tables in ascending id,
    empty tables omitted.  tables: dicts {table_id, row_ids int32[n], oplogs V[n, cap],
    dense_serialized}; sparse records keep the non-zero columns in ascending order
    (DenseRowOpLog::SerializeSparse, dense_row_oplog.hpp:112-131)."""
    parts = []
    live = sorted((t for t in tables if len(t["row_ids"])), key=lambda t: t["table_id"])
    if not live:
        return np.zeros(0, dtype=np.uint8)
    parts.append(np.array([len(live)], dtype=np.int32).view(np.uint8))
    for t in live:
        op = np.ascontiguousarray(t["oplogs"])
        ids = np.asarray(t["row_ids"], dtype=np.int32)
        if t["dense_serialized"] and (t.get("f16") or t.get("versions") is not None):
            parts.append(dense_variant_stream_np(t["table_id"], ids, op, versions=t.get("versions"),
                                                 end_of_version=t.get("end_of_version"), f16=t.get("f16", False))[4:])
        elif t["dense_serialized"]:
            parts.append(dense_stream_np(t["table_id"], ids, op)[4:])
        else:
            rows = []
            for r in range(ids.size):
                nz = np.nonzero(op[r])[0].astype(np.int32)
                rows.append((int(ids[r]), nz, op[r, nz]))
            parts.append(sparse_stream_np(t["table_id"], op.dtype.itemsize, rows)[4:])
    return np.concatenate(parts)


def dense_stream_torch(table_id, row_ids, payload):
    """Device-side builder: row_ids int32[n] and payload V[n, cap] are torch tensors on the
    GPU; returns a uint8 CUDA tensor holding the stream (4-byte aligned)."""
    import torch
    n, cap = payload.shape
    vsize = payload.element_size()
    words_per_rec = 1 + cap * vsize // 4
    nbytes = dense_stream_bytes(n, cap, vsize)
    out = torch.empty(nbytes // 4, dtype=torch.int32, device=payload.device)
    hdr = torch.tensor([1, table_id, vsize, 0, n], dtype=torch.int32)   # update_size hi word = 0
    out[:5].copy_(hdr)
    recs = out[5:].view(n, words_per_rec)
    recs[:, 0].copy_(row_ids.to(torch.int32))
    recs[:, 1:].copy_(payload.contiguous().view(torch.int32).view(n, words_per_rec - 1))
    return out.view(torch.uint8)


def dense_stream_torch_f16(table_id, row_ids, payload16):
    """Device-side builder of a kDenseRowOpLogFloat16 stream (int32 row_id; uint16[cap],
    dense_row_oplog_float16.hpp:135-142; update_size stays sizeof(float)); cap even."""
    import torch
    n, cap = payload16.shape
    assert cap % 2 == 0 and payload16.element_size() == 2
    words = 1 + cap // 2
    out = torch.empty(5 + n * words, dtype=torch.int32, device=payload16.device)
    out[:5].copy_(torch.tensor([1, table_id, 4, 0, n], dtype=torch.int32))
    recs = out[5:].view(n, words)
    recs[:, 0].copy_(row_ids.to(torch.int32))
    recs[:, 1:].copy_(payload16.contiguous().view(torch.int16).view(torch.int32).view(n, cap // 2))
    return out.view(torch.uint8)


def parse_push_body(body):
    """Parse a push body ({table_id; records; -1|-2} per table, as read by the client's
    SerializedRowReader, serialized_row_reader.hpp:49-93) into
    {table_id: {row_id: row bytes}}."""
    import struct
    out, off, n = {}, 0, len(body)
    while off + 4 <= n:
        tid = struct.unpack_from("<i", body, off)[0]
        off += 4
        rows = out.setdefault(tid, {})
        while True:
            rid = struct.unpack_from("<i", body, off)[0]
            off += 4
            if rid == -1:
                break
            if rid == -2:
                return out
            size = struct.unpack_from("<Q", body, off)[0]
            off += 8
            rows[rid] = bytes(body[off:off + size])
            off += size
    return out


# ---- message headers (ClientSendOpLogMsg / ServerPushRowMsg) through libpsx -----------------

def encode_oplog_msg(payload, version, client_id=0, is_clock=False, bg_clock=0, seq_num=0, ack_num=0):
    """A whole ClientSendOpLogMsg: the 41-byte header (psx_encode_oplog_header,
    ps_msgs.hpp:1003-1055) followed by the payload stream."""
    import ctypes
    from . import _abi
    payload = np.ascontiguousarray(np.asarray(payload, dtype=np.uint8))
    h = _abi.psx_oplog_msg_header(seq_num, ack_num, payload.size, 1 if is_clock else 0, client_id, version, bg_clock)
    out = np.zeros(_abi.OPLOG_MSG_HEADER_BYTES + payload.size, dtype=np.uint8)
    assert _abi.load().psx_encode_oplog_header(ctypes.byref(h), ctypes.c_void_p(out.ctypes.data)) == 0
    out[_abi.OPLOG_MSG_HEADER_BYTES:] = payload
    return out


def decode_oplog_msg(msg):
    """(header dict, payload view) of a ClientSendOpLogMsg; raises PsxError if malformed."""
    import ctypes
    from . import _abi
    msg = np.ascontiguousarray(np.asarray(msg, dtype=np.uint8))
    h = _abi.psx_oplog_msg_header()
    st = _abi.load().psx_decode_oplog_header(ctypes.c_void_p(msg.ctypes.data), msg.size, ctypes.byref(h))
    if st:
        raise _abi.PsxError(st, "decode_oplog_msg")
    d = {k: getattr(h, k) for k, _ in h._fields_}
    return d, msg[_abi.OPLOG_MSG_HEADER_BYTES:_abi.OPLOG_MSG_HEADER_BYTES + h.avai_size]


def encode_push_msg(body, clock, version, is_clock=True, seq_num=0, ack_num=0):
    import ctypes
    from . import _abi
    body = np.ascontiguousarray(np.frombuffer(bytes(body), dtype=np.uint8))
    h = _abi.psx_push_msg_header(seq_num, ack_num, body.size, clock, version, 1 if is_clock else 0)
    out = np.zeros(_abi.PUSH_MSG_HEADER_BYTES + body.size, dtype=np.uint8)
    assert _abi.load().psx_encode_push_header(ctypes.byref(h), ctypes.c_void_p(out.ctypes.data)) == 0
    out[_abi.PUSH_MSG_HEADER_BYTES:] = body
    return out


def decode_push_msg(msg):
    import ctypes
    from . import _abi
    msg = np.ascontiguousarray(np.asarray(msg, dtype=np.uint8))
    h = _abi.psx_push_msg_header()
    st = _abi.load().psx_decode_push_header(ctypes.c_void_p(msg.ctypes.data), msg.size, ctypes.byref(h))
    if st:
        raise _abi.PsxError(st, "decode_push_msg")
    d = {k: getattr(h, k) for k, _ in h._fields_}
    return d, msg[_abi.PUSH_MSG_HEADER_BYTES:_abi.PUSH_MSG_HEADER_BYTES + h.avai_size]


def split_stream(stream, tables, max_bytes=(1 << 31) - 1):
    """Split one Appendix-A message into messages of at most max_bytes each, at record
    boundaries, keeping table and record order (what a producer must do for the
    reference reader's int32 offset_, serialized_oplog_reader.hpp:137).  tables:
    {table_id: dense body bytes or None for sparse}, as stream_record_offsets takes.
    Returns a list of numpy uint8 messages; applying them in order equals applying
    `stream` (per-row update order is unchanged)."""
    b = np.asarray(stream, dtype=np.uint8)
    if b.size <= max_bytes:
        return [b]
    ntab = int(b[:4].view(np.int32)[0])
    # every record: (table index, start, end)
    recs, off = [], 4
    heads = []
    for k in range(ntab):
        tid, = np.frombuffer(b[off:off + 4].tobytes(), "<i4")
        usz, = np.frombuffer(b[off + 4:off + 12].tobytes(), "<u8")
        nrows, = np.frombuffer(b[off + 12:off + 16].tobytes(), "<i4")
        heads.append((int(tid), int(usz)))
        off += 16
        body = tables[int(tid)]
        for _ in range(int(nrows)):
            if body is None:
                n, = np.frombuffer(b[off + 4:off + 8].tobytes(), "<i4")
                end = off + 8 + int(n) * (4 + int(usz))
            else:
                end = off + 4 + body
            recs.append((k, off, end))
            off = end
    out, cur, size = [], [], 4
    for k, s0, e0 in recs:
        extra = (e0 - s0) + (16 if not cur or cur[-1][0] != k else 0)
        if cur and size + extra > max_bytes:
            out.append(cur)
            cur, size = [], 4
            extra = (e0 - s0) + 16
        if size + extra > max_bytes:
            raise ValueError("a single record exceeds max_bytes")
        cur.append((k, s0, e0))
        size += extra
    if cur:
        out.append(cur)
    msgs = []
    for piece in out:
        groups = []
        for k, s0, e0 in piece:
            if groups and groups[-1][0] == k and groups[-1][2] == s0:
                groups[-1][2] = e0
                groups[-1][3] += 1
            else:
                groups.append([k, s0, e0, 1])
        parts = [np.array([len(groups)], np.int32).view(np.uint8)]
        for k, s0, e0, n in groups:
            tid, usz = heads[k]
            parts += [np.array([tid], np.int32).view(np.uint8), np.array([usz], np.uint64).view(np.uint8),
                      np.array([n], np.int32).view(np.uint8), b[s0:e0]]
        msgs.append(np.concatenate(parts))
    return msgs
