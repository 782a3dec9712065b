"""The one exchange step of the multi-GPU path: per-owner sub-streams, all-to-all.

A worker's clock produces, per owning server shard, one ClientSendOpLogMsg payload:
the reference client splits its oplog by `GetPartitionServerID` while packing
(`RowOpLogSerializer::AppendRowOpLog`, row_oplog_serializer.hpp:100-124) and sends each
shard its own message (`AbstractBgWorker::SendOpLogMsgs`, abstract_bg_worker.cpp:651-689).
On one MI355X node the messages for all shards sit in one send buffer in owner order,
and a single all-to-all (RCCL over xGMI on GPUs; gloo in the CPU tests) delivers to
every owner the messages of every worker, in worker (source-rank) order.  The owner then
applies them with one fused, order-preserving `psx_apply_streams_device` call, so the
result is bit-identical to the reference server applying the same messages one by one.

When batches are already split by owner at their producer (the default bench), no
collective is needed at all.

`Exchange` is the product path: libpsx's own RCCL communicator (psx_comm_*,
psx_exchange_sizes / psx_exchange_streams — grouped ncclSend/ncclRecv); the process group
only carries the communicator's unique id.  `alltoall_streams` is the same exchange over
torch.distributed (any backend: gloo in the CPU tests).
"""
import ctypes

import torch
import torch.distributed as dist

from . import _abi


class Exchange:
    """A libpsx RCCL communicator over the ranks of a torch.distributed group."""

    def __init__(self, device, group=None):
        L = self._L = _abi.load()
        single = not dist.is_initialized()     # one rank without a process group: a self exchange
        self.world = 1 if single else dist.get_world_size(group)
        self.rank = 0 if single else dist.get_rank(group)
        uid = (ctypes.c_uint8 * 128)()
        if self.rank == 0:
            st = L.psx_comm_unique_id(uid)
            if st:
                raise _abi.PsxError(st, L.psx_comm_last_error(None).decode())
        if not single:
            t = torch.tensor(list(uid), dtype=torch.uint8)
            if dist.get_backend(group) == "nccl":
                t = t.cuda(device)
            dist.broadcast(t, 0, group=group)
            uid = (ctypes.c_uint8 * 128)(*t.cpu().tolist())
        self._c = ctypes.c_void_p()
        st = L.psx_comm_create(uid, self.world, self.rank, device, ctypes.byref(self._c))
        if st:
            raise _abi.PsxError(st, L.psx_comm_last_error(None).decode())

    def close(self):
        if self._c:
            self._L.psx_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def info(self):
        """What RCCL itself reports for this communicator (psx_comm_info): the rank count and
        rank it was built with, its device, the RCCL version and the librccl file loaded."""
        n, r, d, v = (ctypes.c_int32() for _ in range(4))
        path = ctypes.create_string_buffer(512)
        st = self._L.psx_comm_info(self._c, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d), ctypes.byref(v),
                                   path, len(path))
        if st:
            raise _abi.PsxError(st, self._L.psx_comm_last_error(self._c).decode())
        return {"nranks": n.value, "rank": r.value, "device": d.value, "rccl_version": v.value,
                "librccl": path.value.decode()}

    def peer_bytes(self, reset=False):
        """(sent[p], received[p]) bytes enqueued per peer since creation or the last reset."""
        n = self.world
        s, r = (ctypes.c_uint64 * n)(), (ctypes.c_uint64 * n)()
        st = self._L.psx_comm_peer_bytes(self._c, s, r, int(bool(reset)))
        if st:
            raise _abi.PsxError(st, self._L.psx_comm_last_error(self._c).decode())
        return [int(x) for x in s], [int(x) for x in r]

    def alltoall(self, send, send_sizes, stream=None):
        """send: CUDA uint8 tensor with world sub-streams back to back (owner order).
        Returns (recv, recv_sizes) in source-rank order.  With a `stream` other than the
        current one, both tensors are marked as used on it (record_stream), so the caching
        allocator does not hand them out before RCCL is done with them."""
        import torch
        L = self._L
        n = self.world
        if len(send_sizes) != n:
            raise ValueError(f"{len(send_sizes)} sub-stream sizes for {n} ranks")
        if any(int(x) % 4 for x in send_sizes):
            raise ValueError("sub-stream sizes are multiples of 4 bytes")
        if send.numel() < sum(int(x) for x in send_sizes):
            raise ValueError(f"send holds {send.numel()} bytes, the sizes name {sum(int(x) for x in send_sizes)}")
        ss = (ctypes.c_uint64 * n)(*[int(x) for x in send_sizes])
        rs = (ctypes.c_uint64 * n)()
        cur = torch.cuda.current_stream(send.device)
        hs = stream if stream is not None else cur.cuda_stream
        st = L.psx_exchange_sizes(self._c, ss, rs, ctypes.c_void_p(hs))
        if st:
            raise _abi.PsxError(st, L.psx_comm_last_error(self._c).decode())
        rsz = [int(x) for x in rs]
        recv = torch.empty(max(sum(rsz), 4), dtype=torch.uint8, device=send.device)
        if stream is not None and stream != cur.cuda_stream:
            ext = torch.cuda.ExternalStream(stream, device=send.device)
            recv.record_stream(ext)
            send.record_stream(ext)
        st = L.psx_exchange_streams(self._c, send.data_ptr(), ss, recv.data_ptr(), rs, ctypes.c_void_p(hs))
        if st:
            raise _abi.PsxError(st, L.psx_comm_last_error(self._c).decode())
        return recv[:sum(rsz)], rsz

    def sizes_async(self, send_sizes, recv_sizes, stream):
        """psx_exchange_sizes_async: enqueue the sub-stream sizes on `stream` (a HIP stream
        handle); recv_sizes is a page-locked int64 CPU tensor of world entries, valid once the
        stream has passed this point."""
        n = self.world
        if any(int(x) % 4 for x in send_sizes):
            raise ValueError("sub-stream sizes are multiples of 4 bytes")
        assert recv_sizes.is_pinned() and recv_sizes.numel() >= n and recv_sizes.element_size() == 8
        ss = (ctypes.c_uint64 * n)(*[int(x) for x in send_sizes])
        st = self._L.psx_exchange_sizes_async(self._c, ss, ctypes.c_void_p(recv_sizes.data_ptr()),
                                              ctypes.c_void_p(stream))
        if st:
            raise _abi.PsxError(st, self._L.psx_comm_last_error(self._c).decode())

    def streams_v(self, send, send_sizes, send_displs, recv, recv_sizes, recv_displs, stream):
        """psx_exchange_streams_v: explicit displacements; a zero size skips the peer."""
        n = self.world
        if any(int(o) + int(z) > send.numel() for o, z in zip(send_displs, send_sizes)):
            raise ValueError("a send sub-stream past the send buffer")
        if recv is not None and any(int(o) + int(z) > recv.numel() for o, z in zip(recv_displs, recv_sizes)):
            raise ValueError("a receive sub-stream past the receive buffer")
        arr = lambda v: (ctypes.c_uint64 * n)(*[int(x) for x in v])
        st = self._L.psx_exchange_streams_v(self._c, send.data_ptr(), arr(send_sizes), arr(send_displs),
                                            recv.data_ptr() if recv is not None else None, arr(recv_sizes),
                                            arr(recv_displs), ctypes.c_void_p(stream))
        if st:
            raise _abi.PsxError(st, self._L.psx_comm_last_error(self._c).decode())

    def streams_into(self, send, send_sizes, recv, recv_sizes, stream):
        """psx_exchange_streams into a caller-owned recv buffer on `stream` (HIP handle);
        the caller keeps send and recv alive and unused until the stream has passed."""
        n = self.world
        if send.numel() < sum(send_sizes) or recv.numel() < sum(recv_sizes):
            raise ValueError("exchange buffers smaller than the sizes they carry")
        ss = (ctypes.c_uint64 * n)(*[int(x) for x in send_sizes])
        rs = (ctypes.c_uint64 * n)(*[int(x) for x in recv_sizes])
        st = self._L.psx_exchange_streams(self._c, send.data_ptr(), ss, recv.data_ptr(), rs, ctypes.c_void_p(stream))
        if st:
            raise _abi.PsxError(st, self._L.psx_comm_last_error(self._c).decode())


class ShardExchange:
    """One rank's side of the exchange-bearing step (SURVEY §8(e), C4's shape).

    Every rank holds worker batches that span every row-range shard.  The reference client
    splits each batch by owning server while packing and sends each server its message
    (AbstractBgWorker::CreateOpLogMsgs / SendOpLogMsgs, abstract_bg_worker.cpp:590-689); each
    server applies what it receives (Server::ApplyOpLogUpdateVersion, server.cpp:120-179).
    Here a batch arrives as a sequence of Appendix-A messages of at most 2 GiB each (chunks:
    the reference reader keeps its cursor in an int32, serialized_oplog_reader.hpp:137), and
    per chunk:
      1. split per owner on the device (psx_split_stream_formats: record formats only, no
         table) into send slot k % 2, on the split stream;
      2. the sub-stream sizes, then the bytes, to every owner (psx_exchange_sizes_async /
         psx_exchange_streams: RCCL grouped send/recv over xGMI) into recv slot k % 2, on the
         exchange stream;
      3. the owner applies the world's sub-streams in source-rank order in one fused call
         (psx_apply_streams_device on the owner context's stream), bit-exact to applying the
         same messages one by one.
    Chunk k's bytes cross while chunk k-1 applies and chunk k+1 splits; two slots of each
    buffer bound the HBM the step needs beyond the batches and the table to about four
    chunks.  Each sender's messages carry consecutive versions (one per chunk round; an
    owner with no records from a sender gets an empty message, which only bumps it).  With one
    rank nothing routes: the chunks are applied as they are, unless split_single asks for the
    split (and the own sub-stream path) anyway."""

    def __init__(self, server, table_id, info, row_begin, bg_ids, exchange, device, splitter_id=900,
                 split_single=False):
        import torch
        from .server import Server
        self.srv, self.xc, self.device = server, exchange, device
        self.world = exchange.world
        assert len(row_begin) == self.world + 1 and len(bg_ids) == self.world
        self.bounds = [int(x) for x in row_begin]
        self.bgs = list(bg_ids)
        self.formats = {table_id: info}
        self.splitter = Server(device=device, server_id=splitter_id + exchange.rank)   # no tables
        self.s_split = torch.cuda.Stream(device)
        self.s_x = torch.cuda.Stream(device)
        self.s_apply = torch.cuda.Stream(device)
        self.splitter.set_stream(self.s_split.cuda_stream)
        server.set_stream(self.s_apply.cuda_stream)
        self.send = [None, None]
        self.recv = [None, None]
        self.ev_sent = [torch.cuda.Event(), torch.cuda.Event()]     # a send slot's bytes have left
        self.ev_recv = [torch.cuda.Event(), torch.cuda.Event()]     # a recv slot's bytes have arrived
        self.ev_x0 = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
        self.ev_x1 = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
        self.rsz = torch.zeros((2, self.world), dtype=torch.int64).pin_memory()
        self.version = 0
        self.direct = self.world == 1 and not split_single
        self.reset_counters()

    def reset_counters(self):
        self.split_s = self.wait_s = self.sync_s = 0.0
        self.x_ms = 0.0
        self.chunks = 0
        self.sent_bytes = self.recv_bytes = 0
        self._x_pending = []

    def _grow(self, bufs, s, nbytes, ev=None):
        import torch
        if bufs[s] is None or bufs[s].numel() < nbytes:
            if ev is not None:
                ev.synchronize()
            bufs[s] = None
            bufs[s] = torch.empty((max(nbytes, 4) + 3) // 4, dtype=torch.int32,
                                  device=torch.device("cuda", self.device)).view(torch.uint8)
        return bufs[s]

    def _collect_x(self, keep_last=1):
        while len(self._x_pending) > keep_last:
            a, b = self._x_pending.pop(0)
            b.synchronize()
            self.x_ms += a.elapsed_time(b)

    def run(self, chunks, log=None):
        """Apply one batch per rank (a list of <= 2 GiB device messages, this rank's worker
        batch in record order) to the owners' shards.  Returns after every apply settled.

        The chunks may still be in production on the caller's current stream (a non_blocking
        copy, a packing kernel): the split stream waits for it first.  The server stays bound
        to this exchange's apply stream (set by the constructor) after the call."""
        import time
        n = self.world
        if self.direct:
            return self._run_direct(chunks, log)
        self.s_split.wait_stream(torch.cuda.current_stream(self.device))
        for k, msg in enumerate(chunks):
            s = k % 2
            ntab = len(self.formats)
            send = self._grow(self.send, s, msg.numel() + n * (4 + 16 * ntab), self.ev_sent[s])
            t0 = time.perf_counter()
            self.s_split.wait_event(self.ev_sent[s])        # chunk k-2's bytes have left the slot
            parts, sizes = self.splitter.split_stream(msg, self.bounds, formats=self.formats, out=send,
                                                      sync_current=False)
            t1 = time.perf_counter()
            rs = self.rsz[s]
            self.xc.sizes_async(sizes, rs, self.s_x.cuda_stream)
            ev = self.ev_x1[s]
            ev.record(self.s_x)
            ev.synchronize()                                # sizes known = chunk k-1's bytes arrived
            t2 = time.perf_counter()
            rsz = [int(x) for x in rs.tolist()]
            # The rank's own sub-stream does not cross: its owner applies it from the send
            # slot (held until that apply has settled: split k+2 reuses the slot after the
            # srv.sync() of iteration k+1).  The others land back to back in recv slot s,
            # which chunk k-2's apply last read (settled by the last srv.sync()).
            me = self.xc.rank
            sdis = [sum(sizes[:p]) for p in range(n)]
            xs, xr = list(sizes), list(rsz)
            xs[me] = xr[me] = 0
            rdis = [sum(xr[:p]) for p in range(n)]
            recv = self._grow(self.recv, s, sum(xr))
            a, b = torch_event_pair()
            a.record(self.s_x)
            if n > 1:
                self.xc.streams_v(parts, xs, sdis, recv, xr, rdis, self.s_x.cuda_stream)
            b.record(self.s_x)
            self.ev_sent[s].record(self.s_x)
            self.ev_recv[s].record(self.s_x)
            self._x_pending.append((a, b))
            # chunk k-1's apply finishes beside chunk k's exchange; then chunk k's is enqueued
            self.srv.sync()
            t3 = time.perf_counter()
            self.s_apply.wait_event(self.ev_recv[s])
            msgs = []
            for w in range(n):
                ptr = send.data_ptr() + sdis[me] if w == me else recv.data_ptr() + rdis[w]
                msgs.append((ptr, rsz[w], self.bgs[w], self.version))
            self.srv.apply_device(msgs)
            self.version += 1
            self.split_s += t1 - t0
            self.wait_s += t2 - t1
            self.sync_s += t3 - t2
            self.chunks += 1
            self.sent_bytes += sum(sizes)
            self.recv_bytes += sum(rsz)
            self._collect_x()
            if log is not None:
                log(f"chunk {k}: split {t1 - t0:.4f} s, sizes wait {t2 - t1:.4f} s, apply wait {t3 - t2:.4f} s")
        self.srv.sync()
        self._collect_x(0)

    def _run_direct(self, chunks, log=None):
        """One rank: each chunk is its only owner's message; applied in order on s_apply."""
        import time
        self.s_apply.wait_stream(torch.cuda.current_stream(self.device))
        for k, msg in enumerate(chunks):
            t0 = time.perf_counter()
            self.srv.apply_device([(msg.data_ptr(), msg.numel(), self.bgs[0], self.version)])
            self.version += 1
            self.sync_s += time.perf_counter() - t0
            self.chunks += 1
            self.sent_bytes += msg.numel()
            self.recv_bytes += msg.numel()
            if log is not None:
                log(f"chunk {k}: applied directly (one rank)")
        self.srv.sync()

    def close(self):
        self.splitter.close()


def torch_event_pair():
    import torch
    return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def alltoall_streams(send, send_sizes, group=None):
    """send: uint8 tensor holding world_size sub-streams back to back (owner order),
    send_sizes: their byte counts (multiples of 4).  Returns (recv, recv_sizes): the
    sub-streams addressed to this rank, ordered by source rank."""
    world = dist.get_world_size(group)
    assert len(send_sizes) == world
    assert all(s % 4 == 0 for s in send_sizes), "stream sizes are multiples of 4 bytes"
    dev = send.device
    sizes = torch.tensor(send_sizes, dtype=torch.int64, device=dev)
    recv_sizes = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_sizes, sizes, group=group)
    rs = [int(x) for x in recv_sizes.tolist()]
    recv = torch.empty(sum(rs), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send, rs, list(send_sizes), group=group)
    return recv, rs


def split(buf, sizes):
    """Views of consecutive sub-streams (each stays 4-byte aligned)."""
    out, off = [], 0
    for s in sizes:
        out.append(buf[off:off + s])
        off += s
    return out
