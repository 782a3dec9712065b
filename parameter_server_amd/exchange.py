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
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        uid = (ctypes.c_uint8 * 128)()
        if self.rank == 0:
            st = L.psx_comm_unique_id(uid)
            if st:
                raise _abi.PsxError(st, L.psx_comm_last_error(None).decode())
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

    def alltoall(self, send, send_sizes, stream=None):
        """send: CUDA uint8 tensor with world sub-streams back to back (owner order).
        Returns (recv, recv_sizes) in source-rank order."""
        L = self._L
        n = self.world
        ss = (ctypes.c_uint64 * n)(*[int(x) for x in send_sizes])
        rs = (ctypes.c_uint64 * n)()
        hs = stream if stream is not None else torch.cuda.current_stream(send.device).cuda_stream
        st = L.psx_exchange_sizes(self._c, ss, rs, ctypes.c_void_p(hs))
        if st:
            raise _abi.PsxError(st, L.psx_comm_last_error(self._c).decode())
        rsz = [int(x) for x in rs]
        recv = torch.empty(max(sum(rsz), 4), dtype=torch.uint8, device=send.device)
        st = L.psx_exchange_streams(self._c, send.data_ptr(), ss, recv.data_ptr(), rs, ctypes.c_void_p(hs))
        if st:
            raise _abi.PsxError(st, L.psx_comm_last_error(self._c).decode())
        return recv[:sum(rsz)], rsz


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
