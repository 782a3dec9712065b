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
"""
import torch
import torch.distributed as dist


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
