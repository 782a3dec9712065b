"""CPU (gloo, world_size 2) tests of the multi-GPU path's logic.

Each rank is one worker AND one row-range shard.  A worker packs its clock's updates
into one message per owning shard (the reference client's per-server split,
row_oplog_serializer.hpp:100-124), the messages cross ranks through the same
all-to-all the GPU path runs over RCCL, and each owner applies what it received in
source-rank order.  The CPU oracle stands in for the GPU apply here (the GPU apply of
the same messages is covered by tests/test_dense_gpu.py); the per-shard results must be
bit-identical to one server applying every worker's messages in the same order.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHARD_ROWS, CAP, WORLD, CLOCKS = 96, 24, 2, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker_messages(worker, clock, world):
    """Worker `worker`'s messages for one clock: one dense stream per owner shard,
    rows of that shard in a worker/clock-specific random order, partial coverage."""
    import sys
    sys.path.insert(0, ROOT)
    from parameter_server_amd import wire
    rng = np.random.RandomState(1000 * clock + worker)
    msgs = []
    for owner in range(world):
        n = rng.randint(SHARD_ROWS // 2, SHARD_ROWS + 1)
        ids = (owner * SHARD_ROWS + rng.permutation(SHARD_ROWS)[:n]).astype(np.int32)
        msgs.append(wire.dense_stream_np(7, ids, rng.normal(0, 1, size=(n, CAP)).astype(np.float32)))
    return msgs


def _rank_main(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    from parameter_server_amd.exchange import alltoall_streams, split
    from oracle.oracle import OracleServer, DENSE, F32
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    bgs = [100 + w for w in range(world)]
    shard = OracleServer(bgs)            # CPU stand-in for this rank's GPU shard
    shard.create_table(7, DENSE, F32, CAP)
    for clock in range(CLOCKS):
        msgs = _worker_messages(rank, clock, world)
        send = torch.from_numpy(np.concatenate(msgs))
        recv, sizes = alltoall_streams(send, [m.size for m in msgs])
        parts = split(recv, sizes)
        for src, part in enumerate(parts):     # source-rank order = fused apply order
            data = part.numpy()
            ids = data[20:].view(np.int32).reshape(-1, 1 + CAP)[:, 0]
            assert ((ids // SHARD_ROWS) == rank).all()
            assert shard.apply_stream(data, bgs[src], clock) == 0
    rows = shard.read_dense_rows(7, rank * SHARD_ROWS, SHARD_ROWS)
    np.save(os.path.join(outdir, f"shard{rank}.npy"), rows)
    dist.barrier()
    dist.destroy_process_group()


def test_alltoall_exchange_then_ordered_apply_matches_single_server(tmp_path, oracle_lib):
    port = _free_port()
    mp.start_processes(_rank_main, args=(WORLD, port, str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    from oracle.oracle import OracleServer, DENSE, F32
    bgs = [100 + w for w in range(WORLD)]
    # Single-server reference: one oracle per owner shard fed in source-rank order.
    for owner in range(WORLD):
        srv = OracleServer(bgs)
        srv.create_table(7, DENSE, F32, CAP)
        for clock in range(CLOCKS):
            for w in range(WORLD):
                assert srv.apply_stream(_worker_messages(w, clock, WORLD)[owner], bgs[w], clock) == 0
        want = srv.read_dense_rows(7, owner * SHARD_ROWS, SHARD_ROWS)
        got = np.load(tmp_path / f"shard{owner}.npy")
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
