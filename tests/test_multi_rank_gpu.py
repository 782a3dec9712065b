"""Two ranks (processes) on one GPU: the multi-GPU step with libpsx on both sides of the
transport.  Each rank is one worker and one row-range shard (a psx context with
row_offset = rank x S).  Per clock a worker packs one message covering rows of every
shard (dense and sorted-map tables), splits it on the device by owner
(psx_split_stream: AbstractBgWorker::CreateOpLogMsgs, abstract_bg_worker.cpp:590-649), the
sub-streams cross ranks (gloo all-to-all here — RCCL cannot put two ranks on one GPU; the
RCCL exchange itself is tested as a one-rank self exchange in tests/test_split_gpu.py) and
each owner applies what it received in one fused psx_apply_streams_device call in
source-rank order.  Every shard must equal one oracle server (oracle/psx_oracle.c,
Server::ApplyOpLogUpdateVersion, server.cpp:120-179) applying every worker's whole message
in the same order: dense rows bit-exact, sorted-map rows byte-exact."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S, K, WORLD, CLOCKS = 700, 48, 2, 3


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker_message(worker, clock):
    """Worker `worker`'s whole message for one clock (rows of every shard)."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle.oracle import pack_stream, F32, I32
    rng = np.random.RandomState(100 * clock + worker)
    R = S * WORLD
    ids1 = rng.permutation(R)[: rng.randint(R // 2, R)].astype(np.int32)
    ids3 = rng.permutation(R)[: rng.randint(R // 4, R // 2)].astype(np.int32)
    sp = np.where(rng.rand(ids3.size, K) < 0.8, 0, rng.randint(-3, 4, size=(ids3.size, K))).astype(np.int32)
    if clock == 0:
        sp = np.abs(sp)
    tabs = [dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=ids1,
                 oplogs=rng.normal(0, 1, (ids1.size, K)).astype(np.float32)),
            dict(table_id=3, dtype=I32, dense_serialized=False, row_ids=ids3, oplogs=sp)]
    return np.frombuffer(pack_stream(tabs), np.uint8).copy()


def _rank_main(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import parameter_server_amd as psa
    from parameter_server_amd.exchange import alltoall_streams, split
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    bgs = [100 + w for w in range(world)]
    lo = rank * S
    shard = psa.Server(0, 1 + rank, bgs)
    shard.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=K, row_offset=lo, max_rows=S))
    shard.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=K,
                                       oplog_dense_serialized=False, row_offset=lo, max_rows=S, max_entries=K))
    bounds = [w * S for w in range(world + 1)]
    for clock in range(CLOCKS):
        msg = torch.from_numpy(_worker_message(rank, clock)).cuda()
        out, sizes = shard.split_stream(msg, bounds)                  # device split by owner
        recv, rsizes = alltoall_streams(out.cpu(), sizes)             # gloo transport (CPU)
        parts = [p.cuda() for p in split(recv, rsizes)]
        torch.cuda.synchronize()
        # one fused, order-preserving apply of every source rank's sub-stream
        shard.apply_device([(p.data_ptr() if p.numel() else 0, p.numel(), bgs[src], clock)
                            for src, p in enumerate(parts)])
        shard.sync()
    np.save(os.path.join(outdir, f"dense{rank}.npy"), shard.read_rows(1, lo, S))
    with open(os.path.join(outdir, f"sorted{rank}.bin"), "wb") as f:
        f.write(shard.serialize_rows(3, list(range(lo, lo + S))))
    shard.close()
    dist.barrier()
    dist.destroy_process_group()


def test_device_split_exchange_fused_apply_matches_one_server(tmp_path):
    import torch.multiprocessing as mp
    from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, I32
    port = _free_port()
    mp.start_processes(_rank_main, args=(WORLD, port, str(tmp_path)), nprocs=WORLD, join=True, start_method="spawn")
    bgs = [100 + w for w in range(WORLD)]
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, K)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    for clock in range(CLOCKS):
        for w in range(WORLD):
            assert orc.apply_stream(_worker_message(w, clock), bgs[w], clock) == 0
    for owner in range(WORLD):
        lo = owner * S
        got = np.load(tmp_path / f"dense{owner}.npy")
        assert np.array_equal(got.view(np.uint32), orc.read_dense_rows(1, lo, S).view(np.uint32)), f"shard {owner}"
        assert (tmp_path / f"sorted{owner}.bin").read_bytes() == orc.serialize_records(3, list(range(lo, lo + S)))
