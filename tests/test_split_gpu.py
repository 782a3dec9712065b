"""The multi-GPU path's two device steps, through the C ABI:

psx_split_stream — the client's per-server split (AbstractBgWorker::CreateOpLogMsgs,
abstract_bg_worker.cpp:590-649, routing rows by owner, row_oplog_serializer.hpp:100-124)
of one packed message over row-range owners.  Every owner's sub-stream must be
byte-identical to the oracle's restatement of the reference packer run on that owner's rows
(same tables in the same order, records in message order), and applying the sub-streams
to per-owner shards must equal the oracle applying the whole message.

psx_exchange_sizes / psx_exchange_streams — libpsx's RCCL all-to-all-v, on one GPU as a
one-rank communicator (a self send/receive); the N-rank exchange runs in bench.py --gpus N
(driver-run) and its routing logic in tests/test_multi_rank.py (gloo, world 2)."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import _abi, PsxError
from oracle.oracle import OracleServer, pack_stream, DENSE, SORTED_MAP, F32, F64, I32

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _tables(rng, R, K, rows_per_table=(None, None, None)):
    """Three tables (ascending id): dense f32 (1), sparse sorted-map int32 (3), dense f64 (4)."""
    n1, n3, n4 = [rng.randint(R // 3, R) if r is None else r for r in rows_per_table]
    sp = np.where(rng.rand(n3, K) < 0.85, 0, rng.randint(-3, 4, size=(n3, K))).astype(np.int32)
    return [dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=rng.permutation(R)[:n1].astype(np.int32),
                 oplogs=rng.normal(0, 1, (n1, K)).astype(np.float32)),
            dict(table_id=3, dtype=I32, dense_serialized=False, row_ids=rng.permutation(R)[:n3].astype(np.int32),
                 oplogs=sp),
            dict(table_id=4, dtype=F64, dense_serialized=True, row_ids=rng.permutation(R)[:n4].astype(np.int32),
                 oplogs=rng.normal(0, 1, (n4, K)).astype(np.float64))]


def _server(R, K, row_offset=0, max_rows=None, bgs=(7,)):
    s = psa.Server(0, 1, list(bgs))
    s.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=K, max_rows=max_rows or R,
                                   row_offset=row_offset))
    s.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                   max_rows=max_rows or R, max_entries=K, row_offset=row_offset))
    s.CreateTable(4, psa.TableInfo(row_kind=DENSE, dtype=F64, row_capacity=K, max_rows=max_rows or R,
                                   row_offset=row_offset))
    return s


def _expected(tables, lo, hi):
    sub = []
    for t in tables:
        m = (t["row_ids"] >= lo) & (t["row_ids"] < hi)
        sub.append(dict(t, row_ids=t["row_ids"][m], oplogs=t["oplogs"][m]))
    return pack_stream(sub)


@pytest.mark.parametrize("owners", [1, 3, 8])
@pytest.mark.parametrize("indexed", [False, True])
def test_split_equals_reference_packer_per_owner_and_applies_exactly(owners, indexed):
    rng = np.random.RandomState(11 * owners + indexed)
    R, K = 3000, 40
    tables = _tables(rng, R, K)
    msg = np.frombuffer(pack_stream(tables), np.uint8)
    bounds = np.linspace(0, R, owners + 1).astype(np.int64)
    bounds[1:-1] += rng.randint(-50, 50, size=owners - 1)
    srv = _server(R, K)
    d = torch.from_numpy(msg.copy()).cuda()
    idx = None
    if indexed:
        from parameter_server_amd import wire
        idx = torch.from_numpy(wire.stream_record_offsets(msg, {1: 4 * K, 3: None, 4: 8 * K}).view(np.int64)).cuda()
    out, sizes = srv.split_stream(d, bounds, record_offsets=idx)
    host = out.cpu().numpy().tobytes()
    off = 0
    for o in range(owners):
        want = _expected(tables, bounds[o], bounds[o + 1])
        assert host[off:off + sizes[o]] == want, f"owner {o}"
        off += sizes[o]
    # apply the sub-streams to per-owner shards; the oracle applies the whole message
    orc = OracleServer([7])
    orc.create_table(1, DENSE, F32, K)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    orc.create_table(4, DENSE, F64, K)
    assert orc.apply_stream(msg, 7, 0) == 0
    off = 0
    for o in range(owners):
        lo, hi = int(bounds[o]), int(bounds[o + 1])
        shard = _server(R, K, row_offset=lo, max_rows=max(hi - lo, 1))
        part = out[off:off + sizes[o]]
        off += sizes[o]
        shard.apply_device([(part.data_ptr(), sizes[o], 7, 0)])
        shard.sync()
        if hi > lo:
            for tid in (1, 4):
                assert np.array_equal(shard.read_rows(tid, lo, hi - lo).view(np.uint8),
                                      orc.read_dense_rows(tid, lo, hi - lo).view(np.uint8))
            ids = list(range(lo, hi))
            assert shard.serialize_rows(3, ids) == orc.serialize_records(3, ids)
        shard.close()
    srv.close()


def test_split_many_owners_large_dense_message():
    """16 owners, 200K dense records of 64 f32 (3,125 tiles of 64 records)."""
    rng = np.random.RandomState(3)
    R, K, N = 400_000, 64, 200_000
    ids = rng.permutation(R)[:N].astype(np.int32)
    tables = [dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=ids,
                   oplogs=rng.normal(0, 1, (N, K)).astype(np.float32))]
    msg = np.frombuffer(pack_stream(tables), np.uint8)
    srv = psa.Server(0, 1, [7])
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=K, max_rows=R))
    bounds = np.arange(17, dtype=np.int64) * (R // 16)
    out, sizes = srv.split_stream(torch.from_numpy(msg.copy()).cuda(), bounds)
    host = out.cpu().numpy().tobytes()
    off = 0
    for o in range(16):
        assert host[off:off + sizes[o]] == _expected(tables, bounds[o], bounds[o + 1]), f"owner {o}"
        off += sizes[o]
    srv.close()


def test_split_row_outside_every_owner_is_row_range():
    rng = np.random.RandomState(5)
    R, K = 500, 16
    tables = _tables(rng, R, K)
    msg = np.frombuffer(pack_stream(tables), np.uint8)
    srv = _server(R, K)
    with pytest.raises(PsxError) as e:
        srv.split_stream(torch.from_numpy(msg.copy()).cuda(), [0, 200, 400])   # rows 400.. have no owner
    assert e.value.status == 5
    srv.close()


def test_rccl_exchange_one_rank_self_send():
    """psx_comm_* on one GPU: a one-rank communicator sends its sub-stream to itself."""
    L = _abi.load()
    uid = (ctypes.c_uint8 * 128)()
    assert L.psx_comm_unique_id(uid) == 0
    comm = ctypes.c_void_p()
    st = L.psx_comm_create(uid, 1, 0, 0, ctypes.byref(comm))
    assert st == 0, L.psx_comm_last_error(None)
    try:
        rng = np.random.RandomState(9)
        send = torch.from_numpy(rng.randint(0, 256, size=4096, dtype=np.uint8)).cuda()
        ss = (ctypes.c_uint64 * 1)(4096)
        rs = (ctypes.c_uint64 * 1)()
        stream = torch.cuda.current_stream().cuda_stream
        assert L.psx_exchange_sizes(comm, ss, rs, ctypes.c_void_p(stream)) == 0, L.psx_comm_last_error(comm)
        assert rs[0] == 4096
        recv = torch.empty(4096, dtype=torch.uint8, device="cuda")
        assert L.psx_exchange_streams(comm, send.data_ptr(), ss, recv.data_ptr(), rs, ctypes.c_void_p(stream)) == 0
        torch.cuda.synchronize()
        assert torch.equal(send, recv)
        bad = (ctypes.c_uint64 * 1)(4095)
        assert L.psx_exchange_sizes(comm, bad, rs, ctypes.c_void_p(stream)) == 1
    finally:
        L.psx_comm_destroy(comm)


def _formats(K):
    return {1: psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=K),
            3: psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                             max_entries=K),
            4: psa.TableInfo(row_kind=DENSE, dtype=F64, row_capacity=K)}


@pytest.mark.parametrize("owners", [1, 5])
def test_split_with_formats_equals_split_with_tables(owners):
    """psx_split_stream_formats (a context with no tables, record formats from the caller)
    writes the same sub-streams as psx_split_stream over a context holding the tables."""
    rng = np.random.RandomState(40 + owners)
    R, K = 2500, 24
    tables = _tables(rng, R, K)
    msg = np.frombuffer(pack_stream(tables), np.uint8)
    d = torch.from_numpy(msg.copy()).cuda()
    bounds = np.linspace(0, R, owners + 1).astype(np.int64)
    srv = _server(R, K)
    out_t, sz_t = srv.split_stream(d, bounds)
    bare = psa.Server(0, 2)
    out_f, sz_f = bare.split_stream(d, bounds, formats=_formats(K))
    assert sz_f == sz_t
    assert torch.equal(out_f, out_t)
    off = 0
    for o in range(owners):
        assert out_f[off:off + sz_f[o]].cpu().numpy().tobytes() == _expected(tables, bounds[o], bounds[o + 1])
        off += sz_f[o]
    # a table missing from the formats is an unknown table; a bad format is rejected
    with pytest.raises(PsxError) as e:
        bare.split_stream(d, bounds, formats={1: _formats(K)[1]})
    assert e.value.status == 3
    with pytest.raises(PsxError) as e:
        bare.split_stream(d, bounds, formats={1: psa.TableInfo(row_kind=DENSE, dtype=9, row_capacity=K)})
    assert e.value.status == 1
    srv.close()
    bare.close()


def test_split_dense_only_formats_into_preallocated_output():
    """A dense-only split writes into the caller's buffer and needs no record-offset buffer."""
    rng = np.random.RandomState(77)
    R, K, N = 50_000, 32, 40_000
    ids = rng.permutation(R)[:N].astype(np.int32)
    tables = [dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=ids,
                   oplogs=rng.normal(0, 1, (N, K)).astype(np.float32))]
    msg = np.frombuffer(pack_stream(tables), np.uint8)
    bounds = [0, 10_000, 31_000, R]
    bare = psa.Server(0, 2)
    out = torch.empty(msg.size + 3 * 20 + 64, dtype=torch.uint8, device="cuda")
    part, sizes = bare.split_stream(torch.from_numpy(msg.copy()).cuda(), bounds,
                                    formats={1: psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=K)}, out=out)
    assert part.data_ptr() == out.data_ptr()
    host, off = part.cpu().numpy().tobytes(), 0
    for o in range(3):
        assert host[off:off + sizes[o]] == _expected(tables, bounds[o], bounds[o + 1])
        off += sizes[o]
    bare.close()


def test_rccl_exchange_sizes_async_one_rank():
    """psx_exchange_sizes_async: the sizes land in page-locked memory once the stream passes;
    a pageable destination is rejected."""
    from parameter_server_amd.exchange import Exchange
    xc = Exchange(0)
    s = torch.cuda.Stream()
    rs = torch.zeros(1, dtype=torch.int64).pin_memory()
    xc.sizes_async([1024], rs, s.cuda_stream)
    s.synchronize()
    assert int(rs[0]) == 1024
    for k in range(20):                      # the staging ring wraps
        xc.sizes_async([4 * k], rs, s.cuda_stream)
        s.synchronize()
        assert int(rs[0]) == 4 * k
    with pytest.raises(AssertionError):
        xc.sizes_async([8], torch.zeros(1, dtype=torch.int64), s.cuda_stream)
    L = _abi.load()
    page = (ctypes.c_uint64 * 1)()
    assert L.psx_exchange_sizes_async(xc._c, (ctypes.c_uint64 * 1)(8), page, ctypes.c_void_p(s.cuda_stream)) == 1
    with pytest.raises(ValueError):
        xc.alltoall(torch.zeros(8, dtype=torch.uint8, device="cuda"), [12])
    xc.close()


@pytest.mark.parametrize("rows,cap,chunk_recs", [(20_000, 64, 3_000), (9_000, 256, 9_000), (7_777, 40, 1_000)])
def test_shard_exchange_pipeline_one_rank_bit_exact(rows, cap, chunk_recs):
    """The exchange-bearing step through ShardExchange on one GPU (self exchange): a batch of
    several < max_bytes messages per step, split (formats only), exchanged, applied in chunk
    order with chunk k's exchange beside chunk k-1's apply, three steps — bit for bit equal to
    the in-order f32 sum recomputed from the seeds (bench.exchange_measure's check)."""
    import bench
    for split_single in (True, False):   # the split + own sub-stream path, then the direct one
        m = bench.exchange_measure(rows, cap, 2, 1, 1, 0, 0, seed=7 + rows, max_bytes=20 + (4 + 4 * cap) * chunk_recs,
                                   split_single=split_single)
        assert m["parity"] == "bit-exact", (split_single, m)
        assert m["chunks_per_step"] == -(-rows // chunk_recs)
        assert m["apply_kernel_ms_per_chunk"] and m["exchange_kernel_ms_per_step"] is not None


@pytest.mark.parametrize("nbytes", [(1 << 31) - 2028, (1 << 31) + 4096 * 3])
def test_rccl_exchange_large_sub_stream_in_pieces(nbytes):
    """A sub-stream near and past 2 GiB crosses intact (psx_exchange_streams sends it in
    512 MiB pieces: this RCCL corrupts a single ~2 GiB point-to-point transfer)."""
    from parameter_server_amd.exchange import Exchange
    xc = Exchange(0)
    g = torch.Generator(device="cuda").manual_seed(nbytes)
    send = torch.randint(-2 ** 31, 2 ** 31 - 1, (nbytes // 4,), generator=g, dtype=torch.int32,
                         device="cuda").view(torch.uint8)
    recv, rs = xc.alltoall(send, [nbytes])
    torch.cuda.synchronize()
    assert rs == [nbytes]
    assert torch.equal(recv, send)
    xc.close()


def test_rccl_exchange_streams_v_displacements_one_rank():
    """psx_exchange_streams_v: a sub-stream taken from a send displacement lands at the
    receive displacement; a zero size moves nothing."""
    from parameter_server_amd.exchange import Exchange
    xc = Exchange(0)
    s = torch.cuda.Stream()
    send = torch.arange(4096, dtype=torch.int32, device="cuda").view(torch.uint8)
    recv = torch.full((8192,), 7, dtype=torch.uint8, device="cuda")
    xc.streams_v(send, [1024], [2048], recv, [1024], [4096], s.cuda_stream)
    s.synchronize()
    assert torch.equal(recv[4096:5120], send[2048:3072])
    assert bool((recv[:4096] == 7).all()) and bool((recv[5120:] == 7).all())
    xc.streams_v(send, [0], [0], recv, [0], [0], s.cuda_stream)
    s.synchronize()
    with pytest.raises(ValueError):
        xc.streams_v(send, [1024], [16000], recv, [1024], [0], s.cuda_stream)
    xc.close()


def _selftest_device(world, port, extra=()):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--steps", "2",
                          "--warmup", "1", "--selftest-exchange", "--selftest-device",
                          "--master-port", str(port)] + list(extra),
                         capture_output=True, text=True, timeout=150, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world,port", [(2, 29611), (3, 29612), (4, 29613)])
def test_shard_exchange_multi_rank_on_one_gpu_bit_exact(world, port):
    """ShardExchange's N-rank routing with the real device split and apply: `world` ranks
    share cuda:0 and their sub-streams cross over gloo (bench.GlooExchange), each rank's own
    sub-stream applied from its send slot.  Every owner's shard must equal the in-order sum
    recomputed from the seeds, bit for bit, after 3 steps of 14-28 chunks."""
    rec = _selftest_device(world, port)
    assert rec["n_gpus"] == world and rec["parity"] == "bit-exact", rec
    assert rec["chunks_per_step"] > 5
