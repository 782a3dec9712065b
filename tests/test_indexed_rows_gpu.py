"""psx_apply_indexed_rows: dense records placed from the producer's record-row lists
(psx_pack_stream_indexed's record_rows) instead of the stream's row ids, each record's
row id checked inside the apply.

Parity: bit-exact dense rows and byte-exact sorted-map rows against the checker
(oracle/psx_oracle.c walks the messages itself, Server::ApplyOpLogUpdateVersion,
server.cpp:120-179) and against the walked device path, for every dense dtype, mixed
listed / unlisted messages and multi-table messages.  Contract cases: a list that
disagrees with its stream (PSX_ERR_MALFORMED, those rows unchanged, the rest applied), a
list naming a row twice or outside the shard (replayed from the stream, exact), a stream
row outside the shard under a valid list (a disagreement), and tables whose kernel
ignores the lists."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError
from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, F64, I32, I64

pytestmark = pytest.mark.gpu

NPD = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64}


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _servers(rows, K, bgs, dtype=F32, importance=False):
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=dtype, row_capacity=K, max_rows=rows,
                                     accum_importance=importance))
    srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=K))
    orc = OracleServer(list(bgs))
    orc.create_table(1, DENSE, dtype, K, accum_importance=importance)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    return srv, orc


def _payload(rng, n, K, dtype):
    if dtype in (I32, I64):
        return rng.randint(-1000, 1000, size=(n, K)).astype(NPD[dtype])
    return rng.normal(0, 1, (n, K)).astype(NPD[dtype])


def _message(rng, rows, K, dtype, sparse=True):
    """(message bytes, record rows): sparse sorted-map records, then dense records."""
    ids = rng.permutation(rows)[:rng.randint(rows // 2, rows)].astype(np.int32)
    de = wire.dense_stream_np(1, ids, _payload(rng, ids.size, K, dtype))
    if not sparse:
        return de, ids
    srows = []
    for r in rng.permutation(rows)[:rng.randint(1, rows // 4)]:
        k = rng.randint(0, 17)
        cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
        srows.append((int(r), cols, rng.choice([-2, -1, 1, 2], size=k).astype(np.int32)))
    sp = wire.sparse_stream_np(3, 4, srows)
    msg = np.concatenate([np.array([2], np.int32).view(np.uint8), sp[4:], de[4:]])
    return msg, np.concatenate([np.array([r for r, _, _ in srows], np.int32), ids])


def _dev(arrs):
    return [torch.from_numpy(np.ascontiguousarray(a).copy()).cuda() for a in arrs]


@pytest.mark.parametrize("dtype", [F32, F64, I32, I64], ids=["f32", "f64", "i32", "i64"])
@pytest.mark.parametrize("B", [1, 3, 8])
def test_rows_match_checker_and_walk(B, dtype):
    rng = np.random.RandomState(10 * B + dtype)
    rows, K = 900, 72                    # 72 columns: a vector part and a scalar tail
    bgs = list(range(10, 10 + B))
    srv, orc = _servers(rows, K, bgs, dtype)
    walk, _ = _servers(rows, K, bgs, dtype)
    init = _payload(rng, rows, K, dtype)
    for s in (srv, walk):
        s.load_rows(1, 0, init[: rows // 2])
    orc.load_dense_rows(1, 0, init[: rows // 2])
    for rnd in range(3):
        pairs = [_message(rng, rows, K, dtype) for _ in range(B)]
        dm = _dev([m for m, _ in pairs])
        dr = _dev([r for _, r in pairs])
        # listed and unlisted messages in one call
        use = [r.data_ptr() if (b + rnd) % 3 != 1 else None for b, r in enumerate(dr)]
        torch.cuda.synchronize()
        srv.apply_indexed_rows([(d.data_ptr(), d.numel(), bg, rnd) for d, bg in zip(dm, bgs)], use)
        walk.apply_device([(d.data_ptr(), d.numel(), bg, rnd) for d, bg in zip(dm, bgs)])
        srv.sync()
        walk.sync()
        for (m, _), bg in zip(pairs, bgs):
            assert orc.apply_stream(m, bg, rnd) == 0
    got = srv.read_rows(1, 0, rows)
    assert np.array_equal(got.view(np.uint8), orc.read_dense_rows(1, 0, rows).view(np.uint8))
    assert np.array_equal(got.view(np.uint8), walk.read_rows(1, 0, rows).view(np.uint8))
    assert np.array_equal(srv.row_flags(1, 0, rows), walk.row_flags(1, 0, rows))
    ids = list(range(rows))
    assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids)
    srv.close()
    walk.close()


def test_pack_rows_drive_the_apply():
    """psx_pack_stream_indexed: record rows = the tables' row_ids in record order (ascending
    table id); applying with them matches the checker."""
    rng = np.random.RandomState(5)
    rows, K = 2000, 128
    packer = psa.Server(0, 9, [1])
    ids1 = rng.permutation(rows)[:1500].astype(np.int32)
    ids2 = rng.permutation(rows)[:700].astype(np.int32)
    ids3 = rng.permutation(rows)[:300].astype(np.int32)
    sp = np.where(rng.rand(300, K) < 0.9, 0, rng.randint(-5, 6, size=(300, K))).astype(np.int32)
    tabs = [dict(table_id=4, dtype=F32, dense_serialized=True, row_ids=torch.from_numpy(ids2).cuda(),
                 oplogs=torch.from_numpy(rng.normal(0, 1, (700, K)).astype(np.float32)).cuda()),
            dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=torch.from_numpy(ids1).cuda(),
                 oplogs=torch.from_numpy(rng.normal(0, 1, (1500, K)).astype(np.float32)).cuda()),
            dict(table_id=3, dtype=I32, dense_serialized=False, row_ids=torch.from_numpy(ids3).cuda(),
                 oplogs=torch.from_numpy(sp).cuda())]
    msg, idx, rws = packer.pack_stream(tabs, with_index=True, with_rows=True)
    assert np.array_equal(rws.cpu().numpy(), np.concatenate([ids1, ids3, ids2]))
    srv, orc = _servers(rows, K, [5])
    srv.CreateTable(4, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=K, max_rows=rows))
    orc.create_table(4, DENSE, F32, K)
    srv.apply_indexed_rows([(msg.data_ptr(), msg.numel(), 5, 0)], [rws.data_ptr()], [idx.data_ptr()])
    srv.sync()
    assert orc.apply_stream(msg.cpu().numpy(), 5, 0) == 0
    for t in (1, 4):
        assert np.array_equal(srv.read_rows(t, 0, rows).view(np.uint32), orc.read_dense_rows(t, 0, rows).view(np.uint32))
    assert srv.serialize_rows(3, list(range(rows))) == orc.serialize_records(3, list(range(rows)))
    packer.close()
    srv.close()


def _dense_setup(rows, K, B, seed):
    rng = np.random.RandomState(seed)
    bgs = list(range(1, B + 1))
    srv, orc = _servers(rows, K, bgs)
    init = rng.normal(0, 1, (rows, K)).astype(np.float32)
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    srv.clear_dirty(1)
    pairs = []
    for _ in range(B):             # full coverage: the v3 kernel (the one that checks lists)
        ids = rng.permutation(rows).astype(np.int32)
        pairs.append((wire.dense_stream_np(1, ids, rng.normal(0, 1, (rows, K)).astype(np.float32)), ids))
    return rng, bgs, srv, orc, init, pairs


def test_disagreeing_rows_leave_those_rows_unchanged():
    rows, K, B = 600, 64, 4
    rng, bgs, srv, orc, init, pairs = _dense_setup(rows, K, B, 11)
    lists = [r.copy() for _, r in pairs]
    a, b = 3, 40                       # message 2 claims record 3 is row lists[2][40] and vice versa
    lists[2][[a, b]] = lists[2][[b, a]]
    bad = {int(lists[2][a]), int(lists[2][b])}
    dm, dr = _dev([m for m, _ in pairs]), _dev(lists)
    torch.cuda.synchronize()
    srv.apply_indexed_rows([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dm, bgs)], [r.data_ptr() for r in dr])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 4
    for (m, _), bg in zip(pairs, bgs):
        assert orc.apply_stream(m, bg, 0) == 0
    got, want = srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows)
    flags = srv.row_flags(1, 0, rows)
    touched = set(np.concatenate([r for _, r in pairs]).tolist())
    for r in range(rows):
        if r in bad:
            assert np.array_equal(got[r].view(np.uint32), init[r].view(np.uint32)) and not flags[r] & 2
        else:
            assert np.array_equal(got[r].view(np.uint32), want[r].view(np.uint32))
            assert bool(flags[r] & 2) == (r in touched)
    srv.close()


def test_duplicate_in_rows_replays_from_the_stream():
    rows, K, B = 500, 64, 3
    rng, bgs, srv, orc, init, pairs = _dense_setup(rows, K, B, 12)
    lists = [r.copy() for _, r in pairs]
    lists[1][7] = lists[1][8]          # two records claim one row: counts fall short
    dm, dr = _dev([m for m, _ in pairs]), _dev(lists)
    torch.cuda.synchronize()
    srv.apply_indexed_rows([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dm, bgs)], [r.data_ptr() for r in dr])
    srv.sync()
    for (m, _), bg in zip(pairs, bgs):
        assert orc.apply_stream(m, bg, 0) == 0
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))
    srv.close()


def test_rows_outside_the_shard_replay_from_the_stream():
    """A listed row outside the shard drops that claim; the short count replays the call
    from the stream (whose row ids are valid): exact, no error."""
    rows, K, B = 400, 32, 3
    rng, bgs, srv, orc, init, pairs = _dense_setup(rows, K, B, 13)
    lists = [r.copy() for _, r in pairs]
    lists[1][0] = rows + 5
    dm, dr = _dev([m for m, _ in pairs]), _dev(lists)
    torch.cuda.synchronize()
    srv.apply_indexed_rows([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dm, bgs)], [r.data_ptr() for r in dr])
    srv.sync()
    for (m, _), bg in zip(pairs, bgs):
        assert orc.apply_stream(m, bg, 0) == 0
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))
    srv.close()


def test_stream_row_outside_the_shard_disagrees():
    """A stream row id outside the shard under a valid list entry is a disagreement:
    PSX_ERR_MALFORMED, the listed row unchanged, every other row applied."""
    rows, K, B = 400, 32, 3
    rng, bgs, srv, orc, init, pairs = _dense_setup(rows, K, B, 14)
    m1 = pairs[1][0].copy()
    m1[20:24] = np.array([rows + 7], np.int32).view(np.uint8)     # record 0's row id
    r0 = int(pairs[1][1][0])
    dm, dr = _dev([pairs[0][0], m1, pairs[2][0]]), _dev([r for _, r in pairs])
    torch.cuda.synchronize()
    srv.apply_indexed_rows([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dm, bgs)], [r.data_ptr() for r in dr])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 4
    for (m, _), bg in zip(pairs, bgs):
        assert orc.apply_stream(m, bg, 0) == 0
    got, want = srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows)
    others = np.arange(rows) != r0
    assert np.array_equal(got[others].view(np.uint32), want[others].view(np.uint32))
    assert np.array_equal(got[r0].view(np.uint32), init[r0].view(np.uint32))
    assert not srv.row_flags(1, r0, 1)[0] & 2
    srv.close()


def test_importance_tables_index_from_the_stream():
    """Importance tables (the v2 IMP kernel) do not check lists, so they index from the
    stream: a wrong list changes nothing."""
    rng = np.random.RandomState(21)
    rows, K, B = 4000, 64, 4
    bgs = list(range(1, B + 1))
    srv, orc = _servers(rows, K, bgs, importance=True)
    pairs = []
    for _ in range(B):
        ids = rng.permutation(rows).astype(np.int32)
        pairs.append((wire.dense_stream_np(1, ids, rng.normal(0, 1, (rows, K)).astype(np.float32)), ids))
    lists = [np.roll(r, 1) for _, r in pairs]          # every entry wrong
    dm, dr = _dev([m for m, _ in pairs]), _dev(lists)
    torch.cuda.synchronize()
    srv.apply_indexed_rows([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dm, bgs)], [r.data_ptr() for r in dr])
    srv.sync()
    for (m, _), bg in zip(pairs, bgs):
        assert orc.apply_stream(m, bg, 0) == 0
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))
    srv.close()


def test_partial_coverage_indexes_from_the_stream():
    """Partially covered calls take the compact v4 kernel, which does not check lists
    (profiles/r02/ab_v4_rows.json), so they index from the stream: a wrong list changes
    nothing."""
    rng = np.random.RandomState(23)
    rows, K, B = 4000, 64, 4
    bgs = list(range(1, B + 1))
    srv, orc = _servers(rows, K, bgs)
    pairs = []
    for _ in range(B):
        ids = rng.permutation(rows)[: rows // 8].astype(np.int32)
        pairs.append((wire.dense_stream_np(1, ids, rng.normal(0, 1, (ids.size, K)).astype(np.float32)), ids))
    lists = [np.roll(r, 1) for _, r in pairs]          # every entry wrong
    dm, dr = _dev([m for m, _ in pairs]), _dev(lists)
    torch.cuda.synchronize()
    srv.apply_indexed_rows([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dm, bgs)], [r.data_ptr() for r in dr])
    srv.sync()
    for (m, _), bg in zip(pairs, bgs):
        assert orc.apply_stream(m, bg, 0) == 0
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))
    srv.close()


def test_c2_full_size_rows_bit_exact():
    """The headline shape (2^20 x 256 f32, 8 full-coverage messages) through the record
    rows, two calls, bit-exact against the in-order fp32 torch sum."""
    rows, cap, B = 1 << 20, 256, 8
    g = torch.Generator(device="cuda").manual_seed(2025)
    table0 = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
    bgs = [100 + b for b in range(B)]
    srv = psa.Server(0, 1, bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=rows)
    ref = table0.clone()
    for ver in range(2):
        streams, perms = [], []
        for b in range(B):
            perm = torch.randperm(rows, device="cuda", generator=g)
            upd = torch.randn(rows, cap, device="cuda", generator=g) * 0.01
            streams.append(wire.dense_stream_torch(1, perm.to(torch.int32), upd))
            perms.append(perm.to(torch.int32))
            ref[perm] = ref[perm] + upd
            del upd
        torch.cuda.synchronize()
        srv.apply_indexed_rows([(s.data_ptr(), s.numel(), bg, ver) for s, bg in zip(streams, bgs)],
                               [p.data_ptr() for p in perms])
        srv.sync()
        del streams, perms
    got = torch.empty_like(ref)
    from parameter_server_amd import _abi
    assert _abi.load().psx_table_read_rows(srv.handle, 1, 0, rows, got.data_ptr(), 1) == 0
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    srv.close()


@pytest.mark.parametrize("mode", [1, 2], ids=["listed", "all"])
def test_pipelined_calls_bit_exact(mode):
    """psx_ctx_set_pipeline: consecutive calls without a sync between them, each call's
    index stage overlapping the previous call's apply (listed and walked calls mixed),
    bit-exact against the checker."""
    rows, K, B, calls = 3000, 64, 3, 6
    rng = np.random.RandomState(30 + mode)
    bgs = list(range(1, B + 1))
    srv, orc = _servers(rows, K, bgs)
    srv.set_pipeline(mode)
    keep = []
    for c in range(calls):
        pairs = []
        for _ in range(B):
            ids = rng.permutation(rows).astype(np.int32)
            pairs.append((wire.dense_stream_np(1, ids, rng.normal(0, 1, (rows, K)).astype(np.float32)), ids))
        dm, dr = _dev([m for m, _ in pairs]), _dev([r for _, r in pairs])
        keep.append((dm, dr))
        torch.cuda.synchronize()
        msgs = [(d.data_ptr(), d.numel(), bg, c) for d, bg in zip(dm, bgs)]
        if c % 3 == 2:
            srv.apply_device(msgs)
        else:
            srv.apply_indexed_rows(msgs, [r.data_ptr() for r in dr])
        for (m, _), bg in zip(pairs, bgs):
            assert orc.apply_stream(m, bg, c) == 0
    srv.sync()
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))
    srv.close()

