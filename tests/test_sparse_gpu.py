"""GPU parity of the ordered (sparse-record) apply path vs the CPU oracle.

SortedVectorMapRow rows are compared BYTE-FOR-BYTE on their serialized form, i.e. the
history-dependent entry order of SortedVectorMapStore (sorted_vector_map_store.hpp) is
reproduced exactly; SparseRow (MapStore) rows are compared as {col -> value} maps (the
reference's own order is unordered_map iteration order); DenseRow rows bit-exact."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError, _abi
from oracle.oracle import OracleServer, pack_stream, DENSE, SORTED_MAP, MAP, F32, F64, I32, I64

pytestmark = pytest.mark.gpu
NP = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64}
VS = {F32: 4, F64: 8, I32: 4, I64: 8}


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _sparse_rows(rng, rows, ncols, nrec, dt, max_nnz=32, positive=False):
    out = []
    for rid in rng.choice(rows, size=nrec, replace=False):
        k = rng.randint(1, min(max_nnz, ncols) + 1)
        cols = np.sort(rng.choice(ncols, size=k, replace=False)).astype(np.int32)
        if dt in (I32, I64):
            v = rng.randint(1, 4, size=k) * (1 if positive else rng.choice([-1, 1], size=k))
        else:
            v = rng.normal(0, 1, size=k)
        out.append((int(rid), cols, v.astype(NP[dt])))
    return out


def _pair(kind, dt, rows, ncols, max_entries=None, bgs=range(100, 116)):
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=dt, row_capacity=ncols, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=max_entries or ncols))
    orc = OracleServer(list(bgs))
    orc.create_table(3, kind, dt, ncols if kind == DENSE else 0, oplog_dense_serialized=False)
    return srv, orc


def _apply(srv, orc, streams, bgs, vers=None):
    vers = vers or [0] * len(streams)
    dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg, v in zip(dev, bgs, vers)])
    srv.sync()
    for s, bg, v in zip(streams, bgs, vers):
        assert orc.apply_stream(s, bg, v) == 0


def _as_map(raw, dt, packed):
    vs = VS[dt]
    es = (4 + vs) if packed else (8 if vs == 4 else 16)
    out = {}
    for k in range(len(raw) // es):
        e = raw[k * es:(k + 1) * es]
        col = int(np.frombuffer(e[:4], np.int32)[0])
        off = 4 if (packed or vs == 4) else 8
        out[col] = np.frombuffer(e[off:off + vs], NP[dt])[0]
    return out


@pytest.mark.parametrize("dt", [I32, F32, I64, F64])
def test_sorted_map_rows_byte_exact(dt):
    rng = np.random.RandomState(7 + dt)
    rows, K, B = 3000, 96, 8
    srv, orc = _pair(SORTED_MAP, dt, rows, K)
    bgs = list(range(100, 100 + B))
    streams = [wire.sparse_stream_np(3, VS[dt], _sparse_rows(rng, rows, K, 400, dt, positive=(b == 0)))
               for b in range(B)]
    _apply(srv, orc, streams, bgs)
    ids = list(range(rows))
    assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids)


def test_sorted_map_zero_crossing_and_growth():
    """Entries reach zero and are removed (compaction), rows grow past 64 entries
    (the store's kBlockSize), and values tie (strict > in LinearSearchAndMove)."""
    rows, K = 16, 200
    srv, orc = _pair(SORTED_MAP, I32, rows, K)
    bgs = [100, 101, 102]
    cols = np.arange(0, 150, dtype=np.int32)
    s0 = wire.sparse_stream_np(3, 4, [(r, cols, (cols % 5 + 1).astype(np.int32)) for r in range(rows)])
    s1 = wire.sparse_stream_np(3, 4, [(r, cols[::2], -(cols[::2] % 5 + 1).astype(np.int32)) for r in range(rows)])
    s2 = wire.sparse_stream_np(3, 4, [(r, np.arange(150, 200, dtype=np.int32), np.full(50, 3, np.int32))
                                      for r in range(0, rows, 2)])
    _apply(srv, orc, [s0, s1, s2], bgs)
    assert srv.serialize_rows(3, list(range(rows))) == orc.serialize_records(3, list(range(rows)))


def test_lda_like_plus_minus_one_stream_over_several_calls():
    """Collapsed-Gibbs style +1/-1 count updates (fast_doc_sampler.cpp:164-174) over many
    calls: the store order keeps evolving between calls."""
    rng = np.random.RandomState(3)
    rows, K = 500, 64
    srv, orc = _pair(SORTED_MAP, I32, rows, K)
    ver = 0
    for step in range(6):
        recs = []
        for rid in rng.choice(rows, size=200, replace=False):
            cols = np.sort(rng.choice(K, size=rng.randint(1, 6), replace=False)).astype(np.int32)
            vals = (np.ones(cols.size) if step == 0 else rng.choice([-1, 1], size=cols.size)).astype(np.int32)
            recs.append((int(rid), cols, vals))
        _apply(srv, orc, [wire.sparse_stream_np(3, 4, recs)], [100], [ver])
        ver += 1
    assert srv.serialize_rows(3, list(range(rows))) == orc.serialize_records(3, list(range(rows)))


@pytest.mark.parametrize("dt", [I32, F64])
def test_map_rows_value_maps(dt):
    rng = np.random.RandomState(11)
    rows, K, B = 800, 50, 5
    srv, orc = _pair(MAP, dt, rows, K)
    bgs = list(range(100, 100 + B))
    streams = [wire.sparse_stream_np(3, VS[dt], _sparse_rows(rng, rows, K, 300, dt)) for _ in range(B)]
    _apply(srv, orc, streams, bgs)
    for r in range(rows):
        g = srv.serialize_rows(3, [r])
        w = orc.serialize_records(3, [r])
        assert len(g) == len(w)
        if not g:
            continue
        gm, wm = _as_map(g[12:], dt, True), _as_map(w[12:], dt, True)
        assert gm.keys() == wm.keys()
        for k in gm:
            assert np.array_equal(np.array([gm[k]]).view(np.uint8), np.array([wm[k]]).view(np.uint8))


@pytest.mark.parametrize("dt", [F32, I64])
def test_dense_rows_from_sparse_records(dt):
    """DenseRow with oplog_dense_serialized = false: VectorStore::Inc per (col, val),
    including a record with repeated / descending columns (sequential fallback)."""
    rng = np.random.RandomState(5)
    rows, K, B = 400, 70, 6
    srv, orc = _pair(DENSE, dt, rows, K)
    bgs = list(range(100, 100 + B))
    streams = [wire.sparse_stream_np(3, VS[dt], _sparse_rows(rng, rows, K, 150, dt)) for _ in range(B - 1)]
    odd = [(7, np.array([5, 3, 5, 69], np.int32), np.array([1, 2, 3, 4], NP[dt])),
           (9, np.array([0], np.int32), np.array([9], NP[dt]))]
    streams.append(wire.sparse_stream_np(3, VS[dt], odd))
    _apply(srv, orc, streams, bgs)
    got = srv.read_rows(3, 0, rows)
    want = orc.read_dense_rows(3, 0, rows)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_sparse_column_out_of_range_applies_nothing():
    srv, _ = _pair(DENSE, F32, 10, 8, bgs=[100])
    bad = wire.sparse_stream_np(3, 4, [(1, np.array([2], np.int32), np.ones(1, np.float32)),
                                       (2, np.array([8], np.int32), np.ones(1, np.float32))])
    d = torch.from_numpy(bad).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 6
    assert not srv.read_rows(3, 0, 10).any()


@pytest.mark.parametrize("kind,max_entries,err", [(SORTED_MAP, 96, "row"), (SORTED_MAP, 512, "row"),
                                                   (SORTED_MAP, 512, "col"), (MAP, 96, "row"), (DENSE, None, "col")],
                         ids=["sorted-row", "sorted-split-row", "sorted-split-col", "map-row", "dense-col"])
def test_failed_call_then_valid_call_matches_oracle(kind, max_entries, err):
    """A call that ordered_count rejects part-way (a row outside the shard, or a column
    outside a dense row / a sorted map's key range), then a valid call on the same context:
    the failed call applies nothing and leaves no per-slot counts behind, so the next call
    equals the oracle applying only it (stale counts dropped updates); it gives its
    version back, so the next call reuses it."""
    rng = np.random.RandomState(41)
    rows, K = 600, 96
    srv, orc = _pair(kind, I32, rows, K, max_entries=max_entries, bgs=[100])
    recs = _sparse_rows(rng, rows, K, 500, I32, positive=True)
    if err == "row":
        recs.insert(250, (rows + 7, np.array([1], np.int32), np.ones(1, np.int32)))
    elif kind == DENSE:
        recs.insert(250, (3, np.array([K], np.int32), np.ones(1, np.int32)))
    else:
        # a key outside [0, max_entries) of a row already holding max_entries entries
        recs = [(5, np.arange(max_entries, dtype=np.int32), np.ones(max_entries, np.int32))] + recs[1:]
        recs.insert(250, (5, np.array([max_entries + 3], np.int32), np.ones(1, np.int32)))
    bad = torch.from_numpy(wire.sparse_stream_np(3, 4, recs)).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(bad.data_ptr(), bad.numel(), 100, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status in (5, 6)
    assert "version given back" in str(e.value) and srv.GetBgVersion(100) == -1
    good = wire.sparse_stream_np(3, 4, _sparse_rows(rng, rows, K, 500, I32, positive=True))
    _apply(srv, orc, [good], [100], [0])                            # the rejected call's version again
    if kind == DENSE:
        assert np.array_equal(srv.read_rows(3, 0, rows), orc.read_dense_rows(3, 0, rows))
    elif kind == SORTED_MAP:
        assert srv.serialize_rows(3, list(range(rows))) == orc.serialize_records(3, list(range(rows)))
    else:
        for r in range(rows):
            g, w = srv.serialize_rows(3, [r]), orc.serialize_records(3, [r])
            assert len(g) == len(w) and (not g or _as_map(g[12:], I32, True) == _as_map(w[12:], I32, True))


def test_sorted_map_capacity_overflow_reported():
    srv, _ = _pair(SORTED_MAP, I32, 4, 8, max_entries=4, bgs=[100])
    recs = [(1, np.arange(6, dtype=np.int32), np.ones(6, np.int32))]
    d = torch.from_numpy(wire.sparse_stream_np(3, 4, recs)).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 6


def test_more_than_64_records_for_one_row():
    """A row updated by 70 records inside one call (ordered by insertion sort path)."""
    rng = np.random.RandomState(2)
    srv, orc = _pair(SORTED_MAP, I32, 8, 32)
    recs = []
    for k in range(70):
        cols = np.sort(rng.choice(32, size=3, replace=False)).astype(np.int32)
        recs.append((5, cols, rng.choice([-2, -1, 1, 2, 3], size=3).astype(np.int32)))
    recs.append((6, np.array([1], np.int32), np.array([1], np.int32)))
    _apply(srv, orc, [wire.sparse_stream_np(3, 4, recs)], [100])
    assert srv.serialize_rows(3, [5, 6]) == orc.serialize_records(3, [5, 6])


def test_mixed_dense_and_sparse_tables_in_one_message():
    """Two tables in every message (ascending table id, oplog_serializer.hpp:12-37): a
    fast-path dense table and a sorted-map table, applied in one fused call."""
    rng = np.random.RandomState(17)
    rows, cap, K, B = 300, 32, 40, 4
    bgs = list(range(100, 100 + B))
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=I32, row_capacity=K,
                                     oplog_dense_serialized=False, max_rows=rows, max_entries=K))
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, cap)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    streams = []
    for b in range(B):
        ids1 = rng.permutation(rows)[:200].astype(np.int32)
        ids3 = rng.permutation(rows)[:100].astype(np.int32)
        cnt = np.zeros((100, K), np.int32)
        for r in range(100):
            c = rng.choice(K, size=rng.randint(1, 8), replace=False)
            cnt[r, c] = rng.choice([-1, 1, 2], size=c.size)
        streams.append(np.frombuffer(pack_stream([
            dict(table_id=3, dtype=I32, dense_serialized=False, row_ids=ids3, oplogs=cnt),
            dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=ids1,
                 oplogs=rng.normal(size=(200, cap)).astype(np.float32))]), np.uint8))
    _apply(srv, orc, streams, bgs)
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))
    assert srv.serialize_rows(3, list(range(rows))) == orc.serialize_records(3, list(range(rows)))


def test_duplicate_dense_rows_replayed_in_order():
    """A dense row twice in one message (not produced by the reference packer, but legal
    for Server::ApplyOpLogUpdateVersion): the fused path defers and the ordered replay
    applies it in stream order, bit-exact, including the calls after it."""
    rng = np.random.RandomState(4)
    rows, cap = 50, 40
    bgs = [100, 101, 102]
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, cap)
    s0 = wire.dense_stream_np(1, rng.permutation(rows).astype(np.int32), rng.normal(size=(rows, cap)).astype(np.float32))
    ids = np.array([3, 4, 3, 9, 3], np.int32)
    s1 = wire.dense_stream_np(1, ids, rng.normal(size=(5, cap)).astype(np.float32))
    s2 = wire.dense_stream_np(1, rng.permutation(rows).astype(np.int32), rng.normal(size=(rows, cap)).astype(np.float32))
    dev = [torch.from_numpy(s).cuda() for s in (s0, s1, s2)]
    torch.cuda.synchronize()
    for d, bg in zip(dev, bgs):          # three separate calls; the middle one has duplicates
        srv.apply_device([(d.data_ptr(), d.numel(), bg, 0)])
    srv.sync()
    for s, bg in zip((s0, s1, s2), bgs):
        assert orc.apply_stream(s, bg, 0) == 0
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))


@pytest.mark.parametrize("decode", [1, 0], ids=["walk", "block"])
def test_c3_lda_config_parity(decode):
    """SURVEY §8(d) C3 at full size: 100K SortedVectorMapRow<int32> rows, K = 1024, 8
    batches of 10K distinct Zipf-chosen rows, nnz uniform [1, 32], values +-{1..3}
    (first batch positive).  Every touched row's bytes match the oracle, through the
    window-parallel decode (the default) and through decode_streams."""
    L = _abi.load()
    old = L.psx_debug_set_variant(7, decode)
    L.psx_debug_set_variant(8, 0)
    try:
        _c3_full(walk_expected=decode == 1)
    finally:
        L.psx_debug_set_variant(7, old)


def _c3_full(walk_expected):
    L = _abi.load()
    rng = np.random.RandomState(1234)
    rows, K, B = 100_000, 1024, 8
    bgs = list(range(100, 100 + B))
    srv, orc = _pair(SORTED_MAP, I32, rows, K, bgs=bgs)
    p = 1.0 / np.arange(1, rows + 1)
    p /= p.sum()
    streams = []
    touched = set()
    for b in range(B):
        ids = rng.choice(rows, size=10_000, replace=False, p=p)
        recs = []
        for rid in ids:
            k = rng.randint(1, 33)
            cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
            sign = 1 if b == 0 else rng.choice([-1, 1], size=k)
            recs.append((int(rid), cols, (rng.randint(1, 4, size=k) * sign).astype(np.int32)))
        touched.update(int(x) for x in ids)
        streams.append(wire.sparse_stream_np(3, 4, recs))
    _apply(srv, orc, streams, bgs)
    assert (L.psx_debug_get_variant(8) > 0) == walk_expected
    ids = sorted(touched)
    assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids)
    srv.close()


@pytest.mark.parametrize("dt", [I32, F64])
def test_sorted_map_wide_rows_lds_path(dt):
    """max_entries > 1024 takes the LDS row-image kernel instead of the register one."""
    rng = np.random.RandomState(23)
    rows, K = 200, 3000
    srv, orc = _pair(SORTED_MAP, dt, rows, K, max_entries=2048)
    streams = [wire.sparse_stream_np(3, VS[dt], _sparse_rows(rng, rows, 1500, 120, dt, max_nnz=300))
               for _ in range(4)]
    _apply(srv, orc, streams, [100, 101, 102, 103])
    assert srv.serialize_rows(3, list(range(rows))) == orc.serialize_records(3, list(range(rows)))


def test_serve_back_push_body_matches_oracle():
    """Serve-back of every dirty row of three tables (dense, sorted map, map) in the push
    format of Server::CreateSendServerPushRowMsgs (server.cpp:189-309), then the dirty
    bits are cleared (second body is empty tables only)."""
    rng = np.random.RandomState(31)
    rows, cap, K = 200, 20, 40
    bgs = [100, 101]
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=I32, row_capacity=K,
                                     oplog_dense_serialized=False, max_rows=rows, max_entries=K))
    srv.CreateTable(4, psa.TableInfo(row_kind=psa.ROW_MAP, dtype=F64, row_capacity=K,
                                     oplog_dense_serialized=False, max_rows=rows, max_entries=K))
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, cap)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    orc.create_table(4, MAP, F64, 0, oplog_dense_serialized=False)
    init = rng.normal(size=(rows, cap)).astype(np.float32)
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams = []
    for b in range(2):
        d_ids = rng.permutation(rows)[:60].astype(np.int32)
        cnt = np.zeros((50, K), np.int32)
        mp_ = np.zeros((30, K), np.float64)
        for r in range(50):
            c = rng.choice(K, size=rng.randint(1, 6), replace=False)
            cnt[r, c] = rng.choice([-1, 1, 2], size=c.size)
        for r in range(30):
            c = rng.choice(K, size=rng.randint(1, 6), replace=False)
            mp_[r, c] = rng.normal(size=c.size)
        streams.append(np.frombuffer(pack_stream([
            dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=d_ids,
                 oplogs=rng.normal(size=(60, cap)).astype(np.float32)),
            dict(table_id=3, dtype=I32, dense_serialized=False,
                 row_ids=rng.permutation(rows)[:50].astype(np.int32), oplogs=cnt),
            dict(table_id=4, dtype=F64, dense_serialized=False,
                 row_ids=rng.permutation(rows)[:30].astype(np.int32), oplogs=mp_)]), np.uint8))
    _apply(srv, orc, streams, bgs)
    got = srv.serialize_dirty().tobytes()
    want = orc.serialize_dirty([1, 3, 4])
    gp, wp = wire.parse_push_body(got), wire.parse_push_body(want)
    assert gp.keys() == wp.keys() == {1, 3, 4}
    assert gp[1] == wp[1] and gp[3] == wp[3]                  # dense + sorted map: byte-exact
    assert gp[4].keys() == wp[4].keys()
    for r in gp[4]:
        assert _as_map(gp[4][r], F64, True) == _as_map(wp[4][r], F64, True)
    assert len(got) == len(want) and got[:4] == want[:4]
    empty = srv.serialize_dirty()
    assert empty.tobytes() == orc.serialize_dirty([1, 3, 4]) == np.array([1, -1, 3, -1, 4, -2], np.int32).tobytes()
