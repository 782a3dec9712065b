"""GPU parity of the importance-accumulating apply and the partial push (SSPAggr).

Under SSPAggr with a RelativeMagnitude / FIFO_N_ReMag policy ServerTable applies through
ApplyRow{Dense,}BatchIncAccumImportance (server_table.cpp:26-47): every record adds its
NSSumImpCalc importance (ns_sum_imp_calc.hpp:57-98) to ServerRow::importance_
(server_row.hpp:43-62,124-126), and the partial push sends the most important dirty rows
first (server_table.cpp:272-346, server.cpp:311-420).

Tolerances: row values bit-exact (the add order is the reference's).  Importance is an
f64 sum of non-negative terms; the device reassociates the sum (lane-parallel within a
record; the vectorised kernel also across the records of one call) and builds f32
quotients from an f32 reciprocal plus an exact f64 remainder step (rel < 2^-45 per
term), so it is within (cap*B)*2^-53 + 2^-45 relative of the reference's
element-by-element sum; the tests allow rel 1e-12 (cap*B <= 2700 here).  Partial push bodies are compared byte-for-byte (the data keeps
row importances far apart relative to that tolerance, so the send order is the same)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire
from oracle.oracle import OracleServer, DENSE, SORTED_MAP, MAP, F32, F64, I32, I64

pytestmark = pytest.mark.gpu
NP = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64}
VS = {F32: 4, F64: 8, I32: 4, I64: 8}
IMP_RTOL = 1e-12


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _dense_pair(dt, rows, cap, bgs, upper=0, importance=True, tid=1):
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(tid, psa.TableInfo(row_kind=DENSE, dtype=dt, row_capacity=cap, max_rows=rows,
                                       accum_importance=importance, server_push_row_upper_bound=upper))
    orc = OracleServer(list(bgs))
    orc.create_table(tid, DENSE, dt, cap, accum_importance=importance)
    return srv, orc


def _vals(rng, shape, dt, zero_frac=0.0):
    if dt in (I32, I64):
        v = rng.randint(-50, 51, size=shape)
    else:
        v = rng.normal(0, 1, size=shape)
    if zero_frac:
        v = np.where(rng.rand(*shape) < zero_frac, 0, v)
    return v.astype(NP[dt])


def _apply_dev(srv, orc, streams, bgs, vers=None):
    vers = vers or [0] * len(streams)
    dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg, v in zip(dev, bgs, vers)])
    srv.sync()
    for s, bg, v in zip(streams, bgs, vers):
        assert orc.apply_stream(s, bg, v) == 0


def _check_importance(srv, orc, tid, rows):
    got = srv.row_importance(tid, 0, rows)
    want = np.array([orc.importance(tid, r) for r in range(rows)])
    np.testing.assert_allclose(got, want, rtol=IMP_RTOL, atol=0)
    return got


@pytest.mark.parametrize("dt", [F32, F64, I32, I64])
@pytest.mark.parametrize("B", [1, 2, 3, 5, 9])
def test_dense_importance_matches_oracle(dt, B, built_lib):
    """The vectorised importance kernel (dense_apply_v2 with IMP)."""
    _dense_importance_case(dt, B)


def _dense_importance_case(dt, B):
    rng = np.random.RandomState(10 * B + dt)
    rows, cap = 2048, 300                      # cap not a multiple of 256: tail chunk
    bgs = list(range(100, 100 + B))
    srv, orc = _dense_pair(dt, rows, cap, bgs)
    init = _vals(rng, (rows, cap), dt, zero_frac=0.3)   # zeros take the |u| branch
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams = []
    for b in range(B):
        ids = rng.choice(rows, size=rows // 2 + 37 * b, replace=False).astype(np.int32)
        streams.append(wire.dense_stream_np(1, ids, _vals(rng, (ids.size, cap), dt, zero_frac=0.1)))
    _apply_dev(srv, orc, streams, bgs)
    got = srv.read_rows(1, 0, rows)
    assert np.array_equal(got.view(np.uint8), orc.read_dense_rows(1, 0, rows).view(np.uint8))
    imp = _check_importance(srv, orc, 1, rows)
    assert (imp > 0).sum() >= rows // 2


def test_dense_importance_special_values():
    """Zeros, signed zeros, denormals, huge/tiny quotients, inf and NaN in the old
    values and the updates (the f32 fast quotient falls back to the exact division
    outside the normal range)."""
    specials = np.array([0.0, -0.0, 1e-45, -3e-39, 1.2e-38, 1.0, -2.5, 3e38, -3.4e38, np.inf, -np.inf, np.nan,
                         7e-20, 6e19, 1e-30, 123456.7], np.float32)
    n = specials.size
    rows, cap = n, n
    init = np.stack([np.roll(specials, k) for k in range(rows)])
    upd = np.stack([np.roll(specials[::-1], 3 * k) for k in range(rows)])
    srv, orc = _dense_pair(F32, rows, cap, [1])
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    st = wire.dense_stream_np(1, np.arange(rows, dtype=np.int32), upd)
    _apply_dev(srv, orc, [st], [1])
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint8), orc.read_dense_rows(1, 0, rows).view(np.uint8))
    got = srv.row_importance(1, 0, rows)
    want = np.array([orc.importance(1, r) for r in range(rows)])
    np.testing.assert_allclose(got, want, rtol=IMP_RTOL, atol=0, equal_nan=True)


def test_dense_importance_accumulates_across_calls_and_host_path():
    rng = np.random.RandomState(5)
    rows, cap = 512, 64
    srv, orc = _dense_pair(F32, rows, cap, [7])
    for v in range(3):
        ids = rng.choice(rows, size=200, replace=False).astype(np.int32)
        st = wire.dense_stream_np(1, ids, _vals(rng, (200, cap), F32))
        srv.ApplyOpLogUpdateVersion(st, st.size, 7, v)          # host bytes
        assert orc.apply_stream(st, 7, v) == 0
    _check_importance(srv, orc, 1, rows)


def test_duplicate_row_replay_keeps_importance():
    """A row twice in one message goes through the ordered replay; importance follows
    the record order there too."""
    rng = np.random.RandomState(9)
    rows, cap = 256, 40
    bgs = [1, 2]
    srv, orc = _dense_pair(F32, rows, cap, bgs)
    init = _vals(rng, (rows, cap), F32, zero_frac=0.2)
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    ids0 = np.array([3, 9, 3, 100, 9, 3], np.int32)
    ids1 = rng.choice(rows, size=50, replace=False).astype(np.int32)
    streams = [wire.dense_stream_np(1, ids0, _vals(rng, (ids0.size, cap), F32)),
               wire.dense_stream_np(1, ids1, _vals(rng, (ids1.size, cap), F32))]
    _apply_dev(srv, orc, streams, bgs)
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint8), orc.read_dense_rows(1, 0, rows).view(np.uint8))
    _check_importance(srv, orc, 1, rows)


@pytest.mark.parametrize("kind", [SORTED_MAP, MAP, DENSE])
@pytest.mark.parametrize("dt", [I32, F32])
def test_sparse_importance_matches_oracle(kind, dt):
    rng = np.random.RandomState(31 + kind + dt)
    rows, K, B = 1500, 80, 4
    bgs = list(range(200, 200 + B))
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=dt, row_capacity=K, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=K, accum_importance=True))
    orc = OracleServer(bgs)
    orc.create_table(3, kind, dt, K if kind == DENSE else 0, oplog_dense_serialized=False, accum_importance=True)
    streams = []
    for b in range(B):
        recs = []
        for rid in rng.choice(rows, size=300, replace=False):
            k = rng.randint(1, 20)
            cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
            recs.append((int(rid), cols, _vals(rng, (k,), dt)))
        streams.append(wire.sparse_stream_np(3, VS[dt], recs))
    _apply_dev(srv, orc, streams, bgs)
    _check_importance(srv, orc, 3, rows)


def test_tables_without_importance_read_zero():
    srv, orc = _dense_pair(F32, 64, 8, [1], importance=False)
    st = wire.dense_stream_np(1, np.arange(10, dtype=np.int32), np.ones((10, 8), np.float32))
    _apply_dev(srv, orc, [st], [1])
    assert not srv.row_importance(1, 0, 64).any()


def _two_table_pair(bgs, ub_dense, ub_sparse, rows=3000):
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=48, max_rows=rows,
                                     accum_importance=True, server_push_row_upper_bound=ub_dense))
    srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=64, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=64, server_push_row_upper_bound=ub_sparse))
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, 48, accum_importance=True)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    return srv, orc


def _round(rng, rows):
    """One two-table message: dense records for 900 rows, sparse records for 700."""
    d_ids = rng.choice(rows, size=900, replace=False).astype(np.int32)
    s_ids = rng.choice(rows, size=700, replace=False).astype(np.int32)
    counts = np.zeros((700, 64), np.int32)
    for i in range(700):
        k = rng.randint(1, 12)
        counts[i, rng.choice(64, size=k, replace=False)] = rng.randint(1, 4, size=k)
    return wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=d_ids, oplogs=_vals(rng, (900, 48), F32)),
                         dict(table_id=3, dense_serialized=False, row_ids=s_ids, oplogs=counts)])


def test_partial_push_matches_oracle():
    """Importance-ordered partial push over several clocks: the body (send order and
    row bytes), the dirty bits and the importance reset of the sent rows all match."""
    rng = np.random.RandomState(77)
    rows = 3000
    bgs = [10]
    srv, orc = _two_table_pair(bgs, ub_dense=250, ub_sparse=300, rows=rows)
    for clock in range(3):
        _apply_dev(srv, orc, [_round(rng, rows)], bgs, vers=[clock])
        for _ in range(2):        # two partial pushes per clock: the second sends the next rows
            got = bytes(srv.serialize_partial())
            want = orc.serialize_partial([1, 3], [250, 300])
            assert got == want
        _check_importance(srv, orc, 1, rows)
        flags = srv.row_flags(1, 0, rows)
        assert [bool(f & 2) for f in flags] == [orc.row_dirty(1, r) for r in range(rows)]
    # drain everything, then nothing is left to send
    while orc.serialize_partial([1, 3], [250, 300]):
        assert len(srv.serialize_partial()) > 0
    assert len(srv.serialize_partial()) == 0
    assert not srv.row_importance(1, 0, rows).any()


def test_partial_push_parses_and_orders_by_importance():
    rng = np.random.RandomState(3)
    rows = 1000
    srv = psa.Server(0, 1, [1])
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=16, max_rows=rows,
                                     accum_importance=True, server_push_row_upper_bound=40))
    srv.load_rows(1, 0, _vals(rng, (rows, 16), F32))
    ids = rng.choice(rows, size=500, replace=False).astype(np.int32)
    st = torch.from_numpy(wire.dense_stream_np(1, ids, _vals(rng, (500, 16), F32))).cuda()
    srv.apply_device([(st.data_ptr(), st.numel(), 1, 0)])
    srv.sync()
    imp = srv.row_importance(1, 0, rows)
    body = bytes(srv.serialize_partial(clear=False))
    sent = list(wire.parse_push_body(body)[1].keys())
    order = sorted(ids.tolist(), key=lambda r: (-imp[r], r))[:40]
    assert sent == order
    # clear=False left every row dirty with its importance
    assert np.array_equal(srv.row_importance(1, 0, rows), imp)


def test_full_push_resets_importance():
    rng = np.random.RandomState(4)
    rows = 400
    srv, orc = _dense_pair(F32, rows, 12, [1])
    ids = rng.choice(rows, size=100, replace=False).astype(np.int32)
    st = wire.dense_stream_np(1, ids, _vals(rng, (100, 12), F32))
    _apply_dev(srv, orc, [st], [1])
    assert bytes(srv.serialize_dirty()) == orc.serialize_dirty([1])
    assert not srv.row_importance(1, 0, rows).any()
    assert orc.importance(1, int(ids[0])) == 0.0
