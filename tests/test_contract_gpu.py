"""Error contract of the C ABI on the GPU: a call that fails applies nothing, and every
accepted message is applied exactly once before anything observes or serves the table.

Covers the cases a review found: two fast dense tables where only one
has a duplicate row, a push built while a duplicate-row replay is pending, an AdaRevision
push that runs out of snapshot slots, binary16 records of one element on the ordered
replay, and the all-or-nothing forms of PSX_ERR_CAPACITY and PSX_ERR_STATE.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError
from oracle.oracle import OracleServer, DENSE, SORTED_MAP, MAP, F32, I32, pack_stream

pytestmark = pytest.mark.gpu

CAPACITY, STATE = 6, 13


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _dev(streams):
    d = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
    torch.cuda.synchronize()
    return d


def _u32(a):
    return np.ascontiguousarray(a).view(np.uint32)


def test_two_dense_tables_duplicate_in_one_applied_once():
    """Table 2 repeats a row inside message 1; table 1 is clean.  The call is replayed on
    the ordered path and both tables end bit-exact with the sequential reference — the
    clean table is not applied twice (the gate stops every fast table of the call)."""
    rng = np.random.RandomState(11)
    rows, cap, B = 120, 48, 3
    bgs = [100, 101, 102]
    srv = psa.Server(0, 1, bgs)
    orc = OracleServer(bgs)
    for tid in (1, 2):
        srv.CreateTable(tid, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
        orc.create_table(tid, DENSE, F32, cap)
    streams = []
    for b in range(B):
        ids1 = rng.permutation(rows)[:80].astype(np.int32)
        ids2 = rng.permutation(rows)[:60].astype(np.int32)
        if b == 1:
            ids2[5] = ids2[17]            # a duplicate row in table 2 only
        streams.append(np.frombuffer(pack_stream([
            dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=ids1,
                 oplogs=rng.normal(size=(80, cap)).astype(np.float32)),
            dict(table_id=2, dtype=F32, dense_serialized=True, row_ids=ids2,
                 oplogs=rng.normal(size=(60, cap)).astype(np.float32))]), np.uint8))
    dev = _dev(streams)
    srv.apply_device([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dev, bgs)])
    srv.sync()
    for s, bg in zip(streams, bgs):
        assert orc.apply_stream(s, bg, 0) == 0
    for tid in (1, 2):
        assert np.array_equal(_u32(srv.read_rows(tid, 0, rows)), _u32(orc.read_dense_rows(tid, 0, rows)))


def test_push_settles_a_pending_replay():
    """psx_serialize_dirty right after a call whose message repeats a row (no psx_sync in
    between): the push holds every accepted update (server_thread.cpp applies each
    message before any push)."""
    rng = np.random.RandomState(12)
    rows, cap = 40, 16
    srv = psa.Server(0, 1, [100, 101])
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    orc = OracleServer([100, 101])
    orc.create_table(1, DENSE, F32, cap)
    s0 = wire.dense_stream_np(1, np.array([3, 7, 3, 9], np.int32), rng.normal(size=(4, cap)).astype(np.float32))
    s1 = wire.dense_stream_np(1, np.array([7, 1], np.int32), rng.normal(size=(2, cap)).astype(np.float32))
    dev = _dev([s0, s1])
    srv.apply_device([(dev[0].data_ptr(), dev[0].numel(), 100, 0)])
    srv.apply_device([(dev[1].data_ptr(), dev[1].numel(), 101, 0)])
    got = bytes(srv.serialize_dirty(clear=True))
    assert orc.apply_stream(s0, 100, 0) == 0 and orc.apply_stream(s1, 101, 0) == 0
    assert got == orc.serialize_dirty([1], clear=True)


def test_adarevision_push_without_snapshot_slot_changes_nothing():
    """max_snapshots_per_row = 1 and a second push of a row under a new version while the
    first snapshot is live: PSX_ERR_CAPACITY before anything is cleared — the rows stay
    dirty, no snapshot is added, and a later push (after the client releases the first
    version) succeeds."""
    rows, cap = 20, 8
    srv = psa.Server(0, 1, [1])
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=cap, max_rows=rows,
                                     version_maintain=True))
    srv.set_adarevision(1, init_step_size=0.1, gaussian_init=False, push_clients=1, max_snapshots_per_row=1)
    ids = np.array([2, 5], np.int32)
    one = np.ones((2, cap), np.float32)
    s0 = wire.dense_variant_stream_np(1, ids, one, versions=[0, 0])
    d0 = _dev([s0])[0]
    srv.apply_device([(d0.data_ptr(), d0.numel(), 1, 0)])
    first = bytes(srv.serialize_dirty(clear=True))          # snapshot (row, version 2)
    assert len(first) > 8
    assert srv.adarevision_state(1, 0, rows)[3] == 2
    s1 = wire.dense_variant_stream_np(1, ids, one, versions=[0, 0])   # version 0: no snapshot needed
    d1 = _dev([s1])[0]
    srv.apply_device([(d1.data_ptr(), d1.numel(), 1, 1)])
    srv.sync()
    flags_before = srv.row_flags(1, 0, rows).copy()
    with pytest.raises(PsxError) as e:
        srv.serialize_dirty(clear=True)                    # needs (row, 3): no free slot
    assert e.value.status == CAPACITY
    assert np.array_equal(srv.row_flags(1, 0, rows), flags_before)
    assert srv.adarevision_state(1, 0, rows)[3] == 2
    # the client finishes version 2: end_of_version releases the snapshot
    s2 = wire.dense_variant_stream_np(1, ids, one, versions=[2, 2], end_of_version=[True, True])
    d2 = _dev([s2])[0]
    srv.apply_device([(d2.data_ptr(), d2.numel(), 1, 2)])
    srv.sync()
    assert srv.adarevision_state(1, 0, rows)[3] == 0
    assert len(bytes(srv.serialize_dirty(clear=True))) > 8
    assert srv.adarevision_state(1, 0, rows)[3] == 2


def test_float16_one_element_records_on_the_replay():
    """binary16 records of dense_row_oplog_capacity 1 are 6 bytes: the ordered replay of
    a message with a repeated row sizes its record lists for them."""
    rng = np.random.RandomState(13)
    rows, n = 64, 3000
    srv = psa.Server(0, 1, [100])
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=4,
                                     dense_row_oplog_capacity=1, max_rows=rows, row_oplog_type=3))
    orc = OracleServer([100])
    orc.create_table(1, DENSE, F32, 4, dense_row_oplog_capacity=1, f16_records=True)
    ids = rng.randint(0, rows, size=n).astype(np.int32)       # many repeats
    h = rng.normal(0, 1, size=(n, 1)).astype(np.float16)
    s = wire.dense_variant_stream_np(1, ids, h, f16=True)
    d = _dev([s])[0]
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    srv.sync()
    assert orc.apply_stream(s, 100, 0) == 0
    assert np.array_equal(_u32(srv.read_rows(1, 0, rows)), _u32(orc.read_dense_rows(1, 0, rows)))


def _sorted_pair(max_entries, bgs):
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=I32, row_capacity=8,
                                     oplog_dense_serialized=False, max_rows=16, max_entries=max_entries))
    orc = OracleServer(bgs)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    return srv, orc


def test_capacity_overflow_applies_nothing():
    """A sorted-map row would exceed max_entries in message 1 of a 2-message call: the
    capacity dry run fails the whole call (PSX_ERR_CAPACITY) and message 0's rows are
    untouched too."""
    srv, _ = _sorted_pair(4, [100, 101])
    base = wire.sparse_stream_np(3, 4, [(1, np.array([10, 11, 12], np.int32), np.array([5, 4, 3], np.int32))])
    d = _dev([base])[0]
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    srv.sync()
    before = srv.serialize_rows(3, list(range(16)))
    m0 = wire.sparse_stream_np(3, 4, [(2, np.array([1], np.int32), np.array([7], np.int32))])
    m1 = wire.sparse_stream_np(3, 4, [(1, np.array([20, 21], np.int32), np.array([1, 1], np.int32))])
    dv = _dev([m0, m1])
    srv.apply_device([(dv[0].data_ptr(), dv[0].numel(), 100, 1), (dv[1].data_ptr(), dv[1].numel(), 101, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == CAPACITY
    assert srv.serialize_rows(3, list(range(16))) == before
    assert not (srv.row_flags(3, 0, 16)[2] & 1)


def test_capacity_dry_run_passes_when_removals_make_room():
    """The dry run simulates the reference order exactly: a record that first zeroes an
    entry and then adds a new key fits a full row, and is applied byte-exact."""
    srv, orc = _sorted_pair(3, [100])
    recs = [(1, np.array([10, 11, 12], np.int32), np.array([5, 4, 3], np.int32)),
            (1, np.array([11, 30], np.int32), np.array([-4, 9], np.int32))]
    s = wire.sparse_stream_np(3, 4, recs)
    d = _dev([s])[0]
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    srv.sync()
    assert orc.apply_stream(s, 100, 0) == 0
    assert srv.serialize_rows(3, [1]) == orc.serialize_records(3, [1])


def test_state_error_applies_nothing():
    """An AdaRevision record naming a (row, version) without a snapshot fails the call
    before any table is touched — including the other dense table of the same message."""
    rows, cap = 30, 8
    srv = psa.Server(0, 1, [1])
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=cap, max_rows=rows,
                                     version_maintain=True))
    srv.CreateTable(2, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    srv.set_adarevision(1, init_step_size=0.1, gaussian_init=False, push_clients=1)
    t1 = wire.dense_variant_stream_np(1, np.array([4, 6], np.int32), np.ones((2, cap), np.float32),
                                      versions=[0, 9])      # version 9 was never sent
    t2 = wire.dense_stream_np(2, np.array([1, 2], np.int32), np.ones((2, cap), np.float32))
    msg = np.concatenate([np.array([2], np.int32).view(np.uint8), t1[4:], t2[4:]])
    d = _dev([msg])[0]
    srv.apply_device([(d.data_ptr(), d.numel(), 1, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == STATE
    assert not srv.read_rows(1, 0, rows).any() and not srv.read_rows(2, 0, rows).any()
    assert not (srv.row_flags(1, 0, rows) & 1).any() and not (srv.row_flags(2, 0, rows) & 1).any()
