"""The window-parallel walk doing ordered_count's work for split sorted/map tables
(PSX_VARIANT_WALK_COUNT, WalkCount in psx_device.hpp): on walked calls the walk adds each
record to the call slot's cnt/grow as it writes the record's offset and the ordered prep
launches no ordered_count.  Every form — walk-counted, ordered_count, and walk-counted with
the decode pipelined beside the previous call's ordered work — with and without the walk
also placing each record in its slot's list (WalkCount.wfill) — must give the oracle's rows byte for byte
(SortedVectorMapStore, sorted_vector_map_store.hpp:175-197,305-337) over several calls, and a
call that names a row outside the shard must fail with nothing applied and leave the counts
clean for the next call (the reference rejects such a row: server_table.hpp FindRow/CreateRow
on an unowned id)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError, _abi
from oracle.oracle import OracleServer, SORTED_MAP, MAP, I32

pytestmark = pytest.mark.gpu
DECODE, WALK_CALLS, ORD_SPLIT, WALK_COUNT = 7, 8, 6, 13
PIPELINE_ALL = 2


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


WALK_RANK = 20


@pytest.fixture(autouse=True, params=[1, 0], ids=["walk-ranked", "fill-counted"])
def walk_rank(request, _gpu):
    """Every test with the walk also giving each record its list place (ordered_fill without
    atomics, PSX_VARIANT_WALK_RANK 1, the default) and without (ordered_fill takes the places
    back from the counts)."""
    L = _abi.load()
    old = L.psx_debug_set_variant(WALK_RANK, request.param)
    yield request.param
    L.psx_debug_set_variant(WALK_RANK, old)


def _batches(rng, rows, K, calls, per_batch=6_000, B=4):
    p = 1.0 / np.arange(1, rows + 1)
    p /= p.sum()
    out = []
    for c in range(calls):
        msgs = []
        for b in range(B):
            ids = rng.choice(rows, size=per_batch, replace=False, p=p)
            recs = []
            for rid in ids:
                k = int(rng.randint(1, 33))
                cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
                v = (rng.randint(1, 4, size=k) * rng.choice([-1, 1], size=k)).astype(np.int32)
                if c == 0:
                    v = np.abs(v)
                recs.append((int(rid), cols, v))
            msgs.append(wire.sparse_stream_np(3, 4, recs))
        out.append(msgs)
    return out


def _run(kind, calls, rows, K, walk_count, pipeline, split):
    L = _abi.load()
    old = [L.psx_debug_set_variant(WALK_COUNT, walk_count), L.psx_debug_set_variant(ORD_SPLIT, split),
           L.psx_debug_set_variant(DECODE, 1)]
    try:
        bgs = [100, 101, 102, 103]
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(pipeline)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        L.psx_debug_set_variant(WALK_CALLS, 0)
        snaps = []
        for v, msgs in enumerate(calls):
            dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs]
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
            srv.sync()
            snaps.append(srv.serialize_rows(3, list(range(rows))))
        walked = L.psx_debug_get_variant(WALK_CALLS)
        srv.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old[0])
        L.psx_debug_set_variant(ORD_SPLIT, old[1])
        L.psx_debug_set_variant(DECODE, old[2])
    assert walked == len(calls)
    return snaps


@pytest.mark.parametrize("walk_count,pipeline", [(1, 0), (0, 0), (1, PIPELINE_ALL), (0, PIPELINE_ALL)],
                         ids=["walk-counted", "ordered_count", "pipelined-walk-counted", "pipelined-ordered_count"])
@pytest.mark.parametrize("split", [3, 1], ids=["spill-heavy-first", "concurrent"])
def test_split_tables_counted_by_the_walk(walk_count, pipeline, split):
    rng = np.random.RandomState(31)
    rows, K = 12_000, 1024
    calls = _batches(rng, rows, K, 3)
    snaps = _run(SORTED_MAP, calls, rows, K, walk_count, pipeline, split)
    orc = OracleServer([100, 101, 102, 103])
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate(calls):
        for s, bg in zip(msgs, [100, 101, 102, 103]):
            assert orc.apply_stream(s, bg, v) == 0
        assert snaps[v] == orc.serialize_records(3, list(range(rows))), f"call {v}"
    orc.close()


def test_map_table_walk_counted_matches_ordered_count():
    rng = np.random.RandomState(32)
    rows, K = 8_000, 512
    calls = _batches(rng, rows, K, 2, per_batch=4_000)
    a = _run(MAP, calls, rows, K, 1, 0, 3)
    b = _run(MAP, calls, rows, K, 0, 0, 3)
    assert a == b


@pytest.mark.parametrize("walk_count", [1, 0], ids=["walk-counted", "ordered_count"])
def test_row_outside_the_shard_fails_and_leaves_counts_clean(walk_count):
    """A call with one record naming a row past the shard: PSX_ERR_ROW_RANGE, nothing of the
    call applied; the next call (valid) must equal the oracle, so no count of the failed call
    may survive it."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(WALK_COUNT, walk_count), L.psx_debug_set_variant(DECODE, 1)]
    rng = np.random.RandomState(33)
    rows, K = 6_000, 1024
    good = _batches(rng, rows, K, 2, per_batch=3_000, B=2)
    bad = [list(m) for m in _batches(rng, rows, K, 1, per_batch=3_000, B=2)][0]
    # the second message of the bad call: its records plus one for row `rows` (outside)
    recs = [(5, np.array([1, 2], np.int32), np.array([1, 1], np.int32)),
            (rows, np.array([3], np.int32), np.array([1], np.int32)),
            (7, np.array([4], np.int32), np.array([2], np.int32))]
    bad[1] = wire.sparse_stream_np(3, 4, recs)
    bgs = [100, 101]
    try:
        srv = psa.Server(0, 1, bgs)
        srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        orc = OracleServer(bgs)
        orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)

        def apply(msgs, v):
            dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs]
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
            srv.sync()

        apply(good[0], 0)
        for s, bg in zip(good[0], bgs):
            assert orc.apply_stream(s, bg, 0) == 0
        before = srv.serialize_rows(3, list(range(rows)))
        with pytest.raises(PsxError):
            apply(bad, 1)
        assert srv.serialize_rows(3, list(range(rows))) == before
        apply(good[1], 1)   # the failed call gave version 1 back
        for s, bg in zip(good[1], bgs):
            assert orc.apply_stream(s, bg, 1) == 0
        assert srv.serialize_rows(3, list(range(rows))) == orc.serialize_records(3, list(range(rows)))
        srv.close()
        orc.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old[0])
        L.psx_debug_set_variant(DECODE, old[1])


@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted_map", "map"])
@pytest.mark.parametrize("split", [3, 1], ids=["spill-heavy-first", "concurrent"])
def test_pipelined_walk_counts_without_sync_between_calls(kind, split):
    """Six walked calls enqueued back to back with PSX_PIPELINE_ALL and no sync between them
    (the device buffers all kept alive), so call k's walk counts into its slot while call
    k-1's ordered work still runs on the other slot's counts; the fourth call names a row
    outside the shard.  One sync at the end reports that call's error; every other call is
    applied, and the rows equal the oracle fed the five good calls byte for byte (sorted map:
    entry order; map: {col -> value})."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(WALK_COUNT, 1), L.psx_debug_set_variant(ORD_SPLIT, split),
           L.psx_debug_set_variant(DECODE, 1)]
    rng = np.random.RandomState(90 + split)
    rows, K, bgs = 8_000, 1024, [100, 101, 102, 103]
    calls = _batches(rng, rows, K, 6, per_batch=3_000)
    bad = 3
    recs = [(5, np.array([1, 2], np.int32), np.array([1, 1], np.int32)),
            (rows + 3, np.array([3], np.int32), np.array([1], np.int32)),
            (7, np.array([4], np.int32), np.array([2], np.int32))]
    calls[bad] = list(calls[bad])
    calls[bad][2] = wire.sparse_stream_np(3, 4, recs)
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(PIPELINE_ALL)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        L.psx_debug_set_variant(WALK_CALLS, 0)
        dev = [[torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs] for msgs in calls]
        torch.cuda.synchronize()
        for v, msgs in enumerate(dev):
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(msgs, bgs)])
        with pytest.raises(PsxError) as e:
            srv.sync()
        assert e.value.status == 5
        walked = L.psx_debug_get_variant(WALK_CALLS)
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old[0])
        L.psx_debug_set_variant(ORD_SPLIT, old[1])
        L.psx_debug_set_variant(DECODE, old[2])
    assert walked == len(calls)
    orc = OracleServer(bgs)
    orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
    ov = 0
    for v, msgs in enumerate(calls):
        if v == bad:
            continue
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, ov) == 0
        ov += 1
    want = orc.serialize_records(3, list(range(rows)))
    orc.close()
    if kind == SORTED_MAP:
        assert got == want
    else:
        assert _map_rows(got) == _map_rows(want)


def _map_rows(body):
    """{row: {col: value}} of RecordBuff records {int32 row; size_t size; Entry<int32>[n]}."""
    import struct
    out, off = {}, 0
    while off < len(body):
        rid, size = struct.unpack_from("<iQ", body, off)
        off += 12
        e = np.frombuffer(body[off:off + size], np.int32).reshape(-1, 2)
        out[rid] = dict(zip(e[:, 0].tolist(), e[:, 1].tolist()))
        off += size
    return out


FOLD_FINISH = 14


@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted_map", "map"])
def test_finish_folded_into_the_last_ordered_launch(kind):
    """PSX_VARIANT_FOLD_FINISH: a call ending in an ordered apply does finish_call's work in
    that launch's last block.  Rows after every call equal the unfolded run's, and a failing
    call's status still reaches psx_sync through the folded finish (the call fails, nothing
    of it applied, the next call is clean)."""
    L = _abi.load()
    rng = np.random.RandomState(71)
    rows, K = 5_000, 1024
    calls = _batches(rng, rows, K, 3, per_batch=2_000)
    old = L.psx_debug_set_variant(FOLD_FINISH, 0)
    try:
        a = _run(kind, calls, rows, K, 1, 0, 3)
        L.psx_debug_set_variant(FOLD_FINISH, 1)
        b = _run(kind, calls, rows, K, 1, 0, 3)
    finally:
        L.psx_debug_set_variant(FOLD_FINISH, old)
    assert a == b
    # the error path through the folded finish (the default)
    test_row_outside_the_shard_fails_and_leaves_counts_clean(1)


PREP_HALVES = 25


@pytest.mark.parametrize("halves", [1, 0], ids=["prep-halves", "prep-on-context-stream"])
@pytest.mark.parametrize("split", [3, 2, 1], ids=["spill-heavy-first", "spill", "concurrent"])
@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted_map", "map"])
def test_pipelined_prep_halves_back_to_back(halves, split, kind, walk_rank):
    """a pipelined call's split tables run the records' half of the ordered
    prep (ordered_place, ordered_fill: list ranges and record lists, into the call slot's own
    list region) on the prep stream beside the previous call's apply, and the rows' half
    (ordered_classify on the images that apply left, the dry run) on the context stream.
    Eight walked calls back to back with no sync between them, hot Zipf rows whose images
    cross 256 entries (spills, heavy and light rows), against the oracle byte for byte —
    and the same with the whole prep on the context stream (PSX_VARIANT_PREP_HALVES 0)."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(WALK_COUNT, 1), L.psx_debug_set_variant(ORD_SPLIT, split),
           L.psx_debug_set_variant(DECODE, 1), L.psx_debug_set_variant(PREP_HALVES, halves)]
    rng = np.random.RandomState(500 + split + 7 * halves)
    rows, K, bgs = 6_000, 1024, [100, 101, 102, 103]
    calls = _batches(rng, rows, K, 8, per_batch=2_500)
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(PIPELINE_ALL)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        dev = [[torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs] for msgs in calls]
        torch.cuda.synchronize()
        for v, msgs in enumerate(dev):
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(msgs, bgs)])
        srv.sync()
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old[0])
        L.psx_debug_set_variant(ORD_SPLIT, old[1])
        L.psx_debug_set_variant(DECODE, old[2])
        L.psx_debug_set_variant(PREP_HALVES, old[3])
    orc = OracleServer(bgs)
    orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate(calls):
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    want = orc.serialize_records(3, list(range(rows)))
    orc.close()
    if kind == SORTED_MAP:
        assert got == want
    else:
        assert _map_rows(got) == _map_rows(want)


CLASSIFY_DRY = 27


@pytest.mark.parametrize("pipeline", [PIPELINE_ALL, 0], ids=["pipelined", "walked"])
@pytest.mark.parametrize("classify_dry", [1, 0], ids=["classify-in-dry-run", "classify-launch"])
@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted_map", "map"])
def test_pipelined_capacity_overflow_applies_nothing(classify_dry, kind, pipeline, walk_rank):
    """The capacity dry run of a split table, with the classification as its prologue
    (PSX_VARIANT_CLASSIFY_DRY 1: a pipelined call's compact list, or an unpipelined call's
    slots with bucket lists; each block dry-runs the rows it filed as able to overflow) or as
    a launch of its own (0): a call that would take one row past
    max_entries (300) fails with PSX_ERR_CAPACITY and applies nothing, in any row; the
    call's version comes back, and the corrected call then equals the oracle byte for byte."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(WALK_COUNT, 1), L.psx_debug_set_variant(DECODE, 1),
           L.psx_debug_set_variant(CLASSIFY_DRY, classify_dry)]
    rng = np.random.RandomState(61 + classify_dry)
    rows, cap, bgs = 3000, 300, [100, 101]

    def msg(nrows, lo, hi, extra=None):
        recs = []
        for rid in rng.choice(rows, size=nrows, replace=False):
            if rid == 7:              # row 7's image is set by the calls themselves
                continue
            k = int(rng.randint(1, 20))
            cols = np.sort(rng.choice(np.arange(lo, hi), size=k, replace=False)).astype(np.int32)
            recs.append((int(rid), cols, rng.randint(1, 4, size=k).astype(np.int32)))
        if extra:
            recs.append(extra)
        return wire.sparse_stream_np(3, 4, recs)

    # call 0: row 7 holds 280 entries (keys 0..279); others a few
    first = [wire.sparse_stream_np(3, 4, [(7, np.arange(280, dtype=np.int32), np.ones(280, np.int32))]),
             msg(800, 0, 1000)]
    # call 1 (bad): row 7 gets 40 new keys -> 320 > 300
    bad = [msg(900, 0, 1000, (7, np.arange(1000, 1040, dtype=np.int32), np.ones(40, np.int32))), msg(900, 0, 1000)]
    good = [msg(900, 0, 1000, (7, np.arange(1000, 1010, dtype=np.int32), np.ones(10, np.int32))), msg(900, 0, 1000)]
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(pipeline)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=100_000, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=cap))
        keep = []

        def send(msgs, v):
            dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs]
            keep.append(dev)
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])

        send(first, 0)
        srv.sync()
        before = srv.serialize_rows(3, list(range(rows)))
        send(bad, 1)
        with pytest.raises(PsxError) as e:
            srv.sync()
        assert e.value.status == 6 and "version given back" in str(e.value)
        assert srv.serialize_rows(3, list(range(rows))) == before
        send(good, 1)
        srv.sync()
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old[0])
        L.psx_debug_set_variant(DECODE, old[1])
        L.psx_debug_set_variant(CLASSIFY_DRY, old[2])
    orc = OracleServer(bgs)
    orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate([first, good]):
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    want = orc.serialize_records(3, list(range(rows)))
    orc.close()
    if kind == SORTED_MAP:
        assert got == want
    else:
        assert _map_rows(got) == _map_rows(want)


@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted_map", "map"])
def test_pipelined_prep_halves_calls_of_different_sizes(kind, walk_rank):
    """The call slots' record-list regions must not overlap whatever each call's size: a
    large call, then small ones, back to back with no sync (a small call's lists are filled
    on the prep stream while the large call's apply still reads its own), then large again —
    byte for byte against the oracle (round 6: the regions sit at multiples of the allocated
    capacity, not of the current call's need)."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(WALK_COUNT, 1), L.psx_debug_set_variant(DECODE, 1)]
    rng = np.random.RandomState(808)
    rows, K, bgs = 8_000, 1024, [100, 101, 102, 103]
    sizes = [5_000, 200, 150, 4_000, 100, 3_000, 50, 5_000]
    calls = [_batches(rng, rows, K, 1, per_batch=z)[0] for z in sizes]
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(PIPELINE_ALL)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        dev = [[torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs] for msgs in calls]
        torch.cuda.synchronize()
        for v, msgs in enumerate(dev):
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(msgs, bgs)])
        srv.sync()
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old[0])
        L.psx_debug_set_variant(DECODE, old[1])
    orc = OracleServer(bgs)
    orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate(calls):
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    want = orc.serialize_records(3, list(range(rows)))
    orc.close()
    if kind == SORTED_MAP:
        assert got == want
    else:
        assert _map_rows(got) == _map_rows(want)


ORD_BUCKET = 30


PIPE_SLOTS = 31


@pytest.mark.parametrize("pipeline,pipe_slots", [(0, 0), (PIPELINE_ALL, 0), (PIPELINE_ALL, 1)],
                         ids=["walked", "pipelined", "pipelined-slots"])
@pytest.mark.parametrize("bucket", [1, 0], ids=["bucket-lists", "prefix-lists"])
@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted_map", "map"])
def test_bucket_lists_and_their_overflow_replay(bucket, pipeline, pipe_slots, kind, walk_rank):
    """Bucket record lists (PSX_VARIANT_ORD_BUCKET 1, the default with ranked counts): the
    walk writes each record's list entry at [slot][place] for places < 16, and the dry run's
    prologue classifies the slots (unpipelined calls, or PSX_VARIANT_PIPE_SLOTS 1).  Three calls: an
    ordinary one; one where row 5 has 20 records (a message repeating it: more than a
    bucket holds) — that call and the next, enqueued behind it, are replayed with prefix
    lists at the sync; then an ordinary one.  Byte for byte against the oracle, in both
    list forms, walked and pipelined."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(WALK_COUNT, 1), L.psx_debug_set_variant(DECODE, 1),
           L.psx_debug_set_variant(ORD_BUCKET, bucket), L.psx_debug_set_variant(PIPE_SLOTS, pipe_slots)]
    rng = np.random.RandomState(4242 + bucket)
    rows, K, bgs = 5_000, 1024, [100, 101, 102, 103]
    calls = _batches(rng, rows, K, 3, per_batch=1_500)
    recs = []
    for _ in range(20):      # row 5, 20 records in one message
        k = int(rng.randint(1, 30))
        cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
        recs.append((5, cols, (rng.randint(1, 4, size=k) * rng.choice([-1, 1], size=k)).astype(np.int32)))
    for rid in rng.choice(np.arange(6, rows), size=500, replace=False):
        cols = np.sort(rng.choice(K, size=8, replace=False)).astype(np.int32)
        recs.append((int(rid), cols, rng.randint(1, 4, size=8).astype(np.int32)))
    calls[1] = list(calls[1])
    calls[1][2] = wire.sparse_stream_np(3, 4, recs)
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(pipeline)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        dev = [[torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs] for msgs in calls]
        torch.cuda.synchronize()
        for v, msgs in enumerate(dev):
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(msgs, bgs)])
        srv.sync()
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old[0])
        L.psx_debug_set_variant(DECODE, old[1])
        L.psx_debug_set_variant(ORD_BUCKET, old[2])
        L.psx_debug_set_variant(PIPE_SLOTS, old[3])
    orc = OracleServer(bgs)
    orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate(calls):
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    want = orc.serialize_records(3, list(range(rows)))
    orc.close()
    if kind == SORTED_MAP:
        assert got == want
    else:
        assert _map_rows(got) == _map_rows(want)


SIDE_CU_MASK = 32


@pytest.mark.parametrize("mask", [2, 4, -2], ids=["prep-on-half", "prep-on-quarter", "disjoint-halves"])
def test_cu_masked_streams_leave_results_unchanged(mask, walk_rank):
    """PSX_VARIANT_SIDE_CU_MASK (read when the context is created): the prep stream — and with
    a negative value the context's own stream too — on CU-mask subsets, the pipelined walk
    sized to its CUs.  Six pipelined calls back to back against the oracle byte for byte."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(SIDE_CU_MASK, mask), L.psx_debug_set_variant(DECODE, 1)]
    rng = np.random.RandomState(700 + mask)
    rows, K, bgs = 6_000, 1024, [100, 101, 102, 103]
    calls = _batches(rng, rows, K, 6, per_batch=2_500)
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(PIPELINE_ALL)
        srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K,
                                         oplog_dense_serialized=False, max_rows=rows, max_entries=K))
        L.psx_debug_set_variant(WALK_CALLS, 0)
        dev = [[torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs] for msgs in calls]
        torch.cuda.synchronize()
        for v, msgs in enumerate(dev):
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(msgs, bgs)])
        srv.sync()
        walked = L.psx_debug_get_variant(WALK_CALLS)
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(SIDE_CU_MASK, old[0])
        L.psx_debug_set_variant(DECODE, old[1])
    assert walked == len(calls)
    orc = OracleServer(bgs)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate(calls):
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    assert got == orc.serialize_records(3, list(range(rows)))
    orc.close()


EVENT_SCOPE = 33


@pytest.mark.parametrize("scope", [2, 0], ids=["no-system-fence", "system-fence"])
def test_pipelined_many_calls_small_table(scope, walk_rank):
    """The call slots' cross-stream events (PSX_VARIANT_EVENT_SCOPE, read at context creation;
    2 the default: no system-scope fence): 24 pipelined calls back to back on a table small
    enough to stay in the XCDs' L2s, every call's records different, the slots' lists and
    counts reused every second call — the rows must equal the oracle's byte for byte."""
    L = _abi.load()
    old = [L.psx_debug_set_variant(EVENT_SCOPE, scope), L.psx_debug_set_variant(DECODE, 1)]
    rng = np.random.RandomState(800 + scope)
    rows, K, bgs = 3_000, 1024, [100, 101, 102, 103]
    calls = _batches(rng, rows, K, 24, per_batch=1_200)
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(PIPELINE_ALL)
        srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K,
                                         oplog_dense_serialized=False, max_rows=rows, max_entries=K))
        dev = [[torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs] for msgs in calls]
        torch.cuda.synchronize()
        for v, msgs in enumerate(dev):
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(msgs, bgs)])
        srv.sync()
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(EVENT_SCOPE, old[0])
        L.psx_debug_set_variant(DECODE, old[1])
    orc = OracleServer(bgs)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate(calls):
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    assert got == orc.serialize_records(3, list(range(rows)))
    orc.close()


@pytest.mark.parametrize("pipeline", [0, PIPELINE_ALL], ids=["unpipelined", "pipelined"])
@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted_map", "map"])
def test_indexed_calls_counted_by_idx_verify(kind, pipeline, walk_rank):
    """Indexed calls (every message with the producer's record offsets): idx_verify checks
    the chains over a grid and does ordered_count's work for the split tables, as the walk
    does on walked calls (including the reset of the split lists' counters).  Ten calls back
    to back, no sync between them, against the oracle byte for byte."""
    L = _abi.load()
    old = L.psx_debug_set_variant(WALK_COUNT, 1)
    rng = np.random.RandomState(900 + pipeline + kind)
    rows, K, bgs = 6_000, 1024, [100, 101, 102, 103]
    calls = _batches(rng, rows, K, 10, per_batch=2_500)
    try:
        srv = psa.Server(0, 1, bgs)
        srv.set_pipeline(pipeline)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        dev = [[torch.from_numpy(np.array(s, copy=True)).cuda() for s in msgs] for msgs in calls]
        idx = [[torch.from_numpy(wire.stream_record_offsets(np.asarray(s), {3: None}).view(np.int64)).cuda()
                for s in msgs] for msgs in calls]
        torch.cuda.synchronize()
        for v, (msgs, offs) in enumerate(zip(dev, idx)):
            srv.apply_indexed([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(msgs, bgs)],
                              [o.data_ptr() for o in offs])
        srv.sync()
        got = srv.serialize_rows(3, list(range(rows)))
        srv.close()
    finally:
        L.psx_debug_set_variant(WALK_COUNT, old)
    orc = OracleServer(bgs)
    orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
    for v, msgs in enumerate(calls):
        for s, bg in zip(msgs, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    want = orc.serialize_records(3, list(range(rows)))
    orc.close()
    if kind == SORTED_MAP:
        assert got == want
    else:
        assert _map_rows(got) == _map_rows(want)
