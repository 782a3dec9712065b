"""GPU parity of the split sorted/map apply (256 < max_entries <= 1,024) in each of its
three launch forms (PSX_VARIANT_ORD_SPLIT, include/psx_debug.h): one 1,024-entry launch
(0), the 256- and 1,024-entry launches run concurrently on rows classified by
`entries + incs > 256` (1), and spill mode (2), where rows start on the 256-entry launch
unless already 7/8 full and a row that outgrows 256 entries mid-call is handed, untouched,
to a 1,024-entry launch that follows; (3) is spill mode with rows of >= 4 records listed
apart and taken first.

The rows are built to hit every branch of the spill: images that cross 256 entries inside
one call (spilled after some of their records were processed in registers), images that
start above 224 (classified big), rows that would be classified big by their Inc count
but never outgrow 256 (they stay on the small launch in spill mode), and ordinary rows.
Sorted-map rows byte-exact against the oracle (SortedVectorMapStore's entry order,
sorted_vector_map_store.hpp:175-197,305-337), map rows as {col -> value}."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, _abi
from oracle.oracle import OracleServer, SORTED_MAP, MAP, I32, F64, F32

pytestmark = pytest.mark.gpu
NP = {F32: np.float32, F64: np.float64, I32: np.int32}
VS = {F32: 4, F64: 8, I32: 4}
ORD_SPLIT = 6


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _vals(rng, k, dt, sign=True):
    if dt == I32:
        v = rng.randint(1, 4, size=k) * (rng.choice([-1, 1], size=k) if sign else 1)
    else:
        v = rng.normal(0, 1, size=k)
    return v.astype(NP[dt])


def _calls(rng, dt, rows, K):
    """Three calls of 4 messages.  Call 0 builds images of known sizes; calls 1-2 grow,
    shrink and cross the 256-entry line."""
    calls = []
    # call 0: row r gets an image of size sizes[r] (one record per message, disjoint columns)
    sizes = [0] * rows
    for r in range(rows):
        sizes[r] = [10, 60, 200, 240, 250, 300, 700, 200][r % 8]
    msgs = []
    for b in range(4):
        recs = []
        for r in range(rows):
            n = sizes[r]
            lo, hi = b * n // 4, (b + 1) * n // 4
            if hi > lo:
                cols = np.arange(lo, hi, dtype=np.int32)
                recs.append((r, cols, _vals(rng, cols.size, dt, sign=False)))
        msgs.append(recs)
    calls.append(msgs)
    for c in range(2):
        msgs = []
        for b in range(4):
            recs = []
            for r in rng.choice(rows, size=rows * 3 // 4, replace=False):
                kind = int(r) % 8
                if kind in (2, 3, 4):      # around 256: many new columns (inserts) + some found
                    k = int(rng.randint(20, 40))
                    cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
                elif kind == 7:            # entries + Incs > 256, but Incs on existing columns only
                    cols = np.arange(0, 30, dtype=np.int32)
                else:
                    k = int(rng.randint(1, 33))
                    cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
                recs.append((int(r), cols, _vals(rng, cols.size, dt)))
            msgs.append(recs)
        calls.append(msgs)
    return calls


def _as_map(raw, dt):
    """A serialized map row's packed (int32 col, V value) entries as {col: value bytes}."""
    es = 4 + VS[dt]
    return {int(np.frombuffer(raw[k:k + 4], np.int32)[0]): bytes(raw[k + 4:k + es]) for k in range(0, len(raw), es)}


@pytest.mark.parametrize("split", [3, 2, 1, 0], ids=["spill-heavy-first", "spill", "concurrent", "single"])
@pytest.mark.parametrize("kind,dt", [(SORTED_MAP, I32), (SORTED_MAP, F64), (MAP, I32)],
                         ids=["sorted-i32", "sorted-f64", "map-i32"])
def test_split_forms_match_oracle(split, kind, dt):
    L = _abi.load()
    old = L.psx_debug_set_variant(ORD_SPLIT, split)
    try:
        rng = np.random.RandomState(100 + 10 * kind + dt)
        rows, K = 512, 1024
        bgs = [100, 101, 102, 103]
        srv = psa.Server(0, 1, bgs)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=dt, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        orc = OracleServer(bgs)
        orc.create_table(3, kind, dt, 0, oplog_dense_serialized=False)
        for v, msgs in enumerate(_calls(rng, dt, rows, K)):
            streams = [wire.sparse_stream_np(3, VS[dt], recs) for recs in msgs]
            dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
            srv.sync()
            for s, bg in zip(streams, bgs):
                assert orc.apply_stream(s, bg, v) == 0
            ids = list(range(rows))
            if kind == SORTED_MAP:
                assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids), f"call {v}"
            else:
                for r in ids:
                    g, w = srv.serialize_rows(3, [r]), orc.serialize_records(3, [r])
                    assert len(g) == len(w), f"call {v} row {r}"
                    if g:
                        assert _as_map(g[12:], dt) == _as_map(w[12:], dt), f"call {v} row {r}"
        srv.close()
    finally:
        L.psx_debug_set_variant(ORD_SPLIT, old)


@pytest.mark.parametrize("split", [3, 1], ids=["spill-heavy-first", "concurrent"])
@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted", "map"])
def test_keys_outside_the_key_map_range(split, kind):
    """Split tables no longer scan every record's columns before the apply: the apply checks
    each record chunk's columns and finishes a row whose columns fall outside
    [0, max_entries) (negative keys, keys far past it, alone or in one chunk with keys inside
    it) without the key map; the capacity dry
    run takes only the rows whose entries + Incs exceed max_entries.  Byte-exact (sorted) /
    {col -> value} (map) against the oracle over several calls, mixing such rows with rows
    inside the range and rows whose Incs exceed max_entries without overflowing."""
    L = _abi.load()
    old = L.psx_debug_set_variant(ORD_SPLIT, split)
    try:
        rng = np.random.RandomState(7 + split + 10 * kind)
        rows, cap = 300, 512
        bgs = [100, 101, 102]
        srv = psa.Server(0, 1, bgs)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=cap, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=cap))
        orc = OracleServer(bgs)
        orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
        for v in range(4):
            msgs = []
            for b in range(3):
                recs = []
                for r in rng.choice(rows, size=200, replace=False):
                    r = int(r)
                    if r % 3 == 0:     # keys outside the map's range, few per row
                        cols = np.unique(rng.choice(np.r_[np.arange(-40, 0), np.arange(cap, cap + 80),
                                                          np.arange(100000, 100040)], size=rng.randint(1, 12)))
                        if r % 2:      # mixed into a record of keys inside it (one chunk, both kinds)
                            cols = np.unique(np.r_[cols, rng.choice(cap, size=rng.randint(1, 20))])
                    elif r % 3 == 1:   # many Incs on a few keys: entries + Incs > cap, no overflow
                        cols = np.arange(0, 200, dtype=np.int64)
                    else:
                        cols = np.unique(rng.choice(cap, size=rng.randint(1, 33)))
                    vals = rng.randint(1, 4, size=cols.size) * (1 if v == 0 else rng.choice([-1, 1], size=cols.size))
                    recs.append((r, cols.astype(np.int32), vals.astype(np.int32)))
                msgs.append(recs)
            streams = [wire.sparse_stream_np(3, 4, recs) for recs in msgs]
            dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
            srv.sync()
            for s, bg in zip(streams, bgs):
                assert orc.apply_stream(s, bg, v) == 0
        ids = list(range(rows))
        if kind == SORTED_MAP:
            assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids)
        else:
            for r in ids:
                g, w = srv.serialize_rows(3, [r]), orc.serialize_records(3, [r])
                assert len(g) == len(w), f"row {r}"
                if g:
                    assert _as_map(g[12:], I32) == _as_map(w[12:], I32), f"row {r}"
        srv.close()
    finally:
        L.psx_debug_set_variant(ORD_SPLIT, old)


def test_every_row_heavy_and_spilling():
    """Spill mode with heavy rows first when every row of the table is touched, has >= 4
    records in the call and outgrows 256 entries inside it: the heavy rows' descriptors and
    the spilled rows' descriptors (appended by the 256-entry launch while it runs) must not
    share list space.  R = 40,000 rows is more rows than waves resident at once, so late
    rows read their descriptors after early rows have spilled.  Byte-exact vs the oracle."""
    L = _abi.load()
    old = L.psx_debug_set_variant(ORD_SPLIT, 3)
    try:
        rows, K, dt = 40_000, 1024, I32
        bgs = [100, 101, 102, 103]
        srv = psa.Server(0, 1, bgs)
        srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=dt, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        orc = OracleServer(bgs)
        orc.create_table(3, SORTED_MAP, dt, 0, oplog_dense_serialized=False)
        rng = np.random.RandomState(2024)
        # call 0: 200 entries per row (50 columns per message, values 1..3: no zeros)
        c0 = [[(r, np.arange(50 * b, 50 * b + 50, dtype=np.int32),
                rng.randint(1, 4, size=50).astype(np.int32)) for r in range(rows)] for b in range(4)]
        # call 1: every row 4 records of 20 new columns each (200 + 80 > 256: every row spills)
        c1 = [[(r, np.arange(200 + 20 * b, 220 + 20 * b, dtype=np.int32),
                rng.randint(1, 4, size=20).astype(np.int32)) for r in range(rows)] for b in range(4)]
        for v, msgs in enumerate((c0, c1)):
            streams = [wire.sparse_stream_np(3, VS[dt], recs) for recs in msgs]
            dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
            srv.sync()
            for s, bg in zip(streams, bgs):
                assert orc.apply_stream(s, bg, v) == 0
        ids = list(range(rows))
        assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids)
        srv.close()
    finally:
        L.psx_debug_set_variant(ORD_SPLIT, old)


ORD_LITE = 22


@pytest.mark.parametrize("lite", [1, 0], ids=["lite", "one-row-per-wave"])
@pytest.mark.parametrize("kind,dt", [(SORTED_MAP, I32), (SORTED_MAP, F64), (SORTED_MAP, F32), (MAP, I32),
                                     (MAP, F64)], ids=["sorted-i32", "sorted-f64", "sorted-f32", "map-i32", "map-f64"])
def test_light_rows_four_to_a_wave(lite, kind, dt):
    """Light rows (<= 3 records in the call, image + Incs <= 64 entries: PSX_VARIANT_ORD_LITE)
    go four to a wave, 16 lanes each.  Rows built for every branch of the 16-lane path:
    inserts at every position (values of both signs and ties with existing values), found
    keys, entries that reach zero and are removed (first, middle, last, twice in a row),
    records of 1-48 pairs (1-3 sixteen-pair chunks), images from 0 to 64 entries, a row
    with exactly 64 entries after the call, and light rows mixed with heavy and 256-entry
    ones in one call; rows with < 4 live groups in the last quad.  Byte-exact (sorted) /
    {col -> value} (map) against the oracle over five calls, both with the light path on
    and off."""
    L = _abi.load()
    old_s = L.psx_debug_set_variant(ORD_SPLIT, 3)
    old_l = L.psx_debug_set_variant(ORD_LITE, lite)
    try:
        rng = np.random.RandomState(300 + 10 * kind + dt)
        rows, K = 1501, 1024     # 1501: the last light quad is partly empty
        bgs = [100, 101, 102, 103]
        srv = psa.Server(0, 1, bgs)
        srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=dt, row_capacity=K, oplog_dense_serialized=False,
                                         max_rows=rows, max_entries=K))
        orc = OracleServer(bgs)
        orc.create_table(3, kind, dt, 0, oplog_dense_serialized=False)
        for v in range(5):
            msgs = [[] for _ in bgs]
            for r in range(rows):
                if rng.rand() < 0.2:
                    continue
                cls = r % 10
                nrec = int(rng.randint(1, 4)) if cls < 8 else int(rng.randint(4, 7))   # light / heavy
                for m in rng.choice(len(bgs), size=min(nrec, len(bgs)), replace=False):
                    if cls == 9:      # wide rows: the 256-entry launch
                        cols = np.sort(rng.choice(K, size=rng.randint(40, 90), replace=False))
                    elif cls == 7:    # a small key space: found keys, zeros, removals
                        cols = np.sort(rng.choice(24, size=rng.randint(1, 20), replace=False))
                    else:
                        cols = np.sort(rng.choice(60, size=rng.randint(1, 16 if cls < 4 else 48 // nrec),
                                                  replace=False))
                    if dt == I32:
                        vals = rng.randint(1, 3, size=cols.size) * rng.choice([-1, 1], size=cols.size)
                    else:   # small integers in float: exact zeros and ties happen
                        vals = (rng.randint(1, 3, size=cols.size) * rng.choice([-1, 1], size=cols.size)).astype(float)
                    msgs[m].append((r, cols.astype(np.int32), vals.astype(NP[dt])))
            streams = [wire.sparse_stream_np(3, VS[dt], recs) for recs in msgs]
            dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
            srv.sync()
            for s, bg in zip(streams, bgs):
                assert orc.apply_stream(s, bg, v) == 0
            ids = list(range(rows))
            if kind == SORTED_MAP:
                assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids), f"call {v}"
            else:
                for r in ids:
                    g, w = srv.serialize_rows(3, [r]), orc.serialize_records(3, [r])
                    assert len(g) == len(w), f"call {v} row {r}"
                    if g:
                        assert _as_map(g[12:], dt) == _as_map(w[12:], dt), f"call {v} row {r}"
        srv.close()
    finally:
        L.psx_debug_set_variant(ORD_SPLIT, old_s)
        L.psx_debug_set_variant(ORD_LITE, old_l)


def test_light_path_is_a_variant_off_by_default():
    # one row per wave measured faster on C3 (profiles/r05/s9); the light path stays selectable
    assert _abi.load().psx_debug_get_variant(ORD_LITE) == 0


@pytest.mark.parametrize("kind", [SORTED_MAP, MAP], ids=["sorted", "map"])
def test_empty_records_and_one_chunk_rows(kind):
    """Records with no pairs (a sender may serialize an emptied row oplog), rows whose only
    records are empty, and empty records between full ones, as the last record of a message
    too: the apply takes an empty record as a chunk with no live lane.  Against the oracle
    over three calls on a split sorted-map table (256 < max_entries)."""
    rng = np.random.RandomState(41 + kind)
    rows, K = 400, 512
    bgs = [100, 101]
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(3, psa.TableInfo(row_kind=kind, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=K))
    orc = OracleServer(bgs)
    orc.create_table(3, kind, I32, 0, oplog_dense_serialized=False)
    for v in range(3):
        streams = []
        for b in range(2):
            recs = []
            for r in rng.choice(rows, size=150, replace=False):
                r = int(r)
                if r % 4 == 0:
                    cols = np.zeros(0, np.int32)                      # an empty record
                else:
                    space = K if r % 4 != 1 else 30            # r % 4 == 1: a small key space, overlaps
                    cols = np.sort(rng.choice(space, size=rng.randint(1, min(40, space)), replace=False))
                vals = rng.randint(1, 3, size=cols.size) * (1 if v == 0 else rng.choice([-1, 1], size=cols.size))
                recs.append((r, cols.astype(np.int32), vals.astype(np.int32)))
            recs.append((int(rng.randint(rows)), np.zeros(0, np.int32), np.zeros(0, np.int32)))   # last: empty
            streams.append(wire.sparse_stream_np(3, 4, recs))
        dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
        torch.cuda.synchronize()
        srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg in zip(dev, bgs)])
        srv.sync()
        for s, bg in zip(streams, bgs):
            assert orc.apply_stream(s, bg, v) == 0
    ids = list(range(rows))
    if kind == SORTED_MAP:
        assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids)
    else:
        for r in ids:
            g, w = srv.serialize_rows(3, [r]), orc.serialize_records(3, [r])
            assert len(g) == len(w), r
            if g:
                assert _as_map(g[12:], I32) == _as_map(w[12:], I32), r
    srv.close()
    orc.close()
