"""The window-parallel decode (psx_walk.hip) against the one-workgroup-per-message decode
(decode_streams) and the CPU oracle, on the record-chain shapes that stress it: records
spanning several windows (16-96 KiB by walk shape), windows holding 6,144 records, tables ending mid-window and
exactly on a window boundary, several sparse and dense tables in one message, empty sparse
tables, messages of different lengths in one call, and malformed chains (the same error and
nothing applied).  Reference: SerializedOpLogReader (serialized_oplog_reader.hpp:30-133)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError, _abi
from oracle.oracle import OracleServer, DENSE, SORTED_MAP, MAP, F32, F64, I32, I64

pytestmark = pytest.mark.gpu
DECODE, WALK_CALLS = 7, 8
# psx_walk.hip kWalkShapes: the walk's window grid from byte 0 of a message, per shape
WINDOW_BYTES = {0: 98304, 1: 32768, 2: 24576, 3: 16384, 4: 49152, 5: 49152, 6: 49152}


def _window():
    return WINDOW_BYTES[_abi.load().psx_debug_get_variant(16)]
NP = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64}
VS = {F32: 4, F64: 8, I32: 4, I64: 8}


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


WALK_LEVELS = 15
WALK_SHAPE = 16
WALK_CUS = 12


@pytest.fixture(autouse=True, params=[(4, 0, 0), (1, 0, 0), (0, 0, 0), (4, 3, 4), (0, 2, 4), (2, 1, 4), (3, 4, 4), (4, 4, 1),
                                      (4, 6, 1)],
                ids=["levels4", "levels1", "levels0", "levels4-256x16K", "levels0-512x24K", "levels2-1024x32K",
                     "levels3-512x48K", "levels4-512x48K-default", "levels4-512x48Kx128"])
def walk_levels(request, _gpu):
    """Every test with the walk's composed exit maps at 4 levels (a window's exit state from the
    state 16 windows back), at 1 level (pairs) and off (window by window), on the 96 KiB
    window shape on half the CUs (round 3's form), on the smaller shapes (psx_debug.h
    PSX_VARIANT_WALK_SHAPE) with several blocks per CU, and on the default (48 KiB windows
    on every CU)."""
    L = _abi.load()
    levels, shape, cus = request.param
    old = L.psx_debug_set_variant(WALK_LEVELS, levels)
    old_s = L.psx_debug_set_variant(WALK_SHAPE, shape)
    old_c = L.psx_debug_set_variant(WALK_CUS, cus)
    yield levels
    L.psx_debug_set_variant(WALK_LEVELS, old)
    L.psx_debug_set_variant(WALK_SHAPE, old_s)
    L.psx_debug_set_variant(WALK_CUS, old_c)


def _message(tables):
    """tables: list of (table_id, vsize, rows) for sparse tables or (table_id, 'dense', ids,
    payload) for dense ones, in the given order (empty tables kept)."""
    parts = [np.array([len(tables)], np.int32).view(np.uint8)]
    for t in tables:
        if t[1] == "dense":
            parts.append(wire.dense_stream_np(t[0], np.asarray(t[2], np.int32), t[3])[4:])
        else:
            parts.append(wire.sparse_stream_np(t[0], t[1], t[2])[4:])
    return np.concatenate(parts)


def _rows(rng, ids, ncols, dt, nnz):
    out = []
    for rid, k in zip(ids, nnz):
        cols = np.sort(rng.choice(ncols, size=k, replace=False)).astype(np.int32)
        v = rng.randint(1, 4, size=k) if dt in (I32, I64) else rng.normal(0, 1, size=k)
        out.append((int(rid), cols, v.astype(NP[dt])))
    return out


class _Setup:
    """A libpsx server and the oracle with the same tables."""

    def __init__(self, tables, bgs):
        self.bgs = list(bgs)
        self.srv = psa.Server(0, 1, self.bgs)
        self.orc = OracleServer(self.bgs)
        self.tables = tables
        for tid, kind, dt, ncols, dense_ser, rows in tables:
            self.srv.CreateTable(tid, psa.TableInfo(row_kind=kind, dtype=dt, row_capacity=ncols,
                                                    oplog_dense_serialized=dense_ser, max_rows=rows,
                                                    max_entries=ncols if kind != DENSE else 0))
            self.orc.create_table(tid, kind, dt, ncols if kind == DENSE else 0, oplog_dense_serialized=dense_ser)

    def snapshot(self):
        return {t[0]: self.srv.serialize_rows(t[0], list(range(t[5]))) for t in self.tables}

    def oracle_snapshot(self):
        return {t[0]: self.orc.serialize_records(t[0], list(range(t[5]))) for t in self.tables}

    def apply(self, streams, ver, oracle=True):
        dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
        torch.cuda.synchronize()
        self.srv.apply_device([(d.data_ptr(), d.numel(), bg, ver) for d, bg in zip(dev, self.bgs)])
        self.srv.sync()
        if oracle:
            for s, bg in zip(streams, self.bgs):
                assert self.orc.apply_stream(s, bg, ver) == 0

    def close(self):
        self.srv.close()
        self.orc.close()


def _run_both(tables, streams):
    """Apply the streams with the window-parallel decode and with decode_streams (fresh
    servers); both must equal the oracle, and the walk must have run."""
    L = _abi.load()
    out = []
    for variant in (1, 0):
        old = L.psx_debug_set_variant(DECODE, variant)
        L.psx_debug_set_variant(WALK_CALLS, 0)
        try:
            st = _Setup(tables, range(100, 100 + len(streams)))
            st.apply(streams, 0)
            got, want = st.snapshot(), st.oracle_snapshot()
            st.close()
            walked = L.psx_debug_get_variant(WALK_CALLS)
        finally:
            L.psx_debug_set_variant(DECODE, old)
        assert got == want, f"decode variant {variant} differs from the oracle"
        assert (walked > 0) == (variant == 1)
        out.append(got)
    return out


def test_c3_shaped_messages_every_window():
    """Zipf rows, nnz 1..32, 8 messages of ~30 windows each into sorted-map rows."""
    rng = np.random.RandomState(5)
    rows, K = 20_000, 1024
    p = 1.0 / np.arange(1, rows + 1)
    p /= p.sum()
    streams = []
    for b in range(8):
        ids = rng.choice(rows, size=10_000, replace=False, p=p)
        streams.append(wire.sparse_stream_np(3, 4, _rows(rng, ids, K, I32, rng.randint(1, 33, size=ids.size))))
    _run_both([(3, SORTED_MAP, I32, K, False, rows)], streams)


def test_long_messages_chain_past_the_composed_span():
    """Messages of ~85 and ~35 windows with other message lengths beside them: with 4 levels a
    window's exit state comes from the state 16 windows back, so the chain between windows
    hops 16 at a time past the first span (and the table ends in the last window)."""
    rng = np.random.RandomState(17)
    rows, K = 30_000, 1024
    streams = []
    for b, nrec in enumerate((60_000, 25_000, 3_000)):
        ids = rng.randint(0, rows, size=nrec)
        streams.append(wire.sparse_stream_np(3, 4, _rows(rng, ids, K, I32, rng.randint(1, 33, size=ids.size))))
    _run_both([(3, SORTED_MAP, I32, K, False, rows)], streams)


@pytest.mark.parametrize("dt", [F32, F64])
def test_records_spanning_windows_and_tiny_records(dt):
    """Records of 8,000-24,000 (col, val) pairs (up to 4 windows each) between runs of
    one-pair records (3,072 per window), then a table of zero-pair records (6,144 per
    window) and one-pair records."""
    rng = np.random.RandomState(9)
    RA, KA, RB, KB = 1024, 24_000, 8192, 16
    ids = rng.permutation(RA)
    recs, i = [], 0
    for blk in range(6):
        for _ in range(2):
            recs += _rows(rng, [ids[i]], KA, dt, [rng.randint(8_000, 24_000)])
            i += 1
        recs += _rows(rng, ids[i:i + 150], KA, dt, [1] * 150)
        i += 150
    idb = rng.permutation(RB)
    tiny = [(int(r), np.zeros(0, np.int32), np.zeros(0, NP[dt])) for r in idb[:6000]]
    tiny += _rows(rng, idb[6000:7000], KB, dt, [1] * 1000)
    s = _message([(3, VS[dt], recs), (4, VS[dt], tiny)])
    _run_both([(3, DENSE, dt, KA, False, RA), (4, DENSE, dt, KB, False, RB)], [s])


def test_several_tables_per_message_ending_anywhere():
    """dense, sparse, dense, sparse, empty sparse, sparse tables in one message; table ends
    mid-window, on the first window boundary (padded to it exactly) and at the message end;
    messages of different lengths in one call of 16."""
    rng = np.random.RandomState(13)
    R, K, CAP = 3000, 512, 64
    tabs = [(1, DENSE, F32, CAP, True, R), (2, SORTED_MAP, I32, K, False, R), (4, DENSE, F32, CAP, True, R),
            (5, SORTED_MAP, I32, K, False, R), (6, SORTED_MAP, I32, K, False, R), (7, DENSE, I32, K, False, R)]
    streams = []
    for b in range(16):
        n = int(rng.randint(0, 600)) if b % 3 else 1
        ids = [rng.permutation(R)[:n] for _ in range(6)]
        parts = [(1, "dense", ids[0][: n // 2], rng.normal(0, 1, (n // 2, CAP)).astype(np.float32)),
                 (2, 4, _rows(rng, ids[1], K, I32, rng.randint(1, 40, size=n))),
                 (4, "dense", ids[2][:7], rng.normal(0, 1, (min(7, n), CAP)).astype(np.float32)),
                 (5, 4, _rows(rng, ids[3], K, I32, rng.randint(1, 9, size=n))),
                 (6, 4, []),
                 (7, 4, _rows(rng, ids[5], K, I32, rng.randint(0, 200, size=n)))]
        if b == 4:
            # table 2's records end exactly on the first window boundary of the message
            parts[0] = (1, "dense", ids[0][:1], rng.normal(0, 1, (1, CAP)).astype(np.float32))
            head = 4 + 16 + 1 * (4 + 4 * CAP) + 16
            WINDOW = _window()
            recs, used = [], head
            while used + 8 + 8 * 64 < WINDOW:
                recs += _rows(rng, [len(recs)], K, I32, [64])
                used += 8 + 8 * 64
            assert (WINDOW - used - 8) % 8 == 0
            recs += _rows(rng, [len(recs)], K, I32, [(WINDOW - used - 8) // 8])
            parts[1] = (2, 4, recs)
        streams.append(_message(parts))
    assert any(s.size > 65536 for s in streams) and len({s.size for s in streams}) > 8
    _run_both(tabs, streams)


def test_mixed_value_sizes_fall_back_to_block_decode():
    """Sparse tables of 4- and 8-byte values in one context: the speculation needs one
    record pair size, so the call takes decode_streams (and still matches the oracle)."""
    L = _abi.load()
    rng = np.random.RandomState(17)
    R, K = 500, 128
    tabs = [(2, SORTED_MAP, I32, K, False, R), (3, MAP, F64, K, False, R)]
    s = _message([(2, 4, _rows(rng, rng.permutation(R)[:300], K, I32, rng.randint(1, 20, size=300))),
                  (3, 8, _rows(rng, rng.permutation(R)[:300], K, F64, rng.randint(1, 20, size=300)))])
    old = L.psx_debug_set_variant(DECODE, 1)
    try:
        L.psx_debug_set_variant(WALK_CALLS, 0)
        st = _Setup(tabs, [100])
        st.apply([s], 0)
        assert st.snapshot() == st.oracle_snapshot()
        assert L.psx_debug_get_variant(WALK_CALLS) == 0
        st.close()
    finally:
        L.psx_debug_set_variant(DECODE, old)


def test_walk_is_the_default():
    assert _abi.load().psx_debug_get_variant(DECODE) == 1


def test_concurrent_contexts_on_recycled_workspaces():
    """Round 2's fault: two contexts walking at once, created right after contexts that
    walked and were closed (so their walk workspaces can be the freed ones, holding granules
    of earlier calls).  Each round closes both contexts and opens two new ones; every call
    of both is enqueued before either syncs; both must equal the oracle every round."""
    L = _abi.load()
    old = L.psx_debug_set_variant(DECODE, 1)
    try:
        rng = np.random.RandomState(29)
        rows, K = 3000, 256
        tabs = [(3, SORTED_MAP, I32, K, False, rows)]
        for rnd in range(4):
            L.psx_debug_set_variant(WALK_CALLS, 0)
            pair = [_Setup(tabs, [100, 101, 102]) for _ in range(2)]
            calls = []
            for ver in range(3):
                per = []
                for st in pair:
                    streams = [wire.sparse_stream_np(3, 4, _rows(rng, rng.permutation(rows)[:2500], K, I32,
                                                                 rng.randint(1, 40, size=2500)))
                               for _ in range(3)]
                    dev = [torch.from_numpy(np.array(x, copy=True)).cuda() for x in streams]
                    per.append((st, streams, dev))
                torch.cuda.synchronize()
                for st, streams, dev in per:
                    st.srv.apply_device([(d.data_ptr(), d.numel(), bg, ver) for d, bg in zip(dev, st.bgs)])
                calls.append(per)
            for st in pair:
                st.srv.sync()
            for ver, per in enumerate(calls):
                for st, streams, _ in per:
                    for x, bg in zip(streams, st.bgs):
                        assert st.orc.apply_stream(x, bg, ver) == 0
            assert L.psx_debug_get_variant(WALK_CALLS) == 6
            for st in pair:
                assert st.snapshot() == st.oracle_snapshot(), f"round {rnd}"
                st.close()
    finally:
        L.psx_debug_set_variant(DECODE, old)


def _malformed_cases():
    rng = np.random.RandomState(21)
    R, K = 4000, 256
    good = wire.sparse_stream_np(3, 4, _rows(rng, rng.permutation(R)[:3000], K, I32, rng.randint(1, 30, size=3000)))
    n0 = int(np.frombuffer(good[16:20], np.int32)[0])
    cases = {}
    cases["truncated"] = good[: good.size - 12]
    words = good.view(np.int32).copy()
    # record 1500's n negative: walk to it
    off, w = 5, []
    for r in range(2000):
        w.append(off)
        off += 2 + 2 * int(words[off + 1])
    bad = words.copy()
    bad[w[1500] + 1] = -3
    cases["negative_n"] = bad.view(np.uint8)
    bad = words.copy()
    bad[w[1999] + 1] = 1 << 28
    cases["n_past_end"] = bad.view(np.uint8)
    two = _message([(3, 4, _rows(rng, rng.permutation(R)[:2000], K, I32, rng.randint(1, 30, size=2000))),
                    (9, 4, _rows(rng, [1, 2], K, I32, [3, 3]))])
    cases["unknown_table_after_sparse"] = two
    dup = _message([(3, 4, _rows(rng, rng.permutation(R)[:2000], K, I32, rng.randint(1, 30, size=2000))),
                    (3, 4, _rows(rng, [1, 2], K, I32, [3, 3]))])
    cases["table_twice"] = dup
    more = words.copy()
    more[4] = n0 + 1          # one record more than the message holds
    cases["rows_past_end"] = more.view(np.uint8)
    return R, K, good, cases


@pytest.mark.parametrize("case", ["truncated", "negative_n", "n_past_end", "unknown_table_after_sparse",
                                  "table_twice", "rows_past_end"])
def test_malformed_chain_same_error_nothing_applied(case):
    L = _abi.load()
    R, K, good, cases = _malformed_cases()
    errs = []
    for variant in (1, 0):
        old = L.psx_debug_set_variant(DECODE, variant)
        try:
            st = _Setup([(3, SORTED_MAP, I32, K, False, R)], [100, 101])
            st.apply([good, np.zeros(0, np.uint8)], 0)
            before = st.snapshot()
            with pytest.raises(PsxError) as ei:
                st.apply([good, cases[case]], 1, oracle=False)
            errs.append(ei.value.status)
            assert st.snapshot() == before, f"variant {variant}: a failed call applied something"
            st.close()
        finally:
            L.psx_debug_set_variant(DECODE, old)
    assert errs[0] == errs[1]


def test_composed_exits_publish_early_on_c3_messages(walk_levels):
    """The composed exit maps must actually carry the chain (correct results alone would not
    show it: round 4 found the forward map refusing a record whose count word is the window's
    halo word, which silently sent most windows back to the one-by-one hand-off).  With the
    walk trace on, at least 90% of the non-last windows of C3-shaped messages publish their
    exit state from the composed map (trace word 6: tried, state, table, entry in range, map
    and records left all set) — the ones that cannot are where a table boundary or the message
    head breaks the span."""
    if walk_levels == 0:
        pytest.skip("composition off")
    import ctypes
    L = _abi.load()
    rng = np.random.RandomState(23)
    rows, K = 20_000, 1024
    p = 1.0 / np.arange(1, rows + 1)
    p /= p.sum()
    streams = []
    for b in range(8):
        ids = rng.choice(rows, size=10_000, replace=False, p=p)
        streams.append(wire.sparse_stream_np(3, 4, _rows(rng, ids, K, I32, rng.randint(1, 33, size=ids.size))))
    old = L.psx_debug_set_variant(11, 1)   # PSX_DEBUG_WALK_TRACE
    try:
        st = _Setup([(3, SORTED_MAP, I32, K, False, rows)], range(100, 108))
        st.apply(streams, 0, oracle=False)
        buf = np.zeros(10 * 8192, np.uint64)
        items = L.psx_debug_walk_trace(st.srv.handle, buf.ctypes.data_as(ctypes.c_void_p), 8192)
        st.close()
    finally:
        L.psx_debug_set_variant(11, old)
    assert items > 0
    tr = buf[: 10 * items].reshape(items, 10)
    B = 8
    nwin = items // B
    tried = early = 0
    for b in range(B):
        used = [j for j in range(nwin) if tr[j * B + b, 0] > 0]
        for j in used[:-1]:   # the message's last window publishes nothing
            code = int(tr[j * B + b, 6]) & 0xFF
            tried += 1
            early += code == 0x3F
    assert tried > 8 * 10
    assert early >= 0.9 * tried, f"{early} of {tried} windows published from the composed map"


def test_early_published_state_is_cross_checked(walk_levels):
    """An exit state published early from the composed maps is compared with the state the
    window's own resolve reaches; a difference fails the call before any record offset is used
    (later windows started from the early state).  PSX_DEBUG_WALK_SKEW shifts every early
    state by one record: the call must fail with nothing applied, and the same call with the
    skew off must then apply exactly as the oracle."""
    if walk_levels == 0:
        pytest.skip("composition off")
    L = _abi.load()
    rng = np.random.RandomState(31)
    rows, K = 20_000, 1024
    p = 1.0 / np.arange(1, rows + 1)
    p /= p.sum()
    streams = []
    for b in range(4):
        ids = rng.choice(rows, size=10_000, replace=False, p=p)
        streams.append(wire.sparse_stream_np(3, 4, _rows(rng, ids, K, I32, rng.randint(1, 33, size=ids.size))))
    SKEW = 21
    old = L.psx_debug_set_variant(SKEW, 1)
    try:
        st = _Setup([(3, SORTED_MAP, I32, K, False, rows)], range(100, 104))
        before = st.snapshot()
        with pytest.raises(PsxError):
            st.apply(streams, 0, oracle=False)
        assert st.snapshot() == before, "a call with a skewed early state applied something"
        st.close()
    finally:
        L.psx_debug_set_variant(SKEW, old)
    _run_both([(3, SORTED_MAP, I32, K, False, rows)], streams)
