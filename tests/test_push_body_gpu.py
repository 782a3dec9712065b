"""Client side of serve-back on the GPU: push bodies the server context emits, applied to a
second context used as the client's cache (psx_apply_push_body = SerializedRowReader +
ResetRowData).  Checked against the body itself (wire.parse_push_body, the host parser
of serialized_row_reader.hpp) and against what the server holds: a reset row serializes
back to exactly the record's bytes."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


TABLES = [  # tid, kind, dtype, cap, rows, version
    (1, psa.ROW_DENSE, psa.F32, 40, 300, False),
    (2, psa.ROW_DENSE, psa.F64, 9, 300, True),
    (3, psa.ROW_SORTED_MAP, psa.I32, 64, 300, False),
    (4, psa.ROW_MAP, psa.F64, 64, 300, False),
]


def _ctx(bgs=(100,)):
    s = psa.Server(0, 1, list(bgs))
    for tid, kind, dt, cap, rows, ver in TABLES:
        s.CreateTable(tid, psa.TableInfo(row_kind=kind, dtype=dt, row_capacity=cap,
                                         oplog_dense_serialized=kind == psa.ROW_DENSE, max_rows=rows,
                                         max_entries=cap if kind != psa.ROW_DENSE else 0, version_maintain=ver))
    return s


def _message(rng, rows=300):
    parts = []
    for tid, kind, dt, cap, _, ver in TABLES:
        n = 120
        ids = rng.permutation(rows)[:n].astype(np.int32)
        npdt = {psa.F32: np.float32, psa.F64: np.float64, psa.I32: np.int32}[dt]
        if kind == psa.ROW_DENSE:
            op = rng.normal(size=(n, cap)).astype(npdt)
            d = dict(table_id=tid, dense_serialized=True, row_ids=ids, oplogs=op)
            if ver:
                d["versions"] = np.zeros(n, np.uint64)
        else:
            op = np.zeros((n, cap), npdt)
            for r in range(n):
                c = rng.choice(cap, size=rng.randint(1, 9), replace=False)
                op[r, c] = rng.randint(1, 4, size=c.size)
            d = dict(table_id=tid, dense_serialized=False, row_ids=ids, oplogs=op)
        parts.append(d)
    return wire.pack_np(parts)


def _rows_of(ctx, tid, rows):
    return ctx.serialize_rows(tid, list(range(rows)))


@pytest.mark.parametrize("on_device", [False, True])
def test_push_body_resets_cached_rows(on_device):
    rng = np.random.RandomState(21)
    srv, cli = _ctx(), _ctx()
    msg = _message(rng)
    srv.ApplyOpLogUpdateVersion(msg, msg.size, 100, 0)
    body = bytes(srv.serialize_dirty(clear=False))
    parsed = wire.parse_push_body(body)
    # the client caches the even rows of every table (row requests answered earlier)
    for tid, kind, dt, cap, rows, _ in TABLES:
        cli.subscribe(tid, np.arange(0, rows, 2, dtype=np.int32), 0)   # FindCreateRow: present, empty
    if on_device:
        d = torch.from_numpy(np.frombuffer(body, np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        cli.apply_push_body(None, device_ptr=d.data_ptr(), size=d.numel())
    else:
        cli.apply_push_body(body)
    for tid, kind, dt, cap, rows, ver in TABLES:
        for rid, rec in parsed[tid].items():
            got = cli.serialize_rows(tid, [rid])
            if rid % 2:                                   # not cached: skipped
                assert got == b"" or rid % 2 == 0
                continue
            assert got[12:] == rec, (tid, rid)
    # insert_missing (a row-request reply): every row of the body lands
    cli2 = _ctx()
    cli2.apply_push_body(body, insert_missing=True)
    for tid, kind, dt, cap, rows, ver in TABLES:
        assert _rows_of(cli2, tid, rows) == _rows_of(srv, tid, rows)


def test_push_body_last_record_wins_and_windows():
    """A row twice in one body ends with its last record; bodies far larger than the
    walker's 32 KiB LDS window, and one record larger than the window."""
    rows, cap = 5000, 300
    cli = psa.Server(0, 1, [100])
    cli.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
    cli.CreateTable(2, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=20000, max_rows=2))
    rng = np.random.RandomState(3)
    vals = rng.normal(size=(rows + 1, cap)).astype(np.float32)
    ids = list(range(rows)) + [7]
    parts = [np.array([1], np.int32).tobytes()]
    for k, rid in enumerate(ids):
        parts += [np.array([rid], np.int32).tobytes(), np.array([cap * 4], np.uint64).tobytes(), vals[k].tobytes()]
    big = rng.normal(size=20000).astype(np.float32)
    parts += [np.array([-1, 2, 1], np.int32).tobytes(), np.array([big.nbytes], np.uint64).tobytes(), big.tobytes(),
              np.array([-2], np.int32).tobytes()]
    body = b"".join(parts)
    for on_device in (False, True):
        if on_device:
            d = torch.from_numpy(np.frombuffer(body, np.uint8).copy()).cuda()
            torch.cuda.synchronize()
            cli.apply_push_body(None, insert_missing=True, device_ptr=d.data_ptr(), size=d.numel())
        else:
            cli.apply_push_body(body, insert_missing=True)
        got = cli.read_rows(1, 0, rows)
        want = vals[:rows].copy()
        want[7] = vals[rows]
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        assert np.array_equal(cli.read_rows(2, 1, 1)[0].view(np.uint32), big.view(np.uint32))


def test_malformed_push_body_applies_nothing():
    cli = psa.Server(0, 1, [100])
    cli.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=4, max_rows=10))
    good = np.array([1, 3], np.int32).tobytes() + np.array([16], np.uint64).tobytes() + np.ones(4, np.float32).tobytes()
    for bad in (good,                                             # no -2 terminator
                good + np.array([5], np.int32).tobytes() + np.array([999], np.uint64).tobytes(),   # size past the end
                np.array([9], np.int32).tobytes() + good[4:] + np.array([-2], np.int32).tobytes()):  # unknown table
        with pytest.raises(PsxError):
            cli.apply_push_body(bad, insert_missing=True)
        assert not cli.read_rows(1, 0, 10).any()
        assert not (cli.row_flags(1, 0, 10) & 1).any()
