"""GPU parity of the variant dense record formats against the CPU oracle.

* version tables (TableInfo.version_maintain, configs.hpp:207): records are
  VersionDenseRowOpLog = V[cap] + uint64 version + bool end_of_version
  (version_dense_row_oplog.hpp:161-180) — 9 trailing bytes, so records after the first
  are only byte-aligned — and rows are VersionServerRow: version_ = 1 at creation, +1 per
  applied record, appended to every serialized row (version_server_row.hpp:11-71).
  Row values bit-exact, versions and serialized bytes exact.
* float16 records (row_oplog_type kDenseRowOpLogFloat16, configs.hpp:39): uint16[cap]
  binary16 decompressed to f32 before the add (dense_row_oplog_float16.hpp:144-157).  The
  decompressor lives in the unvendored float16_compressor.hpp: parity for this format is
  UNPINNED; both sides restate IEEE binary16 -> binary32 (exact for every finite value and
  infinity).  Row values bit-exact (NaN compared as NaN).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError
from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, F64, I32, I64

pytestmark = pytest.mark.gpu
NP = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64}


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _vals(rng, shape, dt):
    if dt in (I32, I64):
        return rng.randint(-1000, 1000, size=shape).astype(NP[dt])
    return rng.normal(0, 1, size=shape).astype(NP[dt])


def _bits(a):
    return a.view(np.uint32 if a.dtype.itemsize == 4 else np.uint64)


def _pair(dt, rows, cap, bgs, tid=1, **kw):
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(tid, psa.TableInfo(row_kind=DENSE, dtype=dt, row_capacity=cap, max_rows=rows, **kw))
    orc = OracleServer(list(bgs))
    orc.create_table(tid, DENSE, dt, cap, accum_importance=kw.get("accum_importance", False),
                     version_maintain=kw.get("version_maintain", False),
                     f16_records=kw.get("row_oplog_type", 0) == 3)
    return srv, orc


def _apply_dev(srv, orc, streams, bgs, vers=None):
    vers = vers or [0] * len(streams)
    dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg, v in zip(dev, bgs, vers)])
    srv.sync()
    for s, bg, v in zip(streams, bgs, vers):
        assert orc.apply_stream(s, bg, v) == 0


def _version_stream(rng, tid, rows, n, cap, dt):
    ids = rng.permutation(rows)[:n].astype(np.int32)
    return wire.dense_variant_stream_np(tid, ids, _vals(rng, (n, cap), dt),
                                        versions=rng.randint(0, 1 << 40, size=n).astype(np.uint64),
                                        end_of_version=rng.rand(n) < 0.5)


def _check_versions(srv, orc, tid, rows):
    got = srv.row_versions(tid, 0, rows)
    want = np.array([orc.row_version(tid, r) for r in range(rows)], dtype=np.uint64)
    assert np.array_equal(got, want)
    return got


@pytest.mark.parametrize("dt", [F32, F64, I32, I64])
@pytest.mark.parametrize("B", [1, 3, 8])
def test_version_table_fused_apply(dt, B):
    rng = np.random.RandomState(31 * B + dt)
    rows, cap = 500, 77                      # odd cap: ragged tail, odd record strides
    bgs = list(range(100, 100 + B))
    srv, orc = _pair(dt, rows, cap, bgs, version_maintain=True)
    init = _vals(rng, (rows - 40, cap), dt)  # the last 40 rows are created by the apply
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams = [_version_stream(rng, 1, rows, rng.randint(1, rows + 1), cap, dt) for _ in range(B)]
    _apply_dev(srv, orc, streams, bgs)
    assert np.array_equal(_bits(srv.read_rows(1, 0, rows)), _bits(orc.read_dense_rows(1, 0, rows)))
    v = _check_versions(srv, orc, 1, rows)
    assert v.max() > 1
    ids = list(range(0, rows, 7))
    assert srv.serialize_rows(1, ids) == orc.serialize_records(1, ids)
    assert bytes(srv.serialize_dirty(clear=True)) == orc.serialize_dirty([1], clear=True)


def test_version_table_across_calls_host_path_and_replay():
    """Versions keep counting across calls; a row twice in one message (ordered replay)
    counts twice; the host entry point takes the odd-sized stream too."""
    rng = np.random.RandomState(4)
    rows, cap = 64, 16
    srv, orc = _pair(F32, rows, cap, [100, 101], version_maintain=True)
    for step in range(3):
        s = _version_stream(rng, 1, rows, 40, cap, F32)
        _apply_dev(srv, orc, [s], [100], [step])
    dup = wire.dense_variant_stream_np(1, np.array([5, 9, 5], np.int32), _vals(rng, (3, cap), F32),
                                       versions=np.array([1, 2, 3], np.uint64))
    srv.ApplyOpLogUpdateVersion(dup, dup.size, 101, 0)
    assert orc.apply_stream(dup, 101, 0) == 0
    assert np.array_equal(_bits(srv.read_rows(1, 0, rows)), _bits(orc.read_dense_rows(1, 0, rows)))
    _check_versions(srv, orc, 1, rows)
    assert srv.serialize_rows(1, [5, 9, 63]) == orc.serialize_records(1, [5, 9, 63])


def test_version_table_then_dense_table_in_one_message():
    """A plain dense table behind a version table starts at an odd offset: its records are
    byte-aligned and still apply bit-exactly.  A sparse table there is rejected (the
    sparse walk stages 4-byte words)."""
    rng = np.random.RandomState(5)
    rows, cap = 96, 24
    bgs = [100, 101, 102]
    srv = psa.Server(0, 1, bgs)
    orc = OracleServer(bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=cap, max_rows=rows, version_maintain=True))
    srv.CreateTable(2, psa.TableInfo(row_kind=DENSE, dtype=F64, row_capacity=cap, max_rows=rows))
    srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=cap, max_rows=rows,
                                     oplog_dense_serialized=False, max_entries=cap))
    orc.create_table(1, DENSE, F32, cap, version_maintain=True)
    orc.create_table(2, DENSE, F64, cap)
    orc.create_table(3, SORTED_MAP, I32, cap, oplog_dense_serialized=False)
    n = 33                                  # 33 * 9 trailer bytes: table 2 starts at an odd offset
    msg = wire.pack_np([
        dict(table_id=1, dense_serialized=True, row_ids=rng.permutation(rows)[:n].astype(np.int32),
             oplogs=_vals(rng, (n, cap), F32), versions=np.arange(n, dtype=np.uint64)),
        dict(table_id=2, dense_serialized=True, row_ids=rng.permutation(rows)[:50].astype(np.int32),
             oplogs=_vals(rng, (50, cap), F64))])
    _apply_dev(srv, orc, [msg], [100])
    for tid, dt in [(1, F32), (2, F64)]:
        assert np.array_equal(_bits(srv.read_rows(tid, 0, rows)), _bits(orc.read_dense_rows(tid, 0, rows)))
    _check_versions(srv, orc, 1, rows)
    assert not srv.row_versions(2, 0, rows).any()          # plain ServerRow: get_version() == 0
    bad = wire.pack_np([
        dict(table_id=1, dense_serialized=True, row_ids=np.array([1], np.int32),
             oplogs=np.ones((1, cap), np.float32), versions=np.array([0], np.uint64)),
        dict(table_id=3, dense_serialized=False, row_ids=np.array([2], np.int32),
             oplogs=np.ones((1, cap), np.int32))])
    srv.ApplyOpLogUpdateVersion(bad, bad.size, 101, 0)   # async seam: the device's check fails the call
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 10
    d = torch.from_numpy(np.array(bad, copy=True)).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 102, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 10


def test_version_table_config_errors():
    srv = psa.Server(0, 1, [100])
    with pytest.raises(PsxError) as e:
        srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=8, max_rows=8,
                                         oplog_dense_serialized=False, version_maintain=True))
    assert e.value.status == 10
    with pytest.raises(PsxError) as e:
        srv.CreateTable(2, psa.TableInfo(row_kind=DENSE, dtype=F64, row_capacity=8, max_rows=8, row_oplog_type=3))
    assert e.value.status == 10


def _halves(rng, shape, specials=True):
    h = rng.normal(0, 1, size=shape).astype(np.float16).view(np.uint16)
    if specials:
        pool = np.array([0x0000, 0x8000, 0x0001, 0x83ff, 0x0400, 0x7bff, 0xfbff, 0x7c00, 0xfc00, 0x3c00],
                        np.uint16)
        mask = rng.rand(*shape) < 0.1
        h = np.where(mask, rng.choice(pool, size=shape), h).astype(np.uint16)
    return h


def _same_f32(a, b):
    return bool(((_bits(a) == _bits(b)) | (np.isnan(a) & np.isnan(b))).all())


@pytest.mark.parametrize("B", [1, 2, 5, 8, 11])
@pytest.mark.parametrize("cap", [256, 301])
def test_float16_records_fused_apply(B, cap):
    """cap 301: 2-byte-aligned records and a ragged tail."""
    rng = np.random.RandomState(B * 7 + cap)
    rows = 640
    bgs = list(range(100, 100 + B))
    srv, orc = _pair(F32, rows, cap, bgs, row_oplog_type=3)
    init = rng.normal(0, 1, size=(rows - 30, cap)).astype(np.float32)
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams = []
    for _ in range(B):
        n = rng.randint(1, rows + 1)
        streams.append(wire.dense_variant_stream_np(1, rng.permutation(rows)[:n].astype(np.int32),
                                                    _halves(rng, (n, cap)), f16=True))
    _apply_dev(srv, orc, streams, bgs)
    assert _same_f32(srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows))


def test_float16_records_nan_payloads_and_replay():
    """NaN halves keep their payload in both restatements; a duplicate row goes through
    the ordered replay with the same decompression."""
    rows, cap = 16, 8
    srv, orc = _pair(F32, rows, cap, [100], row_oplog_type=3)
    h = np.array([[0x7e01, 0xfd55, 0x3c00, 0, 0x0200, 0x7c00, 0xbc00, 0x0001]] * 3, np.uint16)
    s = wire.dense_variant_stream_np(1, np.array([2, 3, 2], np.int32), h, f16=True)
    _apply_dev(srv, orc, [s], [100])
    got, want = srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows)
    assert _same_f32(got, want)
    assert got[2, 2] == 2.0 and got[3, 2] == 1.0


def test_float16_records_with_importance():
    rng = np.random.RandomState(12)
    rows, cap, B = 300, 64, 4
    bgs = list(range(100, 100 + B))
    srv, orc = _pair(F32, rows, cap, bgs, row_oplog_type=3, accum_importance=True)
    init = rng.normal(0, 1, size=(rows, cap)).astype(np.float32)
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams = [wire.dense_variant_stream_np(1, rng.permutation(rows)[:200].astype(np.int32),
                                            _halves(rng, (200, cap), specials=False), f16=True) for _ in range(B)]
    _apply_dev(srv, orc, streams, bgs)
    assert _same_f32(srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows))
    got = srv.row_importance(1, 0, rows)
    want = np.array([orc.importance(1, r) for r in range(rows)])
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)


def test_float16_records_large_against_torch():
    """2^16 rows x 256, 8 messages of binary16 records: the expected table is the in-order
    fp32 sum of the float32-converted halves (torch's conversion), 0-ulp tolerance."""
    rows, cap, B = 1 << 16, 256, 8
    g = torch.Generator(device="cuda").manual_seed(77)
    table = torch.randn(rows, cap, device="cuda", generator=g)
    srv, _ = _pair(F32, rows, cap, range(100, 100 + B), row_oplog_type=3)
    srv.load_rows(1, 0, None, on_device_ptr=table.data_ptr(), num_rows=rows)
    want = table.clone()
    msgs = []
    for b in range(B):
        perm = torch.randperm(rows, device="cuda", generator=g)
        upd = (torch.randn(rows, cap, device="cuda", generator=g) * 0.01).half()
        want[perm] += upd.float()
        s = wire.dense_variant_stream_np(1, perm.int().cpu().numpy(), upd.view(torch.int16).cpu().numpy(), f16=True)
        msgs.append(torch.from_numpy(s).cuda())
    torch.cuda.synchronize()
    srv.apply_device([(m.data_ptr(), m.numel(), 100 + b, 0) for b, m in enumerate(msgs)])
    srv.sync()
    got = torch.empty_like(table)
    from parameter_server_amd import _abi
    assert _abi.load().psx_table_read_rows(srv.handle, 1, 0, rows, got.data_ptr(), 1) == 0
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))


@pytest.mark.parametrize("variant", [0, 1], ids=["v3", "v2"])
def test_float16_apply_variants(variant):
    """Both fused-apply kernels for binary16 records (hardware conversion): the default
    saddr-addressed v3 and the v2 fallback; same rows as the checker (NaN as NaN), and
    the two kernels bit-identical to each other, NaN payloads included."""
    from parameter_server_amd import _abi
    L = _abi.load()
    old = L.psx_debug_set_variant(1, variant)
    try:
        rng = np.random.RandomState(40 + variant)
        rows, cap, B = 700, 256, 8
        bgs = list(range(100, 100 + B))
        srv, orc = _pair(F32, rows, cap, bgs, row_oplog_type=3)
        init = rng.normal(0, 1, size=(rows, cap)).astype(np.float32)
        srv.load_rows(1, 0, init)
        orc.load_dense_rows(1, 0, init)
        streams = []
        for _ in range(B):
            n = rng.randint(1, rows + 1)
            streams.append(wire.dense_variant_stream_np(1, rng.permutation(rows)[:n].astype(np.int32),
                                                        _halves(rng, (n, cap)), f16=True))
        _apply_dev(srv, orc, streams, bgs)
        got = srv.read_rows(1, 0, rows)
        assert _same_f32(got, orc.read_dense_rows(1, 0, rows))
        L.psx_debug_set_variant(1, 1 - variant)
        srv2, _ = _pair(F32, rows, cap, bgs, row_oplog_type=3)
        srv2.load_rows(1, 0, init)
        dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
        torch.cuda.synchronize()
        srv2.apply_device([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dev, bgs)])
        srv2.sync()
        assert np.array_equal(_bits(srv2.read_rows(1, 0, rows)), _bits(got))
    finally:
        L.psx_debug_set_variant(1, old)
