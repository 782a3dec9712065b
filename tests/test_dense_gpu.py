"""GPU parity of the dense apply path: libpsx (HIP, gfx950) vs the CPU oracle on the
same serialized streams.  Integer rows must be bit-exact; float rows are bit-exact too
because per-row update order is preserved (tolerance 0 ulp; SURVEY §8(a) parity rules)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError
from oracle.oracle import OracleServer, DENSE, F32, F64, I32, I64

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


def _pair(dt, rows, row_cap, oplog_cap=None, bgs=range(100, 116), **geo):
    info = psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=dt, row_capacity=row_cap,
                         dense_row_oplog_capacity=oplog_cap or row_cap, max_rows=rows, **geo)
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(1, info)
    orc = OracleServer(list(bgs))
    orc.create_table(1, DENSE, dt, row_cap, dense_row_oplog_capacity=oplog_cap or row_cap)
    return srv, orc


def _apply_both(srv, orc, streams, bgs, versions):
    dev = [torch.from_numpy(s).cuda() for s in streams]
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg, v in zip(dev, bgs, versions)])
    srv.sync()
    for s, bg, v in zip(streams, bgs, versions):
        assert orc.apply_stream(s, bg, v) == 0


@pytest.mark.parametrize("dt", [F32, F64, I32, I64])
@pytest.mark.parametrize("B", [1, 2, 3, 5, 8, 16])
def test_fused_apply_bit_exact(dt, B):
    rng = np.random.RandomState(100 + B + 7 * dt)
    rows, cap = 700, 64
    srv, orc = _pair(dt, rows, cap)
    init = _vals(rng, (rows - 50, cap), dt)       # last 50 rows absent until touched
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams, bgs = [], []
    for b in range(B):
        n = rng.randint(1, rows + 1)
        ids = rng.permutation(rows)[:n].astype(np.int32)   # partial coverage, random order
        streams.append(wire.dense_stream_np(1, ids, _vals(rng, (n, cap), dt)))
        bgs.append(100 + b)
    _apply_both(srv, orc, streams, bgs, [0] * B)
    got = srv.read_rows(1, 0, rows)
    want = orc.read_dense_rows(1, 0, rows)
    assert np.array_equal(_bits(got), _bits(want))
    flags = srv.row_flags(1, 0, rows)
    for r in range(rows):
        assert bool(flags[r] & 1) == orc.row_exists(1, r)


@pytest.mark.parametrize("dt", [F32, F64])
def test_wide_rows_tail_and_oplog_capacity(dt):
    """row_capacity 320, dense_row_oplog_capacity 300: two 256-element chunks with a
    ragged tail; elements >= 300 are never touched (numeric_store_row.hpp:177-185)."""
    rng = np.random.RandomState(5)
    rows = 97
    srv, orc = _pair(dt, rows, 320, oplog_cap=300)
    init = _vals(rng, (rows, 320), dt)
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams = [wire.dense_stream_np(1, rng.permutation(rows).astype(np.int32), _vals(rng, (rows, 300), dt))
               for _ in range(5)]
    _apply_both(srv, orc, streams, [100 + b for b in range(5)], [0] * 5)
    got, want = srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows)
    assert np.array_equal(_bits(got), _bits(want))
    assert np.array_equal(_bits(got[:, 300:]), _bits(init[:, 300:]))


def test_special_float_values_bit_exact():
    """Denormals, signed zeros, infinities and huge magnitudes survive bit-for-bit."""
    rows, cap = 64, 256
    srv, orc = _pair(F32, rows, cap)
    specials = np.array([0.0, -0.0, 1e-45, -1e-45, 1.17e-38, 3.4e38, -3.4e38, np.inf, -np.inf, 1e-40],
                        dtype=np.float32)
    rng = np.random.RandomState(9)
    init = rng.choice(specials, size=(rows, cap)).astype(np.float32)
    srv.load_rows(1, 0, init)
    orc.load_dense_rows(1, 0, init)
    streams = [wire.dense_stream_np(1, rng.permutation(rows).astype(np.int32),
                                    rng.choice(specials[:7], size=(rows, cap)).astype(np.float32))
               for _ in range(4)]
    _apply_both(srv, orc, streams, [100, 101, 102, 103], [0] * 4)
    got, want = srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows)
    same = (_bits(got) == _bits(want)) | (np.isnan(got) & np.isnan(want))
    assert same.all()


def test_modulo_partition_geometry():
    """row_offset/row_stride reproduce the reference's server placement
    (client = (row / C) % num_clients, context.hpp:291-304): shard of rows 2, 5, 8, ..."""
    rng = np.random.RandomState(2)
    srv, orc = _pair(F32, 40, 16, row_offset=2, row_stride=3)
    ids = (2 + 3 * rng.permutation(40)).astype(np.int32)
    streams = [wire.dense_stream_np(1, ids, _vals(rng, (40, 16), F32)) for _ in range(2)]
    _apply_both(srv, orc, streams, [100, 101], [0, 0])
    got = srv.read_rows(1, 2, 40)
    want = orc.read_dense_rows(1, 2, 40, stride=3)
    assert np.array_equal(_bits(got), _bits(want))
    bad = wire.dense_stream_np(1, np.array([3], np.int32), np.ones((1, 16), np.float32))
    # the seam returns once the bytes are in HBM; the device's row-range check fails the
    # call at the next sync (PSX_SEAM_ASYNC), or in the call itself with PSX_SEAM_SYNC
    srv.ApplyOpLogUpdateVersion(bad, bad.size, 100, 1)
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 5
    srv.set_seam(1)
    with pytest.raises(PsxError) as e:
        srv.ApplyOpLogUpdateVersion(bad, bad.size, 101, 1)
    assert e.value.status == 5
    assert np.array_equal(_bits(srv.read_rows(1, 2, 40)), _bits(want))   # failed calls applied nothing


def test_host_path_sequence_matches_oracle():
    """Server::ApplyOpLogUpdateVersion on host bytes, one message per call, interleaved
    senders, including empty messages (server.cpp:120-179)."""
    rng = np.random.RandomState(21)
    rows, cap = 300, 40
    srv, orc = _pair(F32, rows, cap, bgs=[100, 101])
    ver = {100: 0, 101: 0}
    for step in range(12):
        bg = 100 + step % 2
        if step % 5 == 4:
            s = np.zeros(0, np.uint8)
        else:
            n = rng.randint(1, rows)
            s = wire.dense_stream_np(1, rng.permutation(rows)[:n].astype(np.int32), _vals(rng, (n, cap), F32))
        srv.ApplyOpLogUpdateVersion(s, s.size, bg, ver[bg])
        assert orc.apply_stream(s, bg, ver[bg]) == 0
        ver[bg] += 1
    srv.sync()
    assert np.array_equal(_bits(srv.read_rows(1, 0, rows)), _bits(orc.read_dense_rows(1, 0, rows)))
    assert srv.GetBgVersion(100) == orc.sender_version(100) == 5


def test_version_gap_applies_nothing():
    srv, orc = _pair(F32, 10, 8, bgs=[100])
    s = wire.dense_stream_np(1, np.array([1], np.int32), np.ones((1, 8), np.float32))
    d = torch.from_numpy(s).cuda()
    with pytest.raises(PsxError) as e:
        srv.apply_device([(d.data_ptr(), d.numel(), 100, 1)])
    assert e.value.status == 2
    with pytest.raises(PsxError) as e:
        srv.ApplyOpLogUpdateVersion(s, s.size, 100, 3)
    assert e.value.status == 2
    with pytest.raises(PsxError) as e:
        srv.apply_device([(d.data_ptr(), d.numel(), 999, 0)])
    assert e.value.status == 11
    srv.sync()
    assert not srv.read_rows(1, 0, 10).any()
    assert srv.GetBgVersion(100) == -1


def test_device_stream_errors_reported_at_sync():
    _device_stream_errors()


def _device_stream_errors():
    srv, _ = _pair(F32, 10, 8, bgs=[100, 101, 102])
    good = wire.dense_stream_np(1, np.array([1, 2], np.int32), np.ones((2, 8), np.float32))
    unknown = good.copy()
    unknown[4:8] = np.array([77], np.int32).view(np.uint8)
    out_of_range = wire.dense_stream_np(1, np.array([1, 50], np.int32), np.ones((2, 8), np.float32))
    cases = [(unknown, 3), (good[:-4].copy(), 4), (out_of_range, 5)]
    for i, (s, code) in enumerate(cases):
        d = torch.from_numpy(s).cuda()
        torch.cuda.synchronize()
        srv.apply_device([(d.data_ptr(), d.numel(), 100 + i, 0)])
        with pytest.raises(PsxError) as e:
            srv.sync()
        assert e.value.status == code
    assert not srv.read_rows(1, 0, 10).any()          # failed calls applied nothing
    srv.sync()                                         # error state cleared


@pytest.mark.parametrize("entry", ["device", "seam_async", "seam_sync"])
def test_rejected_call_gives_its_version_back(entry):
    """a call the device rejects (here a row outside the shard) applies nothing
    and gives its sender's version back, so the corrected message goes again with the same
    version — for device batches, the async seam (error at the next settle) and the sync
    seam (error from the call itself).  If the same sender's next call was accepted before
    the settle, the rejected version stays consumed and the error says so."""
    srv, orc = _pair(F32, 10, 8, bgs=[100, 101])
    if entry == "seam_sync":
        srv.set_seam(1)
    bad = wire.dense_stream_np(1, np.array([1, 50], np.int32), np.ones((2, 8), np.float32))
    good = wire.dense_stream_np(1, np.array([1, 2], np.int32), np.ones((2, 8), np.float32))

    def send(s, bg, v):
        if entry == "device":
            d = torch.from_numpy(s).cuda()
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, v)])
            srv.sync()
        else:
            srv.ApplyOpLogUpdateVersion(s, s.size, bg, v)
            srv.sync()

    with pytest.raises(PsxError) as e:
        send(bad, 100, 0)
    assert e.value.status == 5 and "version given back" in str(e.value)
    assert srv.GetBgVersion(100) == -1
    assert not srv.read_rows(1, 0, 10).any()
    send(good, 100, 0)                                   # the corrected message, same version
    assert orc.apply_stream(good, 100, 0) == 0
    assert srv.GetBgVersion(100) == 0
    assert np.array_equal(_bits(srv.read_rows(1, 0, 10)), _bits(orc.read_dense_rows(1, 0, 10)))
    if entry == "device":
        # a rejected call, then the same sender's next call accepted before the settle
        d0 = torch.from_numpy(bad.copy()).cuda()
        d1 = torch.from_numpy(good.copy()).cuda()
        torch.cuda.synchronize()
        srv.apply_device([(d0.data_ptr(), d0.numel(), 101, 0)])
        srv.apply_device([(d1.data_ptr(), d1.numel(), 101, 1)])
        with pytest.raises(PsxError) as e:
            srv.sync()
        assert "stays consumed" in str(e.value)
        assert srv.GetBgVersion(101) == 1
        assert orc.apply_stream(np.zeros(0, np.uint8), 101, 0) == 0      # the consumed version
        assert orc.apply_stream(good, 101, 1) == 0
        assert np.array_equal(_bits(srv.read_rows(1, 0, 10)), _bits(orc.read_dense_rows(1, 0, 10)))
        # two rejected calls of one sender back to back, and a batch carrying two of its
        # messages: every version comes back, newest first
        d2 = torch.from_numpy(bad.copy()).cuda()
        torch.cuda.synchronize()
        srv.apply_device([(d2.data_ptr(), d2.numel(), 100, 1)])
        srv.apply_device([(d2.data_ptr(), d2.numel(), 100, 2), (d2.data_ptr(), d2.numel(), 100, 3)])
        with pytest.raises(PsxError) as e:
            srv.sync()
        assert "stays consumed" not in str(e.value)
        assert srv.GetBgVersion(100) == 0


def test_duplicate_row_in_one_message_applied_in_order():
    """A row twice in one message is replayed on the ordered path: both records apply."""
    srv, orc = _pair(F32, 10, 8, bgs=[100])
    s = wire.dense_stream_np(1, np.array([3, 4, 3], np.int32), np.ones((3, 8), np.float32))
    _apply_both(srv, orc, [s], [100], [0])
    got = srv.read_rows(1, 0, 10)
    assert np.all(got[3] == 2.0) and np.all(got[4] == 1.0)
    assert np.array_equal(_bits(got), _bits(orc.read_dense_rows(1, 0, 10)))


def test_dirty_flags_and_serialize_rows():
    rng = np.random.RandomState(8)
    srv, orc = _pair(F32, 50, 12, bgs=[100])
    s = wire.dense_stream_np(1, np.array([4, 9, 30], np.int32), _vals(rng, (3, 12), F32))
    _apply_both(srv, orc, [s], [100], [0])
    f = srv.row_flags(1, 0, 50)
    assert set(np.nonzero(f)[0].tolist()) == {4, 9, 30} and (f[[4, 9, 30]] == 3).all()
    srv.clear_dirty(1)
    srv.sync()
    assert (srv.row_flags(1, 0, 50)[[4, 9, 30]] == 1).all()
    ids = [30, 5, 4]
    assert srv.serialize_rows(1, ids) == orc.serialize_records(1, ids)


def test_large_fused_apply_against_torch_reference():
    """2^18 rows x 256 f32 x 8 messages in random row order; the expected table is the
    in-order sum t + u_0 + ... + u_7 computed with fp32 torch adds (0-ulp tolerance)."""
    rows, cap, B = 1 << 18, 256, 8
    g = torch.Generator(device="cuda").manual_seed(1234)
    table = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
    srv, _ = _pair(F32, rows, cap)
    srv.load_rows(1, 0, None, on_device_ptr=table.data_ptr(), num_rows=rows)
    want = table.clone()
    streams = []
    for b in range(B):
        perm = torch.randperm(rows, device="cuda", generator=g).to(torch.int32)
        upd = torch.randn(rows, cap, device="cuda", generator=g) * 0.01
        streams.append(wire.dense_stream_torch(1, perm, upd))
        want[perm.long()] += upd
    torch.cuda.synchronize()
    srv.apply_device([(s.data_ptr(), s.numel(), 100 + b, 0) for b, s in enumerate(streams)])
    srv.sync()
    got = torch.empty_like(table)
    from parameter_server_amd import _abi
    assert _abi.load().psx_table_read_rows(srv.handle, 1, 0, rows, got.data_ptr(), 1) == 0
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))


def test_smoke_entry():
    import __graft_entry__
    __graft_entry__.smoke()


@pytest.mark.parametrize("apply_variant", [0, 1, 2], ids=["auto", "v2", "v4"])
def test_every_kernel_variant_bit_exact(apply_variant):
    """Every dense kernel the product can launch (include/psx_debug.h: v3 default, v2 the
    >= 4 GiB fallback, v4 the partial-coverage kernel) matches the oracle, including a
    ragged row tail (cap 301), rows narrower than one 16-byte vector (cap 3), partial
    coverage and 8-byte values."""
    from parameter_server_amd import _abi
    L = _abi.load()
    old_a = L.psx_debug_set_variant(1, apply_variant)
    try:
        for dt, cap, B in [(F32, 301, 9), (F64, 130, 8), (I32, 64, 3), (F32, 301, 7), (F32, 3, 5), (I64, 77, 6)]:
            rng = np.random.RandomState(apply_variant * 10 + cap)
            rows = 333
            srv, orc = _pair(dt, rows, cap)
            init = _vals(rng, (rows, cap), dt)
            srv.load_rows(1, 0, init)
            orc.load_dense_rows(1, 0, init)
            streams = []
            for b in range(B):
                n = rng.randint(1, rows + 1)
                streams.append(wire.dense_stream_np(1, rng.permutation(rows)[:n].astype(np.int32),
                                                    _vals(rng, (n, cap), dt)))
            _apply_both(srv, orc, streams, [100 + b for b in range(B)], [0] * B)
            assert np.array_equal(_bits(srv.read_rows(1, 0, rows)), _bits(orc.read_dense_rows(1, 0, rows)))
            srv.close()
    finally:
        L.psx_debug_set_variant(1, old_a)


def test_read_sweep_hook_measures_a_rate():
    """psx_debug_read_sweep (include/psx_debug.h): bench.py's same-run HBM read rate."""
    from parameter_server_amd import _abi
    L = _abi.load()
    buf = torch.ones(64 << 20, dtype=torch.uint8, device="cuda")
    g = L.psx_debug_read_sweep(buf.data_ptr(), buf.numel(), 3)
    assert 100.0 < g < 9000.0, g
    assert L.psx_debug_read_sweep(buf.data_ptr() + 4, buf.numel() - 16, 1) == -1.0   # misaligned
    assert L.psx_debug_read_sweep(buf.data_ptr(), 1024, 1) == -1.0                   # below one tile
