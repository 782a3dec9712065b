"""DenseRowFloat16 rows on the GPU (psx_table_config.row_bytes_f16; dense_row_float16.hpp:13,
the row type apps/matrixfact's matrixfact_split16 registers, :47,560): stored and updated in
f32, served back as binary16 through Float16Compressor::compress (vector_store_float16.hpp:
91-99), reset on the client through decompress (:110-115).

Checked against the CPU oracle (orc_float_to_half, the restatement of the unvendored
compressor — parity unpinned): row reads and push bodies byte for byte, for
even and odd row widths (odd widths put records on 2-byte boundaries), the f32 rows bit for
bit; the device compressor on every value class (all 65,536 halves' floats and their
neighbours, the subnormal and overflow edges, NaNs, random floats over every exponent);
and a client cache resetting its rows from a pushed body (each value the decompressed
half)."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError
from oracle.oracle import OracleServer, DENSE, F32

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _tables(cap, rows, bgs=(100, 101)):
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows,
                                     row_bytes_f16=True))
    orc = OracleServer(list(bgs))
    orc.create_table(1, DENSE, F32, cap, f16_rows=True)
    return srv, orc


def _values(rng, shape):
    """f32 values of every class the compressor treats apart."""
    v = rng.normal(0, 1, size=shape) * np.exp2(rng.randint(-30, 20, size=shape))
    return v.astype(np.float32)


@pytest.mark.parametrize("cap", [64, 37])
def test_row_reads_and_push_bodies_match_the_oracle(cap):
    rng = np.random.RandomState(cap)
    rows = 300
    srv, orc = _tables(cap, rows)
    for ver in range(3):
        msgs = []
        for b in range(2):
            ids = rng.permutation(rows)[:150].astype(np.int32)
            msgs.append(wire.dense_stream_np(1, ids, _values(rng, (ids.size, cap))))
        dev = [torch.from_numpy(m).cuda() for m in msgs]
        torch.cuda.synchronize()
        srv.apply_device([(d.data_ptr(), d.numel(), 100 + b, ver) for b, d in enumerate(dev)])
        srv.sync()
        for b, m in enumerate(msgs):
            assert orc.apply_stream(m, 100 + b, ver) == 0
        # the f32 rows themselves
        got, want = srv.read_rows(1, 0, rows), orc.read_dense_rows(1, 0, rows)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        # row requests: {row_id; size; uint16[cap]} records
        ids = list(rng.permutation(rows)[:97]) + [rows - 1, 0]
        assert srv.serialize_rows(1, ids) == orc.serialize_records(1, ids)
        # a push of every dirty row (odd widths: records and the end marker 2-byte aligned)
        body = bytes(srv.serialize_dirty(clear=True))
        assert body == orc.serialize_dirty([1], clear=True)
    srv.close()
    orc.close()


def test_per_client_push_bodies_match_the_oracle():
    rng = np.random.RandomState(4)
    cap, rows = 21, 200
    srv, orc = _tables(cap, rows, bgs=(100,))
    srv.set_num_clients(3)
    for c in range(3):
        sub = rng.permutation(rows)[:80]
        srv.subscribe(1, sub, c)
        for r in sub:
            orc.subscribe(1, int(r), c)
    ids = rng.permutation(rows)[:170].astype(np.int32)
    m = wire.dense_stream_np(1, ids, _values(rng, (ids.size, cap)))
    d = torch.from_numpy(m).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    srv.sync()
    assert orc.apply_stream(m, 100, 0) == 0
    assert srv.serialize_push(clear=True) == orc.serialize_push([1], 3, clear=True)
    srv.close()
    orc.close()


def test_device_compressor_on_every_value_class(oracle_lib):
    """Rows loaded with crafted f32 values, read back as binary16: every half bit pattern's
    float and both its f32 neighbours, the subnormal and overflow edges, signed zeros,
    infinities, NaNs (quiet, signalling, small payloads), random floats of every exponent."""
    halves = np.arange(65536, dtype=np.uint16)
    f = np.array([oracle_lib.orc_half_to_float(int(h)) for h in halves], np.float32)
    f = f[np.isfinite(f)]
    vals = [f, np.nextafter(f, np.float32(np.inf)), np.nextafter(f, np.float32(-np.inf))]
    edge = np.array([65504, 65505, 65519, 65520, 65536, 1e9, 3.4e38, 2**-14, 2**-14 * (1 - 2**-11), 2**-24,
                     2**-25, 2**-25 * 1.5, 2**-26, 1e-40, 1e-45, 0.0], np.float32)
    vals += [edge, -edge]
    nan_bits = np.array([0x7FC00000, 0x7F800001, 0x7F801FFF, 0x7F802000, 0x7FBFFFFF, 0xFFC00000, 0xFF800001,
                         0x7F800000, 0xFF800000], np.uint32)
    vals.append(nan_bits.view(np.float32))
    rng = np.random.RandomState(9)
    vals.append(rng.randint(0, 2**32, size=200_000, dtype=np.uint64).astype(np.uint32).view(np.float32))
    v = np.concatenate(vals).astype(np.float32)
    cap = 1024
    rows = (v.size + cap - 1) // cap
    pad = np.zeros(rows * cap, np.float32)
    pad[: v.size] = v
    srv = psa.Server(0, 1, [100])
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows,
                                     row_bytes_f16=True))
    srv.load_rows(1, 0, pad.reshape(rows, cap))
    want = np.zeros(pad.size, np.uint16)   # the oracle on the raw bits (signalling NaNs untouched)
    oracle_lib.orc_floats_to_halves(pad.ctypes.data, want.ctypes.data, pad.size)
    # the host form (row reads) and the device form (a push body: serve_emit)
    raw = srv.serialize_rows(1, list(range(rows)))
    rec = np.frombuffer(raw, np.uint8).reshape(rows, 12 + 2 * cap)
    got = rec[:, 12:].copy().view(np.uint16).reshape(-1)
    assert np.array_equal(got, want), int(np.sum(got != want))
    srv.clear_dirty(1)
    # make every row dirty without changing a value: a record of zeros (x + 0 keeps x's bits
    # except -0 + 0 = +0 and NaN payloads quieted: compare against the rows the device now holds)
    m = wire.dense_stream_np(1, np.arange(rows, dtype=np.int32), np.zeros((rows, cap), np.float32))
    d = torch.from_numpy(m).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    now = srv.read_rows(1, 0, rows).reshape(-1)
    want2 = np.zeros(now.size, np.uint16)
    oracle_lib.orc_floats_to_halves(now.ctypes.data, want2.ctypes.data, now.size)
    body = bytes(srv.serialize_dirty(clear=True))
    got2 = np.zeros(now.size, np.uint16)
    for rid, payload in wire.parse_push_body(body)[1].items():
        got2[rid * cap:(rid + 1) * cap] = np.frombuffer(payload, np.uint16)
    assert np.array_equal(got2, want2), int(np.sum(got2 != want2))
    srv.close()


def test_client_cache_resets_from_binary16_rows():
    rng = np.random.RandomState(5)
    cap, rows = 48, 120
    srv, _ = _tables(cap, rows, bgs=(100,))
    cli = psa.Server(0, 2, [100])
    cli.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows,
                                     row_bytes_f16=True))
    ids = rng.permutation(rows)[:90].astype(np.int32)
    m = wire.dense_stream_np(1, ids, _values(rng, (ids.size, cap)))
    d = torch.from_numpy(m).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 100, 0)])
    srv.sync()
    body = bytes(srv.serialize_dirty(clear=True))
    cli.apply_push_body(body, insert_missing=True)
    got = cli.read_rows(1, 0, rows)
    want = np.zeros((rows, cap), np.float32)
    for rid, payload in wire.parse_push_body(body)[1].items():
        want[rid] = np.frombuffer(payload, np.float16).astype(np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    srv.close()
    cli.close()


def test_odd_width_client_cache_is_refused_and_non_float_rows_rejected():
    cli = psa.Server(0, 2, [100])
    cli.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=7, max_rows=4,
                                     row_bytes_f16=True))
    with pytest.raises(PsxError) as e:
        cli.apply_push_body(np.array([1, 0, -2], np.int32).tobytes())
    assert e.value.status == 10   # PSX_ERR_UNSUPPORTED
    with pytest.raises(PsxError) as e:
        cli.CreateTable(2, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F64, row_capacity=8, max_rows=4,
                                         row_bytes_f16=True))
    assert e.value.status == 10
    cli.close()


def test_odd_width_f16_table_then_dense_f64_and_sorted_tables_in_one_push():
    """an odd-width binary16 table leaves the next table's records on a 2-byte
    boundary in the same push body; the dense f64 and sorted-map tables behind it must come
    out byte for byte as the oracle writes them (their word stores go out as 16-bit halves
    there, psx_serve.hip emit_row)."""
    from oracle.oracle import SORTED_MAP, F64, I32
    rng = np.random.RandomState(77)
    cap, rows, K = 37, 90, 64
    bgs = [100]
    srv = psa.Server(0, 1, bgs)
    orc = OracleServer(bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows,
                                     row_bytes_f16=True))
    orc.create_table(1, DENSE, F32, cap, f16_rows=True)
    srv.CreateTable(2, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F64, row_capacity=5, max_rows=rows))
    orc.create_table(2, DENSE, F64, 5)
    srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=K))
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    msgs = []
    ids = rng.permutation(rows)[:31].astype(np.int32)          # an odd number of odd-width rows
    msgs.append(wire.dense_stream_np(1, ids, _values(rng, (ids.size, cap))))
    ids2 = rng.permutation(rows)[:40].astype(np.int32)
    msgs.append(wire.dense_stream_np(2, ids2, rng.normal(0, 1, (ids2.size, 5))))
    recs = []
    for rid in rng.choice(rows, size=25, replace=False):
        k = rng.randint(1, 12)
        cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
        recs.append((int(rid), cols, rng.randint(1, 4, size=k).astype(np.int32)))
    msgs.append(wire.sparse_stream_np(3, 4, recs))
    for v, m in enumerate(msgs):
        d = torch.from_numpy(m).cuda()
        torch.cuda.synchronize()
        srv.apply_device([(d.data_ptr(), d.numel(), 100, v)])
        srv.sync()
        assert orc.apply_stream(m, 100, v) == 0
    got = bytes(srv.serialize_dirty(clear=True))
    want = bytes(orc.serialize_dirty([1, 2, 3], clear=True))
    assert got == want
    srv.close()
