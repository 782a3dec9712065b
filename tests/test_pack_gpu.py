"""GPU parity of the device-side pack (psx_pack_stream) against the oracle's restatement
of the reference client packer (CreateOpLogMsgs + OpLogSerializer + RowOpLogSerializer,
abstract_bg_worker.cpp:590-649, oplog_serializer.hpp:12-37,
row_oplog_serializer.hpp:139-166, dense_row_oplog.hpp:112-136): byte-exact messages,
correct record-offset index, and pack -> apply round trips."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import PsxError
from oracle.oracle import OracleServer, pack_stream, DENSE, SORTED_MAP, F32, F64, I32, I64

pytestmark = pytest.mark.gpu
NP = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64}


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def srv():
    s = psa.Server(0, 1, [1])
    yield s
    s.close()


def _oplogs(rng, n, cap, dt, zero_frac):
    if dt in (I32, I64):
        v = rng.randint(-9, 10, size=(n, cap))
    else:
        v = rng.normal(size=(n, cap))
    v = np.where(rng.rand(n, cap) < zero_frac, 0, v)
    return v.astype(NP[dt])


def _dev(tables):
    return [dict(table_id=t["table_id"], dtype=t["dtype"], dense_serialized=t["dense_serialized"],
                 row_ids=torch.from_numpy(np.ascontiguousarray(t["row_ids"], np.int32)).cuda(),
                 oplogs=torch.from_numpy(np.ascontiguousarray(t["oplogs"])).cuda()) for t in tables]


def _check_index(msg, idx, tables):
    """Record offset k points at the row id of the k-th record in message order."""
    want_ids = []
    for t in sorted((t for t in tables if len(t["row_ids"])), key=lambda t: t["table_id"]):
        want_ids += list(np.asarray(t["row_ids"], np.int32))
    offs = idx.cpu().numpy()
    assert len(offs) == len(want_ids)
    got = [int(np.frombuffer(msg[o:o + 4], np.int32)[0]) for o in offs]
    assert got == [int(x) for x in want_ids]


@pytest.mark.parametrize("dt", [F32, F64, I32, I64])
@pytest.mark.parametrize("dense", [True, False])
@pytest.mark.parametrize("cap", [1, 7, 64, 300])
def test_single_table_byte_exact(srv, dt, dense, cap):
    rng = np.random.RandomState(cap * 10 + dt + (100 if dense else 0))
    n = 777
    t = dict(table_id=4, dtype=dt, dense_serialized=dense, row_ids=rng.permutation(5000)[:n].astype(np.int32),
             oplogs=_oplogs(rng, n, cap, dt, 0.6))
    t["oplogs"][5] = 0                     # an all-zero row: a sparse record with n = 0
    got, idx = srv.pack_stream(_dev([t]), with_index=True)
    msg = got.cpu().numpy().tobytes()
    assert msg == pack_stream([t])
    _check_index(msg, idx, [t])


def test_special_values_follow_the_zero_test(srv):
    """SerializeSparse drops `== 0` values: -0.0 is dropped, NaN and denormals kept."""
    v = np.array([[0.0, -0.0, np.nan, 1e-45, -np.inf, 3.0]], np.float32)
    t = dict(table_id=1, dtype=F32, dense_serialized=False, row_ids=np.array([9], np.int32), oplogs=v)
    got = srv.pack_stream(_dev([t])).cpu().numpy().tobytes()
    assert got == pack_stream([t])
    assert np.frombuffer(got[24:28], np.int32)[0] == 4     # n = 4 non-zeros


def test_multi_table_order_and_empty_tables(srv):
    rng = np.random.RandomState(2)
    tabs = [dict(table_id=9, dtype=I32, dense_serialized=False, row_ids=np.arange(50, dtype=np.int32),
                 oplogs=_oplogs(rng, 50, 40, I32, 0.8)),
            dict(table_id=2, dtype=F64, dense_serialized=True, row_ids=np.arange(30, dtype=np.int32) * 3,
                 oplogs=_oplogs(rng, 30, 12, F64, 0.0)),
            dict(table_id=5, dtype=F32, dense_serialized=True, row_ids=np.zeros(0, np.int32),
                 oplogs=np.zeros((0, 8), np.float32)),
            dict(table_id=7, dtype=F32, dense_serialized=False, row_ids=np.array([1, 2], np.int32),
                 oplogs=_oplogs(rng, 2, 1000, F32, 0.99))]
    got, idx = srv.pack_stream(_dev(tabs), with_index=True)
    msg = got.cpu().numpy().tobytes()
    assert msg == pack_stream(tabs)
    _check_index(msg, idx, tabs)
    assert srv.pack_stream(_dev([tabs[2]])).numel() == 0       # all empty -> empty message


def test_pack_then_apply_round_trip(srv):
    rng = np.random.RandomState(11)
    rows, K = 4000, 96
    tabs = [dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=rng.permutation(rows)[:3000].astype(np.int32),
                 oplogs=_oplogs(rng, 3000, K, F32, 0.0)),
            dict(table_id=3, dtype=I32, dense_serialized=False, row_ids=rng.permutation(rows)[:2500].astype(np.int32),
                 oplogs=_oplogs(rng, 2500, K, I32, 0.9))]
    msg = srv.pack_stream(_dev(tabs))
    s2 = psa.Server(0, 2, [5])
    s2.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=K, max_rows=rows))
    s2.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                    max_rows=rows, max_entries=K))
    s2.apply_device([(msg.data_ptr(), msg.numel(), 5, 0)])
    s2.sync()
    orc = OracleServer([5])
    orc.create_table(1, DENSE, F32, K)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    assert orc.apply_stream(msg.cpu().numpy(), 5, 0) == 0
    assert np.array_equal(s2.read_rows(1, 0, rows).view(np.uint8), orc.read_dense_rows(1, 0, rows).view(np.uint8))
    ids = list(range(rows))
    assert s2.serialize_rows(3, ids) == orc.serialize_records(3, ids)
    s2.close()


def test_large_dense_pack_matches_torch_builder(srv):
    from parameter_server_amd import wire
    n, cap = 1 << 16, 256
    ids = torch.randperm(n, device="cuda").to(torch.int32)
    op = torch.randn(n, cap, device="cuda")
    got = srv.pack_stream([dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=ids, oplogs=op)])
    assert torch.equal(got, wire.dense_stream_torch(1, ids, op))


def test_pack_errors(srv):
    t = dict(table_id=1, dtype=F32, dense_serialized=True, row_ids=np.arange(3, dtype=np.int32),
             oplogs=np.ones((3, 4), np.float32))
    with pytest.raises(PsxError):
        srv.pack_stream(_dev([t, dict(t)]))                          # same table twice
    with pytest.raises(PsxError):
        srv.pack_stream(_dev([dict(t, dtype=7)]))                    # bad dtype
