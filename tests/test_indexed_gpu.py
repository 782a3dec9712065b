"""psx_apply_indexed: messages applied with producer-supplied record
indexes, the sequential sparse record walk replaced by a parallel copy + chain check.

Parity: the same rows as the checker (oracle/psx_oracle.c walks the messages itself) and
as the unindexed device path — sorted-map rows byte-exact (entry order included), dense
rows bit-exact.  Indexes come from psx_pack_stream (device pack) and from a host walk
(wire.stream_record_offsets).  A wrong index is PSX_ERR_MALFORMED with nothing applied."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, PsxError
from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, I32

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _servers(rows, K, bgs):
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=K, max_rows=rows))
    srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=K))
    orc = OracleServer(list(bgs))
    orc.create_table(1, DENSE, F32, K)
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    return srv, orc


def _sparse_rows(rng, rows, K, n):
    out = []
    for r in rng.permutation(rows)[:n]:
        k = rng.randint(0, 33)                 # n = 0 records included
        cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
        out.append((int(r), cols, rng.choice([-3, -2, -1, 1, 2, 3], size=k).astype(np.int32)))
    return out


def _message(rng, rows, K):
    """Two tables in one message: sparse sorted-map records, then dense records."""
    sp = wire.sparse_stream_np(3, 4, _sparse_rows(rng, rows, K, rng.randint(1, rows)))
    ids = rng.permutation(rows)[:rng.randint(1, rows)].astype(np.int32)
    de = wire.dense_stream_np(1, ids, rng.normal(0, 1, (ids.size, K)).astype(np.float32))
    msg = np.concatenate([np.array([2], np.int32).view(np.uint8), sp[4:], de[4:]])
    return msg


@pytest.mark.parametrize("B", [1, 3, 8])
def test_indexed_matches_checker_and_walk(B):
    rng = np.random.RandomState(100 + B)
    rows, K = 700, 64
    bgs = list(range(10, 10 + B))
    srv, orc = _servers(rows, K, bgs)
    walk, _ = _servers(rows, K, bgs)
    for rnd in range(3):
        msgs = [_message(rng, rows, K) for _ in range(B)]
        offs = [wire.stream_record_offsets(m, {1: 4 * K, 3: None}) for m in msgs]
        dm = [torch.from_numpy(m.copy()).cuda() for m in msgs]
        do = [torch.from_numpy(o.view(np.int64)).cuda() for o in offs]
        # every other message indexed, the rest walked, in one call
        use = [o.data_ptr() if (b + rnd) % 2 == 0 else None for b, o in enumerate(do)]
        torch.cuda.synchronize()
        srv.apply_indexed([(d.data_ptr(), d.numel(), bg, rnd) for d, bg in zip(dm, bgs)], use)
        walk.apply_device([(d.data_ptr(), d.numel(), bg, rnd) for d, bg in zip(dm, bgs)])
        srv.sync()
        walk.sync()
        for m, bg in zip(msgs, bgs):
            assert orc.apply_stream(m, bg, rnd) == 0
    ids = list(range(rows))
    assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids) == walk.serialize_rows(3, ids)
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))


def test_pack_index_drives_indexed_apply():
    rng = np.random.RandomState(7)
    rows, K = 3000, 96
    packer = psa.Server(0, 9, [1])
    v = np.where(rng.rand(2500, K) < 0.9, 0, rng.randint(-5, 6, size=(2500, K))).astype(np.int32)
    tabs = [dict(table_id=3, dtype=I32, dense_serialized=False,
                 row_ids=torch.from_numpy(rng.permutation(rows)[:2500].astype(np.int32)).cuda(),
                 oplogs=torch.from_numpy(v).cuda())]
    msg, idx = packer.pack_stream(tabs, with_index=True)
    srv, orc = _servers(rows, K, [5])
    srv.apply_indexed([(msg.data_ptr(), msg.numel(), 5, 0)], [idx.data_ptr()])
    srv.sync()
    assert orc.apply_stream(msg.cpu().numpy(), 5, 0) == 0
    ids = list(range(rows))
    assert srv.serialize_rows(3, ids) == orc.serialize_records(3, ids)
    packer.close()


@pytest.mark.parametrize("where", ["first", "middle", "last", "misaligned"])
def test_bad_index_is_malformed(where):
    rng = np.random.RandomState(3)
    rows, K = 200, 32
    srv, _ = _servers(rows, K, [1, 2])
    m = _message(rng, rows, K)
    o = wire.stream_record_offsets(m, {1: 4 * K, 3: None}).copy()
    nsp = int(np.frombuffer(m[16:20].tobytes(), "<i4")[0])   # sparse records come first
    k = {"first": 0, "middle": nsp // 2, "last": nsp - 1, "misaligned": 1}[where]
    o[k] += 2 if where == "misaligned" else 4
    dm = torch.from_numpy(m.copy()).cuda()
    do = torch.from_numpy(o.view(np.int64)).cuda()
    torch.cuda.synchronize()
    srv.apply_indexed([(dm.data_ptr(), dm.numel(), 1, 0)], [do.data_ptr()])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 4
    assert not (srv.row_flags(3, 0, rows) & 1).any() and not (srv.row_flags(1, 0, rows) & 1).any()


@pytest.mark.parametrize("index", ["sound", "bad"])
def test_header_error_after_an_indexed_table(index):
    """decode_streams checks an indexed table's first and last offsets and steps past it;
    idx_verify checks the chain over a grid.  A header error found after the indexed table
    (here an unknown table id) waits for the index's verdict: with a sound index it is the
    call's error (PSX_ERR_UNKNOWN_TABLE, as the reader's CHECK), with a bad one the call is
    PSX_ERR_MALFORMED; nothing is applied either way."""
    rng = np.random.RandomState(11)
    rows, K = 200, 32
    srv, _ = _servers(rows, K, [1])
    m = _message(rng, rows, K)
    o = wire.stream_record_offsets(m, {1: 4 * K, 3: None}).copy()
    nsp = int(np.frombuffer(m[16:20].tobytes(), "<i4")[0])   # sparse records come first
    # the second table's id (its header follows the sparse table's last record) -> 9
    last = int(o[nsp - 1])
    n_last = int(np.frombuffer(m[last + 4:last + 8].tobytes(), "<i4")[0])
    hdr = last + 8 + 8 * n_last
    m[hdr:hdr + 4] = np.array([9], np.int32).view(np.uint8)
    if index == "bad":
        o[nsp // 2] += 4
    dm = torch.from_numpy(m.copy()).cuda()
    do = torch.from_numpy(o.view(np.int64)).cuda()
    torch.cuda.synchronize()
    srv.apply_indexed([(dm.data_ptr(), dm.numel(), 1, 0)], [do.data_ptr()])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == (3 if index == "sound" else 4)
    assert not (srv.row_flags(3, 0, rows) & 1).any() and not (srv.row_flags(1, 0, rows) & 1).any()
