"""GPU parity of the AdaRevision server-table logic (psx_ada.hip) against the checker's
restatement of src/petuum_ps/server/adarevision_server_table_logic.cpp:14-197.

Bit-exact: rows, AdaRevisionRow state (accum_gradients_, z_, z_max_), row versions,
push bodies and live snapshot counts after every call and push.  The f32 rule runs in
the reference's operation order on both sides (no contraction, correctly rounded sqrt
and division), so there is no tolerance.  The Gaussian initial rows come from the
reference's generator (mt19937(12345) + normal_distribution<float>(0, 0.1), drawn by
libstdc++ on the device host and by the checker's restatement, which
tests/test_adarevision_oracle.py pins to libstdc++ bit for bit)."""
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


def _pair(rows, cap, bgs, step=0.1, gaussian=True, upper=10000, clients=2, importance=False, version=True,
          max_snaps=8):
    srv = psa.Server(0, 1, list(bgs))
    srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=cap, max_rows=rows,
                                     accum_importance=importance, version_maintain=version))
    srv.set_adarevision(1, init_step_size=step, gaussian_init=gaussian, old_grad_upper_bound=upper,
                        push_clients=clients, max_snapshots_per_row=max_snaps)
    orc = OracleServer(list(bgs))
    orc.create_table(1, DENSE, F32, cap, accum_importance=importance, version_maintain=version)
    assert orc.set_adarevision(1, init_step_size=step, gaussian_init=gaussian, old_grad_upper_bound=upper,
                               push_clients=clients) == 0
    return srv, orc


def _apply(srv, orc, streams, bgs, vers):
    dev = [torch.from_numpy(np.array(s, copy=True)).cuda() for s in streams]
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), bg, v) for d, bg, v in zip(dev, bgs, vers)])
    srv.sync()
    for s, bg, v in zip(streams, bgs, vers):
        assert orc.apply_stream(s, bg, v) == 0


@pytest.fixture(params=[0])
def ada_variant(request):
    """The register-resident state kernel (the only one; its 16-B and scalar element
    forms are both exercised through row_capacity % 4)."""
    yield request.param


def _check(srv, orc, rows, importance=False):
    u32 = np.uint32
    flags = srv.row_flags(1, 0, rows)
    live = np.nonzero(flags & 1)[0]
    assert np.array_equal(srv.read_rows(1, 0, rows).view(u32), orc.read_dense_rows(1, 0, rows).view(u32))
    acc, z, zm, nsnap = srv.adarevision_state(1, 0, rows)
    for r in range(rows):
        want = orc.ada_state(1, r)
        if want is None:
            assert r not in live
            continue
        for got, w in zip((acc[r], z[r], zm[r]), want):
            assert np.array_equal(got.view(u32), w.view(u32)), r
    assert nsnap == orc.ada_num_snapshots(1)
    if importance:
        # f64 importance: lane-parallel partial sums, rel <= 1e-12 of the element-order sum
        got_i = srv.row_importance(1, 0, rows)
        want_i = np.array([orc.importance(1, r) if r in live else 0.0 for r in range(rows)])
        assert np.allclose(got_i, want_i, rtol=1e-12, atol=0)
    got_v = srv.row_versions(1, 0, rows)
    assert np.array_equal(got_v, np.array([orc.row_version(1, r) for r in range(rows)], np.uint64))
    return got_v


class _Snapshots:
    """The test's model of old_accum_gradients_ keys, to write records that name live
    (row, version) pairs and release them with end_of_version."""

    def __init__(self, clients):
        self.live = {}
        self.clients = clients

    def pushed(self, body, versions):
        for rid in wire.parse_push_body(body).get(1, {}):
            self.live.setdefault((rid, int(versions[rid])), self.clients)

    def record(self, rng, rid):
        keys = [k for k in self.live if k[0] == rid]
        if not keys or rng.rand() < 0.25:
            return 0, False
        k = keys[rng.randint(len(keys))]
        eov = rng.rand() < 0.6
        if eov:
            self.live[k] -= 1
            if self.live[k] == 0:
                del self.live[k]
        return k[1], eov


@pytest.mark.parametrize("gaussian", [False, True])
@pytest.mark.parametrize("B", [1, 4, 16])
@pytest.mark.parametrize("importance", [False, True])
@pytest.mark.parametrize("cap", [70, 260])   # scalar / 16-B paths, ragged element tails
def test_adarevision_rounds_match_checker(gaussian, B, importance, cap, ada_variant):
    rng = np.random.RandomState(7 + 2 * B + gaussian + 4 * importance + cap)
    rows = 300
    bgs = list(range(10, 10 + B))
    srv, orc = _pair(rows, cap, bgs, step=0.05, gaussian=gaussian, clients=2, importance=importance)
    model = _Snapshots(2)
    for rnd in range(4):
        streams = []
        for b in range(B):
            n = rng.randint(1, rows // 2)
            ids = rng.permutation(rows)[:n].astype(np.int32)
            vv = [model.record(rng, int(r)) for r in ids]
            streams.append(wire.dense_variant_stream_np(
                1, ids, rng.normal(0, 1, (n, cap)).astype(np.float32),
                versions=np.array([v for v, _ in vv], np.uint64), end_of_version=[e for _, e in vv]))
        _apply(srv, orc, streams, bgs, [rnd] * B)
        versions = _check(srv, orc, rows, importance)
        got = srv.serialize_dirty(clear=True)
        want = orc.serialize_dirty([1], clear=True)
        assert bytes(got) == bytes(want)
        model.pushed(got, versions)
        _check(srv, orc, rows, importance)
        assert srv.adarevision_state(1, 0, 1)[3] == len(model.live)


def test_adarevision_plain_records(ada_variant):
    """A table without version_maintain: records carry no version (every record is
    version 0, server_table.cpp:527-535) and the push snapshots under version 0."""
    rng = np.random.RandomState(5)
    rows, cap = 200, 64
    srv, orc = _pair(rows, cap, [1, 2], version=False, gaussian=True)
    for rnd in range(3):
        streams = []
        for _ in range(2):
            ids = rng.permutation(rows)[:120].astype(np.int32)
            streams.append(wire.dense_stream_np(1, ids, rng.normal(0, 1, (120, cap)).astype(np.float32)))
        _apply(srv, orc, streams, [1, 2], [rnd, rnd])
        _check(srv, orc, rows)
        assert bytes(srv.serialize_dirty(clear=True)) == bytes(orc.serialize_dirty([1], clear=True))
        _check(srv, orc, rows)


def test_adarevision_allow_send_and_row_sent(ada_variant):
    rng = np.random.RandomState(9)
    rows, cap = 100, 33
    srv, orc = _pair(rows, cap, [1], upper=5, clients=1, gaussian=False)
    ids = np.arange(0, 40, dtype=np.int32)
    s = wire.dense_variant_stream_np(1, ids, rng.normal(0, 1, (40, cap)).astype(np.float32),
                                     versions=np.zeros(40, np.uint64))
    _apply(srv, orc, [s], [1], [0])
    # partial push: at most 100 rows by default, snapshots 40 > upper bound 5 afterwards
    got = srv.serialize_partial(clear=True)
    want = orc.serialize_partial([1], [100], clear=True)
    assert bytes(got) == bytes(want) and len(got) > 8
    _check(srv, orc, rows)
    s2 = wire.dense_variant_stream_np(1, ids[:10], rng.normal(0, 1, (10, cap)).astype(np.float32),
                                      versions=np.zeros(10, np.uint64))
    _apply(srv, orc, [s2], [1], [1])
    assert bytes(srv.serialize_partial(clear=True)) == b"" == orc.serialize_partial([1], [100], clear=True)
    # row request replies (Server::RowSent): a second snapshot under the current version
    srv.row_sent(1, [3, 4], 3)
    for r in (3, 4):
        assert orc.row_sent(1, r, 3) == 0
    _check(srv, orc, rows)


def test_adarevision_missing_snapshot_is_state_error(ada_variant):
    srv, orc = _pair(50, 16, [1], gaussian=False)
    s = wire.dense_variant_stream_np(1, np.array([2], np.int32), np.ones((1, 16), np.float32),
                                     versions=np.array([7], np.uint64))
    d = torch.from_numpy(np.array(s, copy=True)).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 1, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 13
    assert orc.apply_stream(s, 1, 0) == 13


def test_adarevision_duplicate_row_rejected():
    srv, _ = _pair(50, 16, [1], gaussian=False, version=False)
    s = wire.dense_stream_np(1, np.array([2, 5, 2], np.int32), np.ones((3, 16), np.float32))
    d = torch.from_numpy(np.array(s, copy=True)).cuda()
    torch.cuda.synchronize()
    srv.apply_device([(d.data_ptr(), d.numel(), 1, 0)])
    with pytest.raises(PsxError) as e:
        srv.sync()
    assert e.value.status == 10
    assert not (srv.row_flags(1, 0, 50) & 1).any()    # the call applied nothing
