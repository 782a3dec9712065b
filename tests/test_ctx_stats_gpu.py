"""psx_ctx_stats (STATS_SERVER_ACCUM_APPLY_OPLOG_BEGIN/END, server_thread.cpp:240-244 ->
server_accum_apply_oplog_sec / server_accum_oplog_recv_mb, stats.cpp:1153-1162) and the
per-call events behind it: the counters after a few sync intervals, with one event pair per
interval (the default) and one per call (PSX_VARIANT_CALL_EVENTS bit 0); and calls made while
the pipeline mode changes between them (the slot-free events are recorded only while the
context pipelines, psx_ctx_set_pipeline drains the streams on a change) still give the
oracle's rows bit for bit."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, _abi
from oracle.oracle import OracleServer, DENSE, F32

pytestmark = pytest.mark.gpu
CALL_EVENTS = 17


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _msgs(rng, rows, cap, B, n):
    out = []
    for _ in range(B):
        ids = rng.permutation(rows)[:n].astype(np.int32)
        out.append(wire.dense_stream_np(1, ids, rng.normal(0, 1, (n, cap)).astype(np.float32)))
    return out


@pytest.mark.parametrize("per_call", [False, True], ids=["per-interval", "per-call"])
def test_stats_count_calls_messages_bytes_and_device_time(per_call):
    L = _abi.load()
    old = L.psx_debug_set_variant(CALL_EVENTS, 1 if per_call else 0)
    try:
        rng = np.random.RandomState(5)
        rows, cap, B = 4096, 64, 3
        srv = psa.Server(0, 1, [100 + b for b in range(B)])
        srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
        total = 0
        ver = 0
        for interval in range(3):
            for _ in range(4):
                ms = _msgs(rng, rows, cap, B, 1000)
                dev = [torch.from_numpy(m).cuda() for m in ms]
                srv.apply_device([(d.data_ptr(), d.numel(), 100 + b, ver) for b, d in enumerate(dev)])
                total += sum(m.size for m in ms)
                ver += 1
            srv.sync()
        st = srv.stats()
        assert st["calls"] == 12 and st["messages"] == 36 and st["oplog_bytes"] == total
        assert st["settled_calls"] == 12
        assert 0 < st["apply_sec"] < 5
        st2 = srv.stats(reset=True)
        assert st2["calls"] == 12
        assert srv.stats()["calls"] == 0 and srv.stats()["apply_sec"] == 0
        srv.close()
    finally:
        L.psx_debug_set_variant(CALL_EVENTS, old)


def test_pipeline_mode_changes_between_calls_bit_exact():
    rng = np.random.RandomState(9)
    rows, cap, B = 3000, 32, 4
    bgs = [100 + b for b in range(B)]
    init = rng.normal(0, 0.1, (rows, cap)).astype(np.float32)
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
    srv.load_rows(1, 0, init)
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, cap)
    orc.load_dense_rows(1, 0, init)
    keep = []
    for call, mode in enumerate([0, 2, 2, 0, 2, 0, 0, 2, 2, 2, 0]):
        srv.set_pipeline(mode)
        ms = _msgs(rng, rows, cap, B, 700)
        dev = [torch.from_numpy(m).cuda() for m in ms]
        keep.append(dev)
        srv.apply_device([(d.data_ptr(), d.numel(), bgs[b], call) for b, d in enumerate(dev)])
        for b, m in enumerate(ms):
            assert orc.apply_stream(m, bgs[b], call) == 0
    srv.sync()
    got = srv.read_rows(1, 0, rows)
    exp = orc.read_dense_rows(1, 0, rows)
    assert np.array_equal(got.view(np.int32), exp.view(np.int32))
    srv.close()
