"""Server clocks, subscriptions and the per-client push (SSPPush) on the GPU, against the
oracle's restatement, and SURVEY §8(d) C5: a clocked mixed dense + sparse stream under
SSP staleness 4, every push body of every client compared byte for byte.

The caller is parameter_server_amd.ServerThread (server_thread.cpp:185-299), run once
over libpsx and once over the oracle on the identical message/request sequence.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire, ServerThread
from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, I32
from oracle_backend import OracleBackend

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_clock_until_matches_vector_clock():
    rng = np.random.RandomState(5)
    bgs = [1100, 2100, 3100, 4100, 5100]
    srv = psa.Server(0, 1, bgs)
    orc = OracleServer(bgs)
    assert srv.GetMinClock() == orc.min_clock() == 0
    clocks = {b: 0 for b in bgs}
    for _ in range(300):
        b = bgs[rng.randint(len(bgs))]
        target = clocks[b] + rng.randint(0, 3)
        clocks[b] = target
        assert srv.ClockUntil(b, target) == orc.clock_until(b, target)
        assert srv.GetMinClock() == orc.min_clock() == min(clocks.values())
        assert srv.sender_clock(b) == target


def _backends(bgs, C, tables):
    srv = psa.Server(0, 1, bgs)
    srv.set_num_clients(C)
    orc = OracleBackend(bgs, C)
    for tid, kind, dt, cap, rows in tables:
        dense_ser = kind == psa.ROW_DENSE
        srv.CreateTable(tid, psa.TableInfo(row_kind=kind, dtype=dt, row_capacity=cap, oplog_dense_serialized=dense_ser,
                                           max_rows=rows, max_entries=cap if kind != psa.ROW_DENSE else 0))
        orc.create(tid, kind, dt, cap, dense_ser)
    return srv, orc


def test_per_client_push_follows_subscriptions():
    """Three clients subscribe to different rows; a push sends each client its subscribed
    dirty rows, leaves unsubscribed dirty rows dirty (server_table.cpp:222-225), and a row
    subscribed later goes out with the next push."""
    rng = np.random.RandomState(6)
    C, rows, cap, K = 3, 200, 16, 32
    bgs = [c * 1000 + 100 for c in range(C)]
    srv, orc = _backends(bgs, C, [(1, psa.ROW_DENSE, F32, cap, rows), (3, psa.ROW_SORTED_MAP, I32, K, rows)])
    for c in range(C):
        for tid in (1, 3):
            sub = rng.choice(rows, size=40, replace=False).astype(np.int32)
            srv.subscribe(tid, sub, c)
            orc.subscribe(tid, sub, c)
    for t in (1, 3):
        got = srv.row_subscriptions(t, 0, rows)
        assert [int(x) for x in got] == [orc.o.row_subs(t, r) for r in range(rows)]
    for rnd in range(3):
        for b, bg in enumerate(bgs):
            ids1 = rng.permutation(rows)[:120].astype(np.int32)
            ids3 = rng.permutation(rows)[:60].astype(np.int32)
            cnt = np.zeros((60, K), np.int32)
            for r in range(60):
                cc = rng.choice(K, size=rng.randint(1, 6), replace=False)
                cnt[r, cc] = rng.choice([-1, 1, 2], size=cc.size)
            msg = wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=ids1,
                                     oplogs=rng.normal(size=(120, cap)).astype(np.float32)),
                                dict(table_id=3, dense_serialized=False, row_ids=ids3, oplogs=cnt)])
            srv.ApplyOpLogUpdateVersion(msg, msg.size, bg, rnd)
            orc.ApplyOpLogUpdateVersion(msg, msg.size, bg, rnd)
        got, want = srv.serialize_push(), orc.serialize_push()
        assert got == want, f"round {rnd}"
        assert all(len(g) > 16 for g in got)
        # dirty rows nobody subscribes to stay dirty
        flags = srv.row_flags(1, 0, rows)
        for r in range(rows):
            assert bool(flags[r] & 2) == orc.o.row_dirty(1, r)
        late = int(rng.randint(rows))
        srv.subscribe(1, [late], 2)
        orc.subscribe(1, [late], 2)


def _c5_workload(rng, C, rows_d, cap, rows_s, K, per_client_d, per_client_s):
    ids_d = rng.permutation(rows_d)[:per_client_d].astype(np.int32)
    ids_s = rng.choice(rows_s, size=per_client_s, replace=False).astype(np.int32)
    cnt = np.zeros((per_client_s, K), np.int32)
    for r in range(per_client_s):
        cc = rng.choice(K, size=rng.randint(1, 17), replace=False)
        cnt[r, cc] = rng.choice([-1, 1, 2], size=cc.size)
    return wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=ids_d,
                              oplogs=rng.normal(0, 0.01, size=(per_client_d, cap)).astype(np.float32)),
                         dict(table_id=3, dense_serialized=False, row_ids=ids_s, oplogs=cnt)])


def test_c5_ssp_staleness4_clocked_stream():
    """C5 (reduced): 8 clients (one bg thread each), a dense f32 table and a sorted-map
    int32 table, 14 clocks.  Clients send one is_clock message per clock in a random
    arrival order bounded by SSP staleness 4 (a client at clock c blocks in Get until the
    server's pushed min clock reaches c - 4, ssp_push_consistency_controller.cpp:70-88);
    row requests arrive along the way (some wait for their clock, server.cpp:81-118).
    Every push body of every client and every row-request reply must match the oracle."""
    rng = np.random.RandomState(55)
    C, staleness, clocks = 8, 4, 14
    rows_d, cap, rows_s, K = 4096, 64, 3000, 128
    bgs = [c * 1000 + 100 for c in range(C)]
    srv, orc = _backends(bgs, C, [(1, psa.ROW_DENSE, F32, cap, rows_d), (3, psa.ROW_SORTED_MAP, I32, K, rows_s)])
    log = {"gpu": [], "orc": []}
    threads = {
        "gpu": ServerThread(srv, lambda bodies, clk: log["gpu"].append(("push", clk, bodies)),
                            lambda bg, t, r, clk, rec: log["gpu"].append(("reply", bg, t, r, clk, rec))),
        "orc": ServerThread(orc, lambda bodies, clk: log["orc"].append(("push", clk, bodies)),
                            lambda bg, t, r, clk, rec: log["orc"].append(("reply", bg, t, r, clk, rec))),
    }
    for c in range(C):   # initial reads: every client subscribes to its working set
        for tid, n in ((1, rows_d), (3, rows_s)):
            sub = rng.choice(n, size=n // 4, replace=False)
            for th in threads.values():
                th.server.subscribe(tid, sub.astype(np.int32), c)
    client_clock = [0] * C
    min_pushed = 0
    events = 0
    while min(client_clock) < clocks:
        ready = [c for c in range(C) if client_clock[c] < clocks and client_clock[c] - min_pushed <= staleness]
        c = int(rng.choice(ready))
        msg = _c5_workload(rng, C, rows_d, cap, rows_s, K, rows_d // 4, 200)
        req = None
        if rng.rand() < 0.3:   # a Get that misses the cache: row request at the client's clock
            req = (bgs[c], 3, int(rng.randint(rows_s)), client_clock[c] + int(rng.randint(0, 3)))
        for th in threads.values():
            if req:
                th.HandleRowRequest(*req)
            th.HandleOpLogMsg(bgs[c], msg, True, client_clock[c] + 1, client_clock[c])
        client_clock[c] += 1
        min_pushed = srv.GetMinClock()
        events += 1
    assert srv.GetMinClock() == orc.GetMinClock() == clocks
    assert len(log["gpu"]) == len(log["orc"]) and len(log["gpu"]) >= clocks
    for k, (g, o) in enumerate(zip(log["gpu"], log["orc"])):
        assert g == o, f"event {k}: {g[0]}"
    np.testing.assert_array_equal(srv.read_rows(1, 0, rows_d).view(np.uint32),
                                  orc.o.read_dense_rows(1, 0, rows_d).view(np.uint32))
    assert srv.serialize_rows(3, list(range(rows_s))) == orc.o.serialize_records(3, list(range(rows_s)))


def test_handle_oplog_msg_whole_messages():
    """psx_handle_oplog_msg on whole ClientSendOpLogMsgs (41-byte header + stream): apply,
    then ClockUntil(sender, bg_clock) for clock messages; same rows and clocks as the oracle."""
    import ctypes
    from parameter_server_amd import _abi
    rng = np.random.RandomState(31)
    bgs, cap, rows = [1100, 2100], 8, 50
    srv = psa.Server(0, 1, bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, cap)
    L = _abi.load()
    ver = {b: 0 for b in bgs}
    clk = {b: 0 for b in bgs}
    for step in range(12):
        bg = bgs[step % 2] if step < 8 else bgs[0]
        s = wire.dense_stream_np(1, rng.permutation(rows)[:20].astype(np.int32),
                                 rng.normal(size=(20, cap)).astype(np.float32))
        is_clock = step % 3 != 2
        if is_clock:
            clk[bg] += 1
        msg = wire.encode_oplog_msg(s, version=ver[bg], client_id=bg // 1000, is_clock=is_clock, bg_clock=clk[bg])
        changed = ctypes.c_int32()
        assert L.psx_handle_oplog_msg(srv.handle, ctypes.c_void_p(msg.ctypes.data), msg.size, bg,
                                      ctypes.byref(changed)) == 0
        assert orc.apply_stream(s, bg, ver[bg]) == 0
        want = orc.clock_until(bg, clk[bg]) if is_clock else 0
        assert changed.value == want
        ver[bg] += 1
    assert srv.GetMinClock() == orc.min_clock()
    assert np.array_equal(srv.read_rows(1, 0, rows).view(np.uint32), orc.read_dense_rows(1, 0, rows).view(np.uint32))


def test_compat_mode_rejects_2gib_messages():
    from parameter_server_amd import _abi
    srv = psa.Server(0, 1, [100])
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=4, max_rows=8))
    assert _abi.load().psx_ctx_set_compat(srv.handle, _abi.COMPAT_INT32_STREAM_OFFSETS) == 0
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(psa.PsxError) as e:
        srv.apply_device([(d.data_ptr(), 1 << 31, 100, 0)])   # rejected on its size alone
    assert e.value.status == 10
    assert srv.GetBgVersion(100) == -1                        # nothing accepted
