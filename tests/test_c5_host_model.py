"""bench.c5_host_model — the numpy replay behind the C5 line's parity field (no libpsx, no
oracle in the bench) — pinned here against the CPU oracle on a shard of the real C5
workload: the same arrival-ordered per-owner messages give the same dense rows bit for bit
and the same {col -> value} sorted-map rows; and the last push's dirty rows are the rows the
oracle's push serializes (ServerTable::AppendTableToBuffs, server_table.cpp:197-261)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c5_host_model_matches_the_oracle(oracle_lib):
    sys.path.insert(0, ROOT)
    import bench
    from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, I32
    from parameter_server_amd import wire
    wl = bench.c5_workload()
    B = wl["B"]
    arrivals, _ = bench.c5_schedule(B, 6)
    runs, cur = [], []
    for w, c, push in arrivals:
        cur.append((w, c))
        if push or len(cur) == 16:
            runs.append((cur, push))
            cur = []
    # the last run of the replay ends with a push
    upto = max(j for j, (_, p) in enumerate(runs) if p) + 1
    d_lo, d_hi, s_lo, s_hi = 1000, 9000, 200, 3200
    tab, cntm, (dirty_d, dirty_s) = bench.c5_host_model(wl, runs, upto, d_lo, d_hi, s_lo, s_hi)
    bgs = [100 + b for b in range(B)]
    msgs = []
    for ids_d, upd, ids_s, cnt in wl["parts"]:
        md, ms = (ids_d >= d_lo) & (ids_d < d_hi), (ids_s >= s_lo) & (ids_s < s_hi)
        msgs.append(wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=ids_d[md], oplogs=upd[md]),
                                  dict(table_id=3, dense_serialized=False, row_ids=ids_s[ms], oplogs=cnt[ms])]))
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, wl["cap"])
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    ver = [0] * B
    body = b""
    for j in range(upto):
        group, push = runs[j]
        for w, _ in group:
            assert orc.apply_stream(msgs[w], bgs[w], ver[w]) == 0
            ver[w] += 1
        if push:
            body = orc.serialize_dirty([1, 3], clear=True)
    assert np.array_equal(orc.read_dense_rows(1, d_lo, d_hi - d_lo).view(np.uint32), tab.view(np.uint32))
    got_s = bench.c5_parse_rows(orc.serialize_records(3, list(range(s_lo, s_hi))), s_lo, s_hi - s_lo, wl["K"])
    assert np.array_equal(got_s, cntm)
    parsed = wire.parse_push_body(body)
    assert sorted(r - d_lo for r in parsed.get(1, {})) == sorted(dirty_d.tolist())
    assert sorted(r - s_lo for r in parsed.get(3, {})) == sorted(dirty_s.tolist())
    orc.close()
