"""Run by tests/test_env_knobs.py in a child process whose environment sets every PSX_*
variable the A/B (debug) build of libpsx reads.  The shipped libpsx.so must ignore them:
a split sorted-map table (max_entries 1,024 > 256: the register apply the timing probes
cut) and a dense table, applied through the walked and the pipelined paths, must equal
the oracle byte for byte.  Prints "env-knobs ok" on success."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import parameter_server_amd as psa  # noqa: E402
from parameter_server_amd import wire  # noqa: E402
from oracle.oracle import OracleServer, SORTED_MAP, DENSE, I32, F32  # noqa: E402


def main():
    rng = np.random.RandomState(11)
    rows, K, B, cap = 4000, 1024, 6, 64
    bgs = list(range(100, 100 + B))
    srv = psa.Server(0, 1, bgs)
    orc = OracleServer(bgs)
    srv.CreateTable(3, psa.TableInfo(row_kind=SORTED_MAP, dtype=I32, row_capacity=K, oplog_dense_serialized=False,
                                     max_rows=rows, max_entries=K))
    orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    srv.CreateTable(4, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    orc.create_table(4, DENSE, F32, cap)
    for rnd in range(2):
        streams = []
        for b in range(B):
            recs = []
            for rid in rng.choice(rows, size=300, replace=False):
                k = rng.randint(1, 40)
                cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
                v = rng.randint(1, 4, size=k) * (1 if (rnd == 0 and b == 0) else rng.choice([-1, 1], size=k))
                recs.append((int(rid), cols, v.astype(np.int32)))
            streams.append(wire.sparse_stream_np(3, 4, recs))
            ids = rng.permutation(rows)[:500].astype(np.int32)
            streams.append(wire.dense_stream_np(4, ids, rng.normal(0, 1, size=(500, cap)).astype(np.float32)))
        # one message per (worker, table) pair: B senders, two messages each -> versions 2*rnd, 2*rnd+1
        for half in range(2):
            msgs = [streams[2 * b + half] for b in range(B)]
            dev = [torch.from_numpy(np.array(m, copy=True)).cuda() for m in msgs]
            torch.cuda.synchronize()
            srv.apply_device([(d.data_ptr(), d.numel(), bg, 2 * rnd + half) for d, bg in zip(dev, bgs)])
            srv.sync()
            for m, bg in zip(msgs, bgs):
                assert orc.apply_stream(m, bg, 2 * rnd + half) == 0
    ids = list(range(rows))
    got = srv.serialize_rows(3, ids)
    want = orc.serialize_records(3, ids)
    assert got == want, "sorted-map rows differ from the oracle"
    g = srv.read_rows(4, 0, rows)
    w = orc.read_dense_rows(4, 0, rows)
    assert np.array_equal(g.view(np.uint32), w.view(np.uint32)), "dense rows differ from the oracle"
    srv.close()
    print("env-knobs ok")


if __name__ == "__main__":
    main()
