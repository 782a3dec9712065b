import numpy as np, torch
import parameter_server_amd as psa
from parameter_server_amd import wire
from oracle.oracle import OracleServer, DENSE, F32
for cap in (4, 64, 256, 300, 1024):
    for B in (1, 2, 3):
        for pattern in ("ones", "rand"):
            rows = 64
            srv = psa.Server(0, 1, list(range(B)))
            srv.CreateTable(1, psa.TableInfo(row_kind=DENSE, dtype=F32, row_capacity=cap, max_rows=rows, accum_importance=True))
            orc = OracleServer(list(range(B))); orc.create_table(1, DENSE, F32, cap, accum_importance=True)
            rng = np.random.RandomState(1)
            init = np.ones((rows, cap), np.float32) * 2 if pattern == "ones" else rng.normal(size=(rows, cap)).astype(np.float32)
            srv.load_rows(1, 0, init); orc.load_dense_rows(1, 0, init)
            st = []
            for b in range(B):
                ids = np.arange(rows, dtype=np.int32)[b::1]
                u = np.ones((ids.size, cap), np.float32) if pattern == "ones" else rng.normal(size=(ids.size, cap)).astype(np.float32)
                st.append(wire.dense_stream_np(1, ids, u))
            dev = [torch.from_numpy(s).cuda() for s in st]
            srv.apply_device([(d.data_ptr(), d.numel(), b, 0) for b, d in enumerate(dev)]); srv.sync()
            for b, s in enumerate(st): orc.apply_stream(s, b, 0)
            got = srv.row_importance(1, 0, rows); want = np.array([orc.importance(1, r) for r in range(rows)])
            print(cap, B, pattern, "ok" if np.allclose(got, want, rtol=1e-12) else "BAD", got[:3], want[:3])
            srv.close()
