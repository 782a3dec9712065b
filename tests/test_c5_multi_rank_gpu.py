"""C5 (BASELINE configs[4]: mixed dense + sparse tables under SSPPush with
staleness 4) sharded over two ranks sharing one GPU — the N-rank form the bare
`bench.py --gpus N` line now runs.  Each rank serves its row range of both tables from the
workers' per-owner messages, in the SSP arrival order (bench.c5_schedule), with no
collective on the data path (gloo only for the barrier and the timing reductions here).

Every rank's shard is checked against the CPU oracle (oracle/psx_oracle.c, the restated
Server::ApplyOpLogUpdateVersion, server.cpp:120-179) replaying the same per-owner messages
in the order the rank applied them: dense rows bit for bit, sorted-map rows byte for byte
(entry order included, sorted_vector_map_store.hpp:305-337); and the bench's own parity field
(a numpy replay, no libpsx, no oracle) must say bit-exact."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_c5_two_ranks_on_one_gpu_match_the_oracle(tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, I32
    from parameter_server_amd import wire
    world = 2
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--workload", "c5", "--c5-gloo", "--c5-dump", str(tmp_path), "--steps", "3", "--warmup", "1",
           "--cpu-seconds", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == world and line["steps"] == 3
    assert line["parity"]["result"] == "bit-exact", line["parity"]

    wl = bench.c5_workload()
    bgs = [100 + b for b in range(wl["B"])]
    for rank in range(world):
        d = np.load(tmp_path / f"c5_rank{rank}.npz")
        d_lo, d_hi, s_lo, s_hi = (int(x) for x in d["bounds"])
        msgs = []
        for ids_d, upd, ids_s, cnt in wl["parts"]:
            md, ms = (ids_d >= d_lo) & (ids_d < d_hi), (ids_s >= s_lo) & (ids_s < s_hi)
            msgs.append(wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=ids_d[md], oplogs=upd[md]),
                                      dict(table_id=3, dense_serialized=False, row_ids=ids_s[ms], oplogs=cnt[ms])]))
        orc = OracleServer(bgs)
        orc.create_table(1, DENSE, F32, wl["cap"])
        orc.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
        ver = [0] * wl["B"]
        assert len(d["order"]) > 3 * wl["B"]
        for w, _c in d["order"]:
            assert orc.apply_stream(msgs[w], bgs[w], ver[w]) == 0
            ver[w] += 1
        want_d = orc.read_dense_rows(1, d_lo, d_hi - d_lo)
        assert np.array_equal(d["dense"].view(np.uint32), want_d.view(np.uint32)), f"rank {rank} dense rows"
        want_s = orc.serialize_records(3, list(range(s_lo, s_hi)))
        assert d["sparse"].tobytes() == want_s, f"rank {rank} sorted-map rows"
        orc.close()
