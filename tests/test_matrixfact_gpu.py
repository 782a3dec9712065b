"""C1 (BASELINE.json configs[0]): the matrixfact_split App-API driver
(examples/matrixfact/matrixfact_split.cpp, written against include/petuum_ps_common and
linked to libpetuum_ps.so + libpsx.so) runs SGD matrix factorization with 2 worker
threads on a synthetic 2K x 1K, 10K-nonzero split in the data_split binary format.

The runtime records (PSX_TRACE_DIR) every ClientSendOpLogMsg it hands a server shard,
every row request and its reply, and every push body the shard returns.  The test replays
the same messages and requests through parameter_server_amd.ServerThread over the CPU
oracle and requires every reply and every push body, every clock, to be byte-identical
to what the GPU shards produced; and the driver's own loss must fall.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from parameter_server_amd import wire, ServerThread
from oracle.oracle import DENSE, F32
from oracle_backend import OracleBackend

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "bin", "matrixfact_split")


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(BIN):
        pytest.fail("examples/bin/matrixfact_split not built (run __graft_entry__.build())")


def write_split(prefix, rows=2000, cols=1000, nnz=10000, rank=4, seed=1234):
    """data_split.cpp:200-217's partition file <prefix>.0: size_t nnz, rows, cols; int rows[];
    int cols[]; float vals[] grouped by row.  Values are a rank-4 product plus noise."""
    rng = np.random.RandomState(seed)
    flat = np.sort(rng.choice(rows * cols, nnz, replace=False))
    r, c = (flat // cols).astype(np.int32), (flat % cols).astype(np.int32)
    U = rng.normal(0, 0.7, (rows, rank))
    V = rng.normal(0, 0.7, (cols, rank))
    v = ((U[r] * V[c]).sum(1) + rng.normal(0, 0.05, nnz)).astype(np.float32)
    with open(prefix + ".0", "wb") as f:
        f.write(struct.pack("<QQQ", nnz, rows, cols))
        f.write(r.tobytes())
        f.write(c.tobytes())
        f.write(v.tobytes())


def run_driver(tmp_path, channels, staleness, iters=4, K=16, threads=2, extra=()):
    data = str(tmp_path / "mf.bin")
    write_split(data)
    trace = tmp_path / "trace"
    trace.mkdir()
    env = dict(os.environ, PSX_TRACE_DIR=str(trace))
    cmd = [BIN, "--datafile", data, "--K", str(K), "--num_worker_threads", str(threads),
           "--num_iterations", str(iters), "--num_comm_channels_per_client", str(channels),
           "--table_staleness", str(staleness), "--init_step_size", "0.05", "--use_step_dec", "true",
           "--step_dec", "0.995", "--lambda", "0.05", "--nnz_per_row", "5", "--nnz_per_col", "10",
           "--M_cache_size", "1000", *extra]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    losses = [list(map(float, ln.split()[1:])) for ln in p.stdout.splitlines() if ln.startswith("LOSS ")]
    return trace, losses


def replay(trace, channels, K, r_dense_serialized=True):
    """Drive one oracle ServerThread per shard with the recorded events, comparing outputs."""
    events = [ln.split() for ln in open(trace / "index.txt").read().splitlines()]
    threads, got_push, want_push, got_reply, want_reply = [], [], [], [], []
    for ch in range(channels):
        be = OracleBackend([100 + ch], num_clients=1)
        be.create(1, DENSE, F32, K, dense_serialized=r_dense_serialized)
        be.create(2, DENSE, F32, 6)
        want_push.append([])
        want_reply.append([])
        got_push.append([])
        got_reply.append([])
        threads.append(ServerThread(
            be, push=lambda bodies, clock, ch=ch: want_push[ch].append(bodies[0]),
            reply=lambda bg, t, r, clock, rec, ch=ch: want_reply[ch].append(rec)))
    counts = {"msg": 0, "push": 0, "req": 0, "reply": 0}
    for kind, ch, seq, name in events:
        ch = int(ch)
        data = (trace / name).read_bytes()
        counts[kind] += 1
        if kind == "msg":
            h, payload = wire.decode_oplog_msg(np.frombuffer(data, np.uint8))
            assert h["client_id"] == 0 and h["is_clock"] == 1
            threads[ch].HandleOpLogMsg(100 + ch, payload, True, h["bg_clock"], h["version"])
        elif kind == "req":
            tid, row = struct.unpack("<ii", data)
            assert threads[ch].HandleRowRequest(100 + ch, tid, row, 0)
        elif kind == "reply":
            got_reply[ch].append(data)
        else:
            got_push[ch].append(data)
    for ch in range(channels):
        assert len(got_reply[ch]) == len(want_reply[ch])
        for i, (g, w) in enumerate(zip(got_reply[ch], want_reply[ch])):
            assert g == w, f"shard {ch} reply {i} differs"
        assert len(got_push[ch]) == len(want_push[ch]), (len(got_push[ch]), len(want_push[ch]))
        for i, (g, w) in enumerate(zip(got_push[ch], want_push[ch])):
            assert g == w, f"shard {ch} push {i} differs"
    return counts


@pytest.mark.parametrize("channels,staleness", [(1, 0), (2, 2)])
def test_c1_matrixfact_pushes_match_oracle_every_clock(tmp_path, channels, staleness):
    iters, K = 4, 16
    trace, losses = run_driver(tmp_path, channels, staleness, iters=iters, K=K)
    counts = replay(trace, channels, K)
    # init barrier (s+1) + bootstrap barrier (s+1) + iters + final barrier (s+1) process clocks, per shard
    assert counts["msg"] == channels * (3 * (staleness + 1) + iters)
    assert counts["push"] == counts["msg"]          # one client: every clock message moves the min clock
    assert counts["req"] == counts["reply"] > 0
    assert len(losses) == iters
    l2 = [l[4] for l in losses]
    assert l2[-1] < l2[0], l2


def test_c1_sparse_oplog_sparse_serialized(tmp_path):
    """row_oplog_type 1 (SparseRowOpLog) on a sparse-serialized R table, no_oplog_replay:
    the shards receive {n, cols, vals} records for dense rows (zeros dropped)."""
    trace, losses = run_driver(tmp_path, 1, 1, iters=3, extra=("--row_oplog_type", "1", "--oplog_dense_serialized",
                                                               "false", "--no_oplog_replay", "true"))
    replay(trace, 1, 16, r_dense_serialized=False)
    assert len(losses) == 3
