"""The three other App-API callers north_star names, run as C++ programs built against
include/petuum_ps_common (+ include/petuum_ps/server for the logic) and linked to
libpetuum_ps.so + libpsx.so, each replayed message by message through the CPU oracle:

  lda_gibbs               apps/lda's tables: SortedVectorMapRow<int32> word-topic rows
                          (±1 BatchInc per reassignment, lda_engine.cpp:57-76,
                          fast_doc_sampler.cpp:164-174), a DenseRow<int32> summary row and a
                          DenseRow<double> llh table, sparse-serialized (run_lda.sh:82-83)
  mlr_sgd                 apps/mlr's W table: DenseRow<float> of feature_dim per label,
                          DenseBatchInc per label and Get of every row per refresh
                          (mlr_sgd_solver.cpp:66-95); synthetic data, and the reference's own
                          covtype.scale.train.small (libsvm)
  matrixfact_adarevision  apps/matrixfact's AdaRevision build: R's table registers
                          AdaRevisionServerTableLogic as server_table_logic 1 with
                          version_maintain (matrixfact_adarevision.cpp:633-635,
                          run_matrixfact_adarevision.sh:113-116)

The runtime records (PSX_TRACE_DIR) every ClientSendOpLogMsg it hands a shard (clock
messages and, for version tables, the end-of-version messages a push produces), every row
request and reply and every push body; tests/app_replay.py replays them through an oracle
ServerThread per shard and requires every reply and push body to be byte-identical."""
import os
import struct
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle.oracle import DENSE, SORTED_MAP, F32, F64, I32
from app_replay import replay

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "bin")


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    for b in ("lda_gibbs", "mlr_sgd", "matrixfact_adarevision"):
        if not os.path.exists(os.path.join(BIN, b)):
            pytest.fail(f"examples/bin/{b} not built (run __graft_entry__.build())")


def run(tmp_path, prog, args):
    trace = tmp_path / "trace"
    trace.mkdir()
    env = dict(os.environ, PSX_TRACE_DIR=str(trace))
    p = subprocess.run([os.path.join(BIN, prog)] + [str(a) for a in args], env=env, capture_output=True, text=True,
                       timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    return trace, p.stdout


@pytest.mark.parametrize("channels,staleness", [(1, 0), (2, 1)])
def test_lda_word_topic_rows_match_oracle_every_clock(tmp_path, channels, staleness):
    K, iters = 16, 3
    trace, out = run(tmp_path, "lda_gibbs", ["--num_docs", 200, "--vocab", 600, "--num_topics", K, "--doc_len", 40,
                                             "--num_worker_threads", 2, "--num_iterations", iters,
                                             "--num_comm_channels_per_client", channels,
                                             "--table_staleness", staleness])
    counts = replay(trace, channels, [
        dict(tid=1, kind=SORTED_MAP, dtype=I32, cap=K, dense_serialized=False),
        dict(tid=2, kind=DENSE, dtype=I32, cap=K, dense_serialized=False),
        dict(tid=3, kind=DENSE, dtype=F64, cap=3, dense_serialized=False)])
    assert counts["req"] == counts["reply"] > 0 and counts["push"] > 0
    llh = [float(ln.split()[2]) for ln in out.splitlines() if ln.startswith("LLH ")]
    assert len(llh) == iters and llh[-1] > llh[0], llh
    # every token is counted once in the summary row
    tokens = int(next(ln for ln in out.splitlines() if ln.startswith("WORDLLH")).split()[3])
    assert tokens > 200 * 20


@pytest.mark.parametrize("channels,staleness", [(1, 0), (3, 2)])
def test_mlr_weight_rows_match_oracle_every_clock(tmp_path, channels, staleness):
    D, L, epochs = 256, 6, 4
    trace, out = run(tmp_path, "mlr_sgd", ["--num_labels", L, "--feature_dim", D, "--num_train", 1200,
                                           "--num_worker_threads", 2, "--num_epochs", epochs, "--batch_size", 60,
                                           "--num_comm_channels_per_client", channels, "--table_staleness", staleness])
    counts = replay(trace, channels, [dict(tid=0, kind=DENSE, dtype=F32, cap=D),
                                      dict(tid=1, kind=DENSE, dtype=F32, cap=3)])
    assert counts["push"] > 0
    rows = [list(map(float, ln.split()[1:])) for ln in out.splitlines() if ln.startswith("LOSS ")]
    assert len(rows) == epochs
    # rows: {epoch, mean loss, accuracy}
    assert rows[-1][1] < rows[0][1] and rows[-1][2] > 2.0 / L, rows


@pytest.mark.parametrize("channels,staleness", [(1, 0), (2, 2)])
def test_mlr_on_the_reference_covtype_data(tmp_path, channels, staleness):
    """apps/mlr's shipped dataset (apps/mlr/datasets/covtype.scale.train.small + .meta,
    libsvm, 500 rows, feature_dim 54, 7 labels, one-based; kept as a data fixture under
    tests/golden/mlr): the driver reads it as ReadDataLabelLibSVM does, trains W (7 rows of 54)
    and every message, reply and push is replayed through the oracle byte for byte."""
    data = os.path.join(ROOT, "tests", "golden", "mlr", "covtype.scale.train.small")
    epochs = 5
    trace, out = run(tmp_path, "mlr_sgd", ["--train_file", data, "--num_worker_threads", 2, "--num_epochs", epochs,
                                           "--batch_size", 25, "--learning_rate", 0.1, "--decay_rate", 0.95,
                                           "--num_comm_channels_per_client", channels, "--table_staleness", staleness])
    assert "DATA 500 54 7" in out
    counts = replay(trace, channels, [dict(tid=0, kind=DENSE, dtype=F32, cap=54),
                                      dict(tid=1, kind=DENSE, dtype=F32, cap=3)])
    assert counts["push"] > 0 and counts["msg"] > 0
    rows = [list(map(float, ln.split()[1:])) for ln in out.splitlines() if ln.startswith("LOSS ")]
    assert len(rows) == epochs
    assert rows[-1][1] < rows[0][1], rows          # mean cross-entropy falls
    assert rows[-1][2] > 1.0 / 7, rows              # better than chance


def _write_split(prefix, rows=600, cols=300, nnz=4000, seed=77):
    rng = np.random.RandomState(seed)
    flat = np.sort(rng.choice(rows * cols, nnz, replace=False))
    r, c = (flat // cols).astype(np.int32), (flat % cols).astype(np.int32)
    U, V = rng.normal(0, 0.7, (rows, 3)), rng.normal(0, 0.7, (cols, 3))
    v = ((U[r] * V[c]).sum(1) + rng.normal(0, 0.05, nnz)).astype(np.float32)
    with open(prefix + ".0", "wb") as f:
        f.write(struct.pack("<QQQ", nnz, rows, cols))
        f.write(r.tobytes())
        f.write(c.tobytes())
        f.write(v.tobytes())


@pytest.mark.parametrize("channels", [1, 2])
def test_matrixfact_adarevision_logic_matches_oracle_every_clock(tmp_path, channels):
    """The registered AdaRevisionServerTableLogic selects libpsx's device logic: rows created
    with the logic's N(0, 0.1) draws, version records, snapshots per (row, version), the
    end-of-version records a push produces — every reply and push body as the oracle's."""
    K, iters, step = 8, 3, 0.05
    data = str(tmp_path / "mf.bin")
    _write_split(data)
    trace, out = run(tmp_path, "matrixfact_adarevision",
                     ["--datafile", data, "--K", K, "--num_worker_threads", 2, "--num_iterations", iters,
                      "--num_comm_channels_per_client", channels, "--table_staleness", 0, "--init_step_size", step,
                      "--lambda", 0.05, "--nnz_per_row", 5, "--nnz_per_col", 10, "--M_cache_size", 300])
    counts = replay(trace, channels, [
        dict(tid=1, kind=DENSE, dtype=F32, cap=K, version_maintain=True,
             adarevision=dict(init_step_size=step, gaussian_init=True, old_grad_upper_bound=10000)),
        dict(tid=2, kind=DENSE, dtype=F32, cap=6)])
    assert counts["msg"] > counts["clock_msg"] > 0, counts   # end-of-version messages went out
    losses = [list(map(float, ln.split()[1:])) for ln in out.splitlines() if ln.startswith("LOSS ")]
    assert len(losses) == iters
    assert losses[-1][4] < losses[0][4], losses


def test_unregistered_or_host_only_logic_fails_loudly(tmp_path):
    """server_table_logic naming nothing registered stops CreateTable with a message (the
    reference CHECKs, server_table.cpp:87-88)."""
    data = str(tmp_path / "mf.bin")
    _write_split(data)
    p = subprocess.run([os.path.join(BIN, "matrixfact_adarevision"), "--datafile", data, "--K", "8",
                        "--num_iterations", "1", "--M_cache_size", "300", "--server_table_logic", "7"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "server table logic 7 not registered" in p.stderr
