"""C1 (BASELINE.json configs[0]): matrixfact_split with 2 local workers on one client,
tiny synthetic split, through the server interface (examples/matrixfact_split.py).

CPU: the driver against the CPU checker — the loss falls clock by clock.
GPU: the same run against the MI355X server; every clock's ClientSendOpLogMsg is also
applied by the checker, and the push bodies (every dirty R row, server.cpp:189-309) must
be byte-identical (row values bit-exact: per-row update order is the reference's)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples"))

import matrixfact_split as mf  # noqa: E402
from oracle.oracle import OracleServer, DENSE, F32  # noqa: E402

K, COLS = 16, 1000


class CheckerServer:
    def __init__(self):
        self.o = OracleServer([0])
        self.o.create_table(1, DENSE, F32, K)

    def ApplyOpLogUpdateVersion(self, msg, size, bg, version):
        assert self.o.apply_stream(msg, bg, version) == 0

    def push_body(self):
        return self.o.serialize_dirty([1], clear=True)


@pytest.fixture(scope="module")
def split(tmp_path_factory):
    return mf.write_split(str(tmp_path_factory.mktemp("c1") / "mf.0"))


def test_split_format_round_trip(split):
    r, c, v, rows, cols = mf.read_split(split)
    assert (rows, cols, r.size) == (2000, 1000, 10000)
    assert np.all(np.diff(r) >= 0) and v.min() >= 1 and v.max() <= 5
    starts = mf.partition_workload(r, 2)
    assert starts[0] == 0 and r[starts[1] - 1] != r[starts[1]]


def test_c1_loss_falls_on_cpu_checker(split, oracle_lib):
    out = mf.run(CheckerServer(), split, k=K, iters=3)
    losses = [o[0] for o in out]
    assert losses[0] > losses[1] > losses[2]
    assert all(len(o[2]) > 0 for o in out)


@pytest.mark.gpu
def test_c1_gpu_server_matches_checker_every_clock(split, built_lib, oracle_lib):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import parameter_server_amd as psa

    class Both:
        """Applies each message on the GPU server and the checker; returns the GPU body
        after checking it against the checker's."""

        def __init__(self):
            self.g = psa.Server(0, 1, [0])
            self.g.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=K,
                                                max_rows=COLS))
            self.c = CheckerServer()
            self.clocks = 0

        def ApplyOpLogUpdateVersion(self, msg, size, bg, version):
            self.g.ApplyOpLogUpdateVersion(msg, size, bg, version)
            self.c.ApplyOpLogUpdateVersion(msg, size, bg, version)

        def push_body(self):
            got = bytes(self.g.serialize_dirty(clear=True))
            assert got == self.c.push_body(), f"push body differs at clock {self.clocks}"
            self.clocks += 1
            return got

    both = Both()
    out = mf.run(both, split, k=K, iters=3)
    assert both.clocks == 4
    losses = [o[0] for o in out]
    assert losses[0] > losses[1] > losses[2]
