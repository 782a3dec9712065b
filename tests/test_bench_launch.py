"""bench.py --gpus N launches its own N ranks (no external launcher): the harness run
over gloo on the CPU with a no-op step reports n_gpus = N (the GPU runs of the same
harness are the driver's SCALE records)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                          "--warmup", "1", "--selftest-launch", "--master-port", "29533"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3


def _selftest_exchange(extra, port, world=2):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2",
                          "--warmup", "1", "--selftest-exchange", "--master-port", str(port)] + extra,
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world,port", [(2, 29535), (8, 29537)])
def test_exchange_extra_orchestration_and_parity_over_gloo(world, port):
    """The N > 1 exchange extras' code path (exchange_measure: chunked batches spanning every
    shard, split by owner, all-to-all, in-order apply, then every owner's shard checked bit
    for bit against the seeds) at world 2 and at the driver's largest, 8, over gloo, with the
    CPU stand-in of the device split/apply."""
    rec = _selftest_exchange([], port, world)
    assert rec["n_gpus"] == world and rec["parity"] == "bit-exact"
    assert rec["chunks_per_step"] > 1
    assert rec["config"]["shard_rows"] * world == 4096 * world
    # the transport's own view of the run: every rank's communicator size and
    # rank, and the bytes it moved to / from each peer over the timed steps
    comm = rec["comm"]
    assert comm["all_ranks_see_world"] is True and len(comm["ranks"]) == world
    for i, r in enumerate(comm["ranks"]):
        assert r["nranks"] == world and r["rank"] == i
        for k in ("device", "rccl_version", "librccl"):
            assert k in r
        assert len(r["sent_bytes_per_peer"]) == world and len(r["recv_bytes_per_peer"]) == world
        assert r["sent_bytes_per_peer"][i] == 0 and sum(r["sent_bytes_per_peer"]) > 0
    # what every rank sent to p is what p received from it
    for i in range(world):
        for p in range(world):
            assert comm["ranks"][i]["sent_bytes_per_peer"][p] == comm["ranks"][p]["recv_bytes_per_peer"][i]
    assert comm["crossed_bytes_per_step_all_ranks"] > 0


def test_exchange_parity_check_catches_a_reordered_apply():
    """Applying the sources in reverse rank order changes the f32 sums: the check reports it."""
    rec = _selftest_exchange(["--selftest-reverse"], 29536)
    assert rec["parity"] != "bit-exact" and rec["parity"].endswith("values differ")
