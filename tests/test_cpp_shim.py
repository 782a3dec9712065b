"""The C++ host mirror (include/psx_server.hpp) compiles and links against libpsx.so
(CPU), and on the GPU it reproduces the oracle's result for the same message sequence."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def _build(built_lib):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, "build", "psx_server_demo")


def test_cpp_mirror_builds(built_lib):
    assert os.path.exists(_build(built_lib))


@pytest.mark.gpu
def test_cpp_mirror_matches_oracle(built_lib, oracle_lib, tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.oracle import OracleServer, DENSE, F32
    from parameter_server_amd import wire
    exe = _build(built_lib)
    out = tmp_path / "rows.bin"
    r = subprocess.run([exe, str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows, cap = 64, 16
    orc = OracleServer([100, 101])
    orc.create_table(5, DENSE, F32, cap)
    for msg in range(4):
        seen = []
        for rr in range(msg, rows, 3):
            x = (rr * 5 + msg) % rows
            if x not in seen:
                seen.append(x)
        ids = np.array(seen, np.int32)
        vals = np.array([[((x * 31 + c * 7 + msg * 13) % 17 - 8) * 0.25 for c in range(cap)] for x in seen],
                        np.float32)
        assert orc.apply_stream(wire.dense_stream_np(5, ids, vals), 100 + (msg & 1), msg >> 1) == 0
    assert out.read_bytes() == orc.serialize_records(5, list(range(rows)))
    assert "versions 1 1" in r.stdout


def test_cpp_exchange_selftest_builds(built_lib):
    _build(built_lib)
    assert os.path.exists(os.path.join(CPP, "build", "psx_exchange_selftest"))


@pytest.mark.gpu
def test_cpp_exchange_past_2gib_on_the_images_rccl(built_lib):
    """libpsx's exchange from a process without torch (tests/cpp/psx_exchange_selftest.cpp):
    libpsx's -lrccl then loads the ROCm image's RCCL, not torch's copy; a 2 GiB + 12 KiB
    sub-stream, sent in 512 MiB pieces (psx_exchange.cpp), must arrive intact there too."""
    import json
    _build(built_lib)
    exe = os.path.join(CPP, "build", "psx_exchange_selftest")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    info = lines[-1]
    assert info["differing_words"] == 0 and info["bytes"] == (2 << 30) + (12 << 10)
    assert info["rccl"].startswith("/opt/rocm"), info["rccl"]
    # psx_comm_info: RCCL's own view of the communicator (ncclCommCount / UserRank /
    # CuDevice / GetVersion) and the librccl the process loaded
    comm = lines[0]
    assert comm["comm_nranks"] == 1 and comm["comm_rank"] == 0 and comm["comm_device"] == 0, comm
    assert comm["comm_librccl"] == info["rccl"] and comm["rccl_version"] > 20000, comm
    print(comm, info)
