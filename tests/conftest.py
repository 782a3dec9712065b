import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpsx.so on cuda:0)")


@pytest.fixture(scope="session")
def built_lib():
    """libpsx.so built in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-j4", "-C", os.path.join(ROOT, "parameter_server_amd", "csrc")],
                   check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], check=True)
    from parameter_server_amd import _abi
    return _abi.load()


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle.lib()
