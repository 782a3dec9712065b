"""CPU tests of the C-ABI library: it loads and exports every symbol include/psx.h
declares.  No compute calls are made without a GPU."""
import ctypes
import os

from parameter_server_amd import _abi


def test_lib_exports_every_header_symbol(built_lib):
    names = _abi.header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(built_lib, n)]
    assert not missing, missing


def test_abi_version_and_status_strings(built_lib):
    assert built_lib.psx_abi_version() == 1
    assert built_lib.psx_status_string(0) == b"ok"
    assert built_lib.psx_status_string(2) == b"version gap"


def test_null_context_is_rejected(built_lib):
    assert built_lib.psx_sync(None) == 1
    assert built_lib.psx_apply_stream(None, None, 0, 0, 0) == 1
    assert built_lib.psx_last_error(None) == b"null context"


def test_library_is_gfx950_code_object(built_lib):
    """The shared object carries a gfx950 offload bundle (no other GPU target)."""
    data = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert other not in data


def test_product_does_not_import_oracle():
    """The product path never imports, links or loads the CPU oracle."""
    import re
    pkg = os.path.dirname(_abi.__file__)
    pat = re.compile(r"^\s*(from\s+oracle|import\s+oracle)|psx_oracle|libpsx_oracle|#include\s*\"[^\"]*oracle",
                     re.M)
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", "Makefile")) or f == "Makefile":
                src = open(os.path.join(root, f)).read()
                assert not pat.search(src), f
    assert b"orc_" not in open(_abi.LIB_PATH, "rb").read()
