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
    assert built_lib.psx_abi_version() == 9
    assert built_lib.psx_status_string(0) == b"ok"
    assert built_lib.psx_status_string(2) == b"version gap"


def test_null_context_is_rejected(built_lib):
    assert built_lib.psx_sync(None) == 1
    assert built_lib.psx_apply_stream(None, None, 0, 0, 0) == 1
    assert built_lib.psx_last_error(None) == b"null context"


def test_library_is_gfx950_code_object(built_lib):
    """The shared object carries gfx950 offload bundles only (no other GPU target).
    (rocPRIM's host-side dispatch tables name other architectures as strings; only the
    bundle ids say which code objects are inside.)"""
    import re
    data = open(_abi.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-+(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets
    assert b"nvptx" not in data


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


def test_table_config_layout_matches_header(tmp_path):
    """ctypes psx_table_config / psx_stream mirror the C structs: compile a probe against
    include/psx.h with gcc and compare sizeof/offsetof."""
    import subprocess
    inc = os.path.dirname(_abi.HEADER_PATH)
    src = tmp_path / "probe.c"
    src.write_text("""#include <stdio.h>
#include <stddef.h>
#include "psx.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(psx_table_config), offsetof(psx_table_config, max_entries),
         offsetof(psx_table_config, accum_importance), offsetof(psx_table_config, server_push_row_upper_bound),
         sizeof(psx_stream), offsetof(psx_table_config, version_maintain), offsetof(psx_table_config, row_oplog_type));
  return 0;
}
""")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    c = _abi.psx_table_config
    want = [ctypes.sizeof(c), c.max_entries.offset, c.accum_importance.offset,
            c.server_push_row_upper_bound.offset, ctypes.sizeof(_abi.psx_stream), c.version_maintain.offset,
            c.row_oplog_type.offset]
    assert got == want
