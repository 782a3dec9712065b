"""ISA checks of the shipped kernels (CPU: the gfx950 code object is disassembled, no GPU).

dense_apply_v3 addresses records as a wave-uniform 64-bit base plus a 32-bit UNSIGNED
per-lane byte offset (psx_kernels.hip gload16 / gload_h4), which is what lets it reach
records up to 4 GiB into a message (round 5's fault came from a removed
variant whose 32-bit record address was sign-extended).  A sign-extended per-lane offset
would show as a v_ashrrev_i32 by 31 in the kernel; there must be none in any of v3's
instantiations.  tests/test_configs_gpu.py::test_v3_message_between_2_and_4_gib_bit_exact
runs such offsets (bit 31 set) on the GPU."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "parameter_server_amd", "csrc", "build", "psx_kernels.hip.o")
LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.fixture(scope="module")
def kernels_isa(built_lib, tmp_path_factory):
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("no ROCm LLVM tools")
    d = tmp_path_factory.mktemp("isa")
    fat, co = str(d / "fat.bin"), str(d / "k.co")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", OBJ, str(d / "x.o")],
                   check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                       capture_output=True, text=True)
    return r.stdout


def _functions(isa, pattern):
    out, name, body = {}, None, []
    for line in isa.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            if name and re.search(pattern, name):
                out[name] = body
            name, body = m.group(1), []
        elif name:
            body.append(line)
    if name and re.search(pattern, name):
        out[name] = body
    return out


def test_v3_per_lane_record_offsets_are_never_sign_extended(kernels_isa):
    fns = _functions(kernels_isa, r"dense_apply_v3_kernel")
    assert len(fns) >= 20, sorted(fns)            # f32/f64/i32/i64 x batch widths, binary16 records
    bad = {n: [l.strip() for l in body if "v_ashrrev_i32" in l] for n, body in fns.items()}
    bad = {n: v for n, v in bad.items() if v}
    assert not bad, bad
    # and the record loads really take 64-bit addresses built from them
    for n, body in fns.items():
        assert any("global_load_dwordx" in l for l in body), n
