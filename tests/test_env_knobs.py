"""No result-changing environment knobs in the shipped library.

The kernel selectors' PSX_* environment overrides and the ordered apply's timing probes
(PSX_DEBUG_ORD_PROBE: "results wrong") exist only in the A/B build, libpsx_debug.so
(`make -C parameter_server_amd/csrc debug`).  libpsx.so reads none of those variables and
refuses the probe selector, so a stray variable in a user's environment cannot change an
apply — the reference applies one way (server.cpp:120-179)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "parameter_server_amd", "libpsx.so")
KNOBS = ("PSX_ORD_PROBE", "PSX_PIPELINE", "PSX_APPLY_VARIANT", "PSX_ORD_SPLIT", "PSX_ORD_LITE",
         "PSX_DECODE_WALK", "PSX_DENSE_STORE_NT", "PSX_WALK_CUS", "PSX_WALK_COUNT", "PSX_FOLD_FINISH",
         "PSX_WALK_LEVELS", "PSX_WALK_SHAPE")
# values that, read by the debug build, change kernels — PSX_ORD_PROBE=7 makes results wrong
KNOB_ENV = {"PSX_ORD_PROBE": "7", "PSX_PIPELINE": "2", "PSX_APPLY_VARIANT": "2", "PSX_ORD_SPLIT": "0",
            "PSX_ORD_LITE": "1", "PSX_DECODE_WALK": "0", "PSX_DENSE_STORE_NT": "3", "PSX_WALK_CUS": "0",
            "PSX_WALK_COUNT": "0", "PSX_FOLD_FINISH": "0", "PSX_WALK_LEVELS": "0", "PSX_WALK_SHAPE": "3"}


def test_shipped_library_names_no_env_knob(built_lib):
    data = open(LIB, "rb").read()
    present = [k for k in KNOBS if k.encode() in data]
    assert not present, present


def test_probe_selector_refused_in_shipped_library(built_lib):
    PSX_DEBUG_ORD_PROBE = 23
    assert built_lib.psx_debug_set_variant(PSX_DEBUG_ORD_PROBE, 1) == -1
    assert built_lib.psx_debug_get_variant(PSX_DEBUG_ORD_PROBE) == -1


@pytest.mark.gpu
def test_env_knobs_leave_an_apply_unchanged(built_lib, oracle_lib):
    env = dict(os.environ)
    env.update(KNOB_ENV)
    env.pop("PSX_LIB", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "env_knob_probe.py")], env=env,
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0 and "env-knobs ok" in r.stdout, (r.stdout + r.stderr)[-3000:]
