""""Apps link unchanged" (SURVEY §8(b), App API row): every petuum:: name and every STATS_*
macro that apps/matrixfact, apps/lda and apps/mlr use is declared by the headers under
include/ — except the names listed below with the reason they are not the PS library's.
The list of used names is taken from the reference's app sources when /root/reference is
present (this container), else the test is skipped; the headers' side is checked by compiling
a program that uses every STATS_APP_* macro the apps call, without and with PETUUM_STATS
(stats.hpp:317-436, petuum_ps.hpp:13-14)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
REF_APPS = "/root/reference/apps"
APPS = ("matrixfact/src", "lda/src", "mlr/src")

# Names the three apps use that are not the parameter-server library (or are their own).
NOT_PS_LIBRARY = {
    # petuum::ml — the ML utility library (ml/include/ml/: feature vectors, data readers,
    # workload manager); the apps' compute and input side, not the table/row-update path
    "petuum::ml::AbstractFeature", "petuum::ml::DenseFeature", "petuum::ml::SparseFeature",
    "petuum::ml::FeatureScaleAndAdd", "petuum::ml::WorkloadManager", "petuum::ml::WorkloadManagerConfig",
    "petuum::ml::ReadDataLabelLibSVM", "petuum::ml::ReadDataLabelBinary", "petuum::ml::ReadDataLabelSparseFeatureBinary",
    "petuum::ml::MetafileReader", "petuum::ml::SparseDenseFeatureDotProduct", "petuum::ml::DenseDenseFeatureDotProduct",
    "petuum::ml::SparseSparseFeatureDotProduct", "petuum::ml::SafeLog", "petuum::ml::Softmax", "petuum::ml::Sigmoid",
    # defined by the apps themselves (matrixfact/src/process_snapshot.cpp:30, mlr/src/tools/string_buffer.hpp:8)
    "petuum::SnapshotProcessor", "petuum::StringBuffer",
    # named only inside comments (mlr_main.cpp:72, mlr_sgd_solver.cpp:123)
    "petuum::SparseFeatureRow",
}


def _header_text():
    out = []
    for d, _, fs in os.walk(INC):
        for f in fs:
            if f.endswith((".h", ".hpp")):
                out.append(open(os.path.join(d, f)).read())
    return "\n".join(out)


def _used_names():
    names = set()
    for a in APPS:
        for d, _, fs in os.walk(os.path.join(REF_APPS, a)):
            for f in fs:
                if f.endswith((".cpp", ".hpp", ".h")):
                    src = open(os.path.join(d, f), errors="replace").read()
                    names |= set(re.findall(r"\bpetuum::[A-Za-z_][A-Za-z_0-9:]*", src))
                    names |= set(re.findall(r"\bSTATS_[A-Z_0-9]+", src))
    return names


@pytest.mark.skipif(not os.path.isdir(REF_APPS), reason="reference sources not present (GPU box)")
def test_every_app_identifier_is_declared_under_include():
    hdr = _header_text()
    missing = []
    for n in sorted(_used_names()):
        if n in NOT_PS_LIBRARY:
            continue
        last = n.split("::")[-1]
        if n.startswith("STATS_"):
            ok = re.search(r"#define\s+" + re.escape(n) + r"\b", hdr)
        else:
            ok = re.search(r"(class|struct|enum|typedef|using|define)[^;{]*\b" + re.escape(last) + r"\b", hdr) \
                or re.search(r"\b" + re.escape(last) + r"\s*\(", hdr) \
                or re.search(r"enum[^;{]*\{[^}]*\b" + re.escape(last) + r"\b", hdr)   # an enumerator
        if not ok:
            missing.append(n)
    assert not missing, missing
    # the exclusions stay honest: each is still used by the apps
    used = _used_names()
    assert all(n in used for n in NOT_PS_LIBRARY), sorted(NOT_PS_LIBRARY - used)


STATS_PROGRAM = r"""
#include <petuum_ps_common/include/petuum_ps.hpp>
#include <cstdio>
int main() {
  STATS_APP_LOAD_DATA_BEGIN(); STATS_APP_LOAD_DATA_END();
  STATS_APP_INIT_BEGIN(); STATS_APP_INIT_END();
  STATS_APP_BOOTSTRAP_BEGIN(); STATS_APP_BOOTSTRAP_END();
  STATS_APP_ACCUM_COMP_BEGIN(); STATS_APP_ACCUM_COMP_END();
  STATS_APP_ACCUM_OBJ_COMP_BEGIN(); STATS_APP_ACCUM_OBJ_COMP_END();
  STATS_APP_ACCUM_TG_CLOCK_BEGIN(); STATS_APP_ACCUM_TG_CLOCK_END();
  STATS_SET_APP_DEFINED_ACCUM_SEC_NAME("sampling_sec");
  STATS_APP_DEFINED_ACCUM_SEC_BEGIN(); STATS_APP_DEFINED_ACCUM_SEC_END();
  STATS_SET_APP_DEFINED_ACCUM_VAL_NAME("llh");
  STATS_APP_DEFINED_ACCUM_VAL_INC(2.5);
  STATS_SET_APP_DEFINED_VEC_NAME("loss");
  STATS_APPEND_APP_DEFINED_VEC(0.75);
  STATS_SERVER_ACCUM_APPLY_OPLOG_BEGIN(); STATS_SERVER_ACCUM_APPLY_OPLOG_END();
  STATS_BG_ACCUM_TABLE_OPLOG_SENT(1, 2, 3);
  STATS_APP_SAMPLE_SSP_GET_END(1, true);
  STATS_PRINT();
  std::printf("%g %d\n", petuum::RestoreInfNaN(0.0f / 0.0f), (int)petuum::GetConsistencyModel("SSPPush"));
  return 0;
}
"""


@pytest.mark.parametrize("stats", [False, True], ids=["no-PETUUM_STATS", "PETUUM_STATS"])
def test_stats_macros_compile_in_both_forms(tmp_path, built_lib, stats):
    src = tmp_path / "stats.cpp"
    src.write_text(STATS_PROGRAM)
    exe = tmp_path / "stats"
    lib_dir = os.path.join(ROOT, "parameter_server_amd")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", INC, str(src), "-o", str(exe),
           "-L", lib_dir, "-lpetuum_ps", "-lpsx", f"-Wl,-rpath,{lib_dir}", "-lpthread"]
    if stats:
        cmd.insert(1, "-DPETUUM_STATS")
    subprocess.run(cmd, check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, check=True)
    assert r.stdout.split() == ["0.01", "1"]
    if stats:
        # the app-defined names label the accumulators; the server's apply counters come from
        # psx_ctx_stats summed over the process's shard contexts (none here: zeros)
        assert "sampling_sec:" in r.stderr and "llh: 2.5" in r.stderr and "loss: 0.75" in r.stderr
        assert "server_accum_apply_oplog_sec: 0.000000" in r.stderr
        assert "server_accum_oplog_recv_mb: 0.000000" in r.stderr
    else:
        assert r.stderr == ""
