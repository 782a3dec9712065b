""""Apps link unchanged" (SURVEY §8(b), App API row), checked by the compiler: every source
file of apps/matrixfact, apps/lda and apps/mlr — the reference's own files, read in place
under /root/reference, never copied — passes `g++ -std=c++11 -fsyntax-only` against this
repo's include/ (the petuum_ps App API: petuum_ps.hpp, the table/system gflags declare
headers, init_table_config.hpp / init_table_group_config.hpp, DenseRowFloat16, ...).

The apps also include third-party headers this image lacks (gflags, glog, boost, leveldb);
tests/compat_stubs/ holds declaration-only stand-ins for exactly the names the apps use, so
the check reaches the App API.  The petuum::ml library the apps use (src/ml, outside the
row-update path) is taken from the reference tree through a directory holding only an `ml`
link, so no reference petuum_ps header can stand in for a missing one of ours.  Skipped
when /root/reference is absent (the GPU box).

The flags themselves: petuum_flags.cpp (libpetuum_ps.so) compiled against the gflags stub,
so its gflags branch defines every flag; a program then sets flags as `--table_staleness 2
--consistency_model SSP ...` would and checks that InitTableConfig / InitTableGroupConfig
carry them into the configs (init_table_config.cpp:13-42, init_table_group_config.cpp:5-55)."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
STUBS = os.path.join(ROOT, "tests", "compat_stubs")
REF = "/root/reference"
APP_DIRS = ("apps/matrixfact/src", "apps/lda/src", "apps/mlr/src")


def _sources():
    if not os.path.isdir(REF):
        return []
    out = []
    for d in APP_DIRS:
        out += sorted(glob.glob(os.path.join(REF, d, "*.cpp")))
    return out


@pytest.fixture(scope="module")
def ml_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("appinc")
    os.symlink(os.path.join(REF, "src", "ml"), str(d / "ml"))
    return str(d)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference app sources absent")
def test_every_app_translation_unit_compiles(ml_dir):
    srcs = _sources()
    names = {os.path.basename(s) for s in srcs}
    # the four the north star names, and every other file of the three apps
    assert {"matrixfact_split.cpp", "matrixfact_split16.cpp", "lda_main.cpp", "mlr_main.cpp"} <= names
    failed = {}
    for src in srcs:
        r = subprocess.run(["g++", "-std=c++11", "-fsyntax-only", "-I" + INC, "-I" + STUBS, "-I" + ml_dir,
                            "-I" + os.path.dirname(src), src], capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            failed[os.path.relpath(src, REF)] = [l for l in r.stderr.splitlines() if "error" in l][:3]
    assert not failed, failed


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference app sources absent")
def test_app_flag_headers_are_ours(ml_dir):
    """The declare headers the apps include resolve to include/, not to the reference."""
    src = os.path.join(REF, "apps/matrixfact/src/matrixfact_split.cpp")
    r = subprocess.run(["g++", "-std=c++11", "-M", "-I" + INC, "-I" + STUBS, "-I" + ml_dir, src],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    deps = r.stdout.replace("\\\n", " ").split()
    for h in ("table_gflags_declare.hpp", "system_gflags_declare.hpp", "init_table_config.hpp",
              "init_table_group_config.hpp", "petuum_ps.hpp"):
        hit = [d for d in deps if d.endswith("/" + h)]
        assert hit and all(d.startswith(INC) for d in hit), (h, hit)


FLAGS_MAIN = r"""
#include <petuum_ps_common/include/table_gflags_declare.hpp>
#include <petuum_ps_common/include/system_gflags_declare.hpp>
#include <petuum_ps_common/include/init_table_config.hpp>
#include <petuum_ps_common/include/init_table_group_config.hpp>
#include <cstdio>
#include <fstream>
namespace google {
void ParseCommandLineFlags(int *, char ***, bool) {}
}
#define EXPECT(c) do { if (!(c)) { std::printf("FAIL %s\n", #c); return 1; } } while (0)
int main(int argc, char **argv) {
  petuum::ClientTableConfig d;
  petuum::InitTableConfig(&d);   // the reference's defaults (table_gflags.cpp:10-24)
  EXPECT(d.table_info.table_staleness == 0 && d.table_info.row_type == 0 && d.table_info.oplog_dense_serialized);
  EXPECT(d.oplog_type == petuum::Sparse && d.process_storage_type == petuum::BoundedSparse);
  EXPECT(d.table_info.server_push_row_upper_bound == 100 && d.table_info.server_table_logic == -1);
  petuum::TableGroupConfig gd;
  petuum::InitTableGroupConfig(&gd, 3);
  EXPECT(gd.consistency_model == petuum::SSPPush && gd.num_tables == 3 && gd.num_local_app_threads == 2);
  // as `--table_staleness 2 --row_type 5 --oplog_type Dense --process_storage_type BoundedDense
  //      --no_oplog_replay --version_maintain --server_table_logic 1 --consistency_model SSP
  //      --num_comm_channels_per_client 4 --num_table_threads 6 --init_thread_access_table
  //      --client_id 0 --hostfile <file> --update_sort_policy RelativeMagnitude` would set them
  FLAGS_table_staleness = 2;
  FLAGS_row_type = 5;
  FLAGS_oplog_type = "Dense";
  FLAGS_process_storage_type = "BoundedDense";
  FLAGS_no_oplog_replay = true;
  FLAGS_version_maintain = true;
  FLAGS_server_table_logic = 1;
  FLAGS_server_push_row_upper_bound = 7;
  FLAGS_consistency_model = "SSP";
  FLAGS_num_comm_channels_per_client = 4;
  FLAGS_num_table_threads = 6;
  FLAGS_init_thread_access_table = true;
  FLAGS_update_sort_policy = "RelativeMagnitude";
  FLAGS_hostfile = argv[1];
  petuum::ClientTableConfig c;
  petuum::InitTableConfig(&c);
  EXPECT(c.table_info.table_staleness == 2 && c.table_info.row_type == 5);
  EXPECT(c.oplog_type == petuum::Dense && c.process_storage_type == petuum::BoundedDense);
  EXPECT(c.no_oplog_replay && c.table_info.version_maintain && c.table_info.server_table_logic == 1);
  EXPECT(c.table_info.server_push_row_upper_bound == 7);
  petuum::TableGroupConfig g;
  petuum::InitTableGroupConfig(&g, 2);
  EXPECT(g.consistency_model == petuum::SSP && g.num_comm_channels_per_client == 4);
  EXPECT(g.num_local_app_threads == 6 && g.update_sort_policy == petuum::RelativeMagnitude);
  EXPECT(g.host_map.size() == 2 && g.host_map.at(0).ip == "127.0.0.1" && g.host_map.at(1).port == "10001");
  std::printf("flags ok\n");
  return 0;
}
"""


def test_flags_reach_the_configs(tmp_path):
    main = tmp_path / "flags_main.cpp"
    main.write_text(FLAGS_MAIN)
    hosts = tmp_path / "hosts"
    hosts.write_text("0 127.0.0.1 10000\n1 127.0.0.1 10001\n")
    exe = tmp_path / "flags_main"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I" + INC, "-I" + STUBS, str(main),
                        os.path.join(ROOT, "parameter_server_amd", "csrc", "petuum_flags.cpp"), "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe), str(hosts)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "flags ok" in r.stdout, r.stdout + r.stderr


def test_no_gflags_build_uses_the_reference_defaults(tmp_path):
    """Without gflags (this image) the flags are constants at the reference's defaults."""
    main = tmp_path / "nog.cpp"
    main.write_text(r"""
#include <petuum_ps_common/include/table_gflags_declare.hpp>
#include <petuum_ps_common/include/system_gflags_declare.hpp>
#include <petuum_ps_common/include/init_table_config.hpp>
#include <petuum_ps_common/include/init_table_group_config.hpp>
static_assert(!PETUUM_PS_HAVE_GFLAGS, "gflags found");
int main() {
  petuum::ClientTableConfig c;
  petuum::InitTableConfig(&c);
  petuum::TableGroupConfig g;
  petuum::InitTableGroupConfig(&g, 1);
  return (c.table_info.oplog_dense_serialized && c.oplog_type == petuum::Sparse &&
          g.consistency_model == petuum::SSPPush && FLAGS_bg_idle_milli == 10) ? 0 : 1;
}
""")
    exe = tmp_path / "nog"
    r = subprocess.run(["g++", "-std=c++17", "-I" + INC, str(main),
                        os.path.join(ROOT, "parameter_server_amd", "csrc", "petuum_flags.cpp"), "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "gflags found" in r.stderr:
        pytest.skip("gflags installed here")
    assert r.returncode == 0, r.stderr
    assert subprocess.run([str(exe)]).returncode == 0


def _nm(path, *flags):
    r = subprocess.run(["nm", *flags, path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = []
    for line in r.stdout.splitlines():
        parts = line.split()
        if len(parts) >= 2:
            out.append((parts[-2], parts[-1]))   # (type, mangled name)
    return out


def _demangle(names):
    if not names:
        return {}
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, timeout=60)
    return dict(zip(names, r.stdout.splitlines()))


def _is_ours(dem):
    """A symbol libpetuum_ps must supply: petuum:: (not the petuum::ml library, src/ml, which
    is outside the row-update path) or a gflags flag variable."""
    return ((dem.startswith("petuum::") and not dem.startswith("petuum::ml::")) or
            dem.startswith("FLAGS_"))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference app sources absent")
def test_every_app_links_against_libpetuum_ps(ml_dir, tmp_path):
    """"Apps link unchanged", at the linker's level (VERDICT r5 missing #2): every app TU is
    compiled to an object (-c) against include/, and every petuum:: / FLAGS_ symbol an app
    leaves undefined — after its own objects' definitions — is defined by libpetuum_ps.

    The apps compile in gflags mode here (tests/compat_stubs/gflags), so the library they
    are checked against is the same two sources (petuum_runtime.cpp, petuum_flags.cpp)
    built in gflags mode against that stub; the shipped libpetuum_ps.so (no gflags in this
    image) must export the same petuum:: set apart from the flags-mode marker, and an app
    object compiled in gflags mode must NOT resolve against it (the marker)."""
    csrc = os.path.join(ROOT, "parameter_server_amd", "csrc")
    pkg = os.path.join(ROOT, "parameter_server_amd")
    shipped = os.path.join(pkg, "libpetuum_ps.so")
    assert os.path.exists(shipped), "build() first"
    glib = str(tmp_path / "libpetuum_ps_gflags.so")
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-I" + INC, "-I" + STUBS,
                        os.path.join(csrc, "petuum_runtime.cpp"), os.path.join(csrc, "petuum_flags.cpp"),
                        "-L" + pkg, "-lpsx", "-o", glib], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    gdef = {n for t, n in _nm(glib, "-D", "--defined-only")}
    sdef = {n for t, n in _nm(shipped, "-D", "--defined-only")}
    dem = _demangle(sorted(gdef | sdef))
    strong = {n for t, n in _nm(glib, "-D", "--defined-only") + _nm(shipped, "-D", "--defined-only")
              if t in "TDBR"}   # weak inline/template copies differ with inlining; not the API
    g_ours = {n for n in gdef & strong if dem[n].startswith("petuum::")}
    s_ours = {n for n in sdef & strong if dem[n].startswith("petuum::")}
    assert g_ours - s_ours == {n for n in g_ours if "flags_mode" in dem[n]}, sorted(dem[n] for n in g_ours - s_ours)

    missing, checked = {}, 0
    for d in APP_DIRS:
        srcs = sorted(glob.glob(os.path.join(REF, d, "*.cpp")))
        objs = []
        for src in srcs:
            o = str(tmp_path / (d.replace("/", "_") + "_" + os.path.basename(src) + ".o"))
            r = subprocess.run(["g++", "-std=c++11", "-c", "-O0", "-I" + INC, "-I" + STUBS, "-I" + ml_dir,
                                "-I" + os.path.dirname(src), src, "-o", o],
                               capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, (src, r.stderr[-2000:])
            objs.append(o)
        defined, undef = set(), set()
        for o in objs:
            for t, n in _nm(o):
                (undef if t == "U" else defined).add(n)
        need = undef - defined
        dm = _demangle(sorted(need))
        ours = {n for n in need if _is_ours(dm[n])}
        checked += len(ours)
        lack = sorted(dm[n] for n in ours if n not in gdef)
        if lack:
            missing[d] = lack
        marker = [n for n in ours if "flags_mode" in dm[n]]
        assert marker and all(n not in sdef for n in marker), "the flags-mode marker must not resolve across modes"
    assert not missing, missing
    assert checked >= 10, checked
