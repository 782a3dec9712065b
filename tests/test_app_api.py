"""The petuum_ps App API on the host (no GPU): the headers compile a program that uses
every Table / PSTableGroup / row entry point, libpetuum_ps.so exports the runtime the
headers declare, and the client-side rows (DenseRow, SortedVectorMapRow, SparseRow)
keep the reference's store semantics and serialize to the server's row bytes."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "parameter_server_amd", "libpetuum_ps.so")

RUNTIME_FUNCS = ["Init", "ShutDown", "CreateTable", "CreateTableDone", "WaitThreadRegister",
                 "GetTableOrDie", "RegisterThread", "DeregisterThread", "Clock", "GlobalBarrier"]


def test_runtime_exports_every_declared_entry_point(built_lib):
    out = subprocess.run(["nm", "-DC", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    for f in RUNTIME_FUNCS:
        assert f"petuum::runtime::{f}(" in out, f
    # the runtime links libpsx.so (the C ABI) rather than carrying its own server code
    deps = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True, check=True).stdout
    assert "libpsx.so" in deps


ROWS_PROGRAM = r"""
#include <petuum_ps_common/include/petuum_ps.hpp>
#include <cstdio>
#include <vector>
using namespace petuum;
static void dump(const char *tag, const AbstractRow &r) {
  std::vector<unsigned char> b(r.SerializedSize());
  r.Serialize(b.data());
  std::printf("%s", tag);
  for (unsigned char c : b) std::printf(" %02x", c);
  std::printf("\n");
}
int main() {
  DenseRow<float> d; d.Init(4);
  float u[4] = {1.5f, 0.f, -2.f, 0.25f};
  d.ApplyDenseBatchInc(u, 0, 4);
  int32_t cols[2] = {3, 1}; float v[2] = {1.f, 2.f};
  d.ApplyBatchInc(cols, v, 2);
  dump("dense", d);
  SortedVectorMapRow<int32_t> s; s.Init(8);
  int32_t sc[5] = {7, 2, 9, 2, 7}; int32_t sv[5] = {1, 5, 3, 1, -1};
  s.ApplyBatchInc(sc, sv, 5);
  dump("sorted", s);
  SparseRow<double> m; m.Init(0);
  double dv[3] = {0.5, -1.0, 2.0}; int32_t dc[3] = {10, 4, 10};
  m.ApplyBatchInc(dc, dv, 3);
  dump("map", m);
  // a pushed row resets a cached one (ResetRowData)
  DenseRow<float> d2; d2.Init(4);
  std::vector<unsigned char> b(d.SerializedSize()); d.Serialize(b.data());
  d2.ResetRowData(b.data(), b.size());
  dump("reset", d2);
  UpdateBatch<float> ub; ub.Update(2, 1.f); ub.Update(0, 3.f);
  DenseUpdateBatch<float> db(1, 2); db[1] = 4.f; db[2] = 5.f;
  std::printf("batch %d %d %d\n", ub.GetBatchSize(), db.get_index_st(), db.get_num_updates());
  return 0;
}
"""


def _hex(arr):
    return " ".join(f"{c:02x}" for c in np.asarray(arr).tobytes())


def test_client_rows_match_server_row_bytes(tmp_path, built_lib):
    src = tmp_path / "rows.cpp"
    src.write_text(ROWS_PROGRAM)
    exe = tmp_path / "rows"
    lib_dir = os.path.join(ROOT, "parameter_server_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-L", lib_dir, "-lpetuum_ps", "-lpsx", f"-Wl,-rpath,{lib_dir}", "-lpthread"], check=True)
    out = dict(ln.split(" ", 1) for ln in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.strip().splitlines())
    # VectorStore: V[cap], adds in place
    assert out["dense"] == _hex(np.array([1.5, 2.0, -2.0, 1.25], np.float32))
    assert out["reset"] == out["dense"]
    # SortedVectorMapStore: 7:+1 -> [7:1]; 2:+5 -> [2:5, 7:1] (moves ahead of smaller);
    # 9:+3 -> [2:5, 9:3, 7:1]; 2:+1 stays; 7:-1 reaches 0 and is removed
    ent = np.zeros(2, dtype=[("c", "<i4"), ("v", "<i4")])
    ent["c"], ent["v"] = [2, 9], [6, 3]
    assert out["sorted"] == _hex(ent)
    # MapStore: {int32 col, V} ascending by col
    m = np.zeros(2, dtype=np.dtype([("c", "<i4"), ("v", "<f8")], align=False))
    m["c"], m["v"] = [4, 10], [-1.0, 2.5]
    assert out["map"] == _hex(m)
    assert out["batch"] == "2 1 2"


LOGIC_PROGRAM = r"""
#include <petuum_ps_common/include/petuum_ps.hpp>
#include <petuum_ps_common/include/constants.hpp>
#include <petuum_ps_common/include/abstract_server_table_logic.hpp>
#include <petuum_ps/server/adarevision_server_table_logic.hpp>
#include <cstdio>
// an app's own logic without a device implementation compiles against the interface
class MyLogic : public petuum::AbstractServerTableLogic {
 public:
  void Init(const petuum::TableInfo &, petuum::ApplyRowBatchIncFunc) override {}
  void ServerRowCreated(int32_t, petuum::ServerRow *) override {}
  void ApplyRowOpLog(int32_t, const int32_t *, const void *, int32_t, petuum::ServerRow *, uint64_t, bool) override {}
  void ServerRowSent(int32_t, uint64_t, size_t) override {}
  bool AllowSend() override { return true; }
};
int main() {
  auto &reg = petuum::ClassRegistry<petuum::AbstractServerTableLogic>::GetRegistry();
  reg.AddCreator(1, petuum::CreateObj<petuum::AbstractServerTableLogic, petuum::AdaRevisionServerTableLogic>);
  reg.AddCreator(2, petuum::CreateObj<petuum::AbstractServerTableLogic, MyLogic>);
  FLAGS_init_step_size = 0.25;
  petuum::TableInfo ti;
  ti.server_table_logic = 1;
  petuum::AbstractServerTableLogic *a = reg.CreateObject(1), *m = reg.CreateObject(2);
  a->Init(ti, nullptr);
  m->Init(ti, nullptr);
  const petuum::DeviceTableLogic d = a->GetDeviceLogic();
  std::printf("%d %g %d %llu %d %zu %llu\n", (int)d.kind, d.init_step_size, (int)d.gaussian_init,
              (unsigned long long)d.old_grad_upper_bound, (int)m->GetDeviceLogic().kind,
              petuum::k1_Mi, (unsigned long long)petuum::kMaxPendingMsgs);
  delete a;
  delete m;
  return 0;
}
"""


def test_server_table_logic_seam_compiles_and_selects_adarevision(tmp_path, built_lib):
    """abstract_server_table_logic.hpp (the reference's interface, :13-32), constants.hpp and
    adarevision_server_table_logic.hpp: an app registers logics through ClassRegistry as
    matrixfact_adarevision.cpp:633-635 does; AdaRevision maps to libpsx's device logic with
    its flags, an app-defined logic to none (CreateTable then refuses it)."""
    src = tmp_path / "logic.cpp"
    src.write_text(LOGIC_PROGRAM)
    exe = tmp_path / "logic"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["1", "0.25", "1", "10000", "0", str(1024 * 1024), "200"]
