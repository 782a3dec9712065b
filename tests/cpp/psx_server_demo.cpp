// Drives libpsx through the C++ mirror (include/psx_server.hpp) the way
// ServerThread::HandleOpLogMsg drives petuum::Server (server_thread.cpp:224-299):
// one ApplyOpLogUpdateVersion per message, then serve-back of the rows.
// Messages are built with the reference packer's layout (oplog_serializer.hpp:12-37,
// row_oplog_serializer.hpp:139-166).  Writes the serialized rows to argv[1].
#include <cstdio>
#include <cstring>
#include <vector>

#include "psx_server.hpp"

static void put(std::vector<uint8_t> &b, const void *p, size_t n) {
  const uint8_t *q = (const uint8_t *)p;
  b.insert(b.end(), q, q + n);
}

// value pattern shared with tests/test_cpp_shim_gpu.py
static float val(int msg, int row, int col) { return (float)((row * 31 + col * 7 + msg * 13) % 17 - 8) * 0.25f; }

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const int kRows = 64, kCap = 16, kTable = 5;
  try {
    psx::Server server;
    server.Init(1, {100, 101});
    psx::TableInfo ti;
    ti.row_capacity = kCap;
    ti.max_rows = kRows;
    server.CreateTable(kTable, ti);
    for (int msg = 0; msg < 4; ++msg) {
      std::vector<uint8_t> b;
      int32_t num_tables = 1, tid = kTable, nrows = 0;
      uint64_t usz = sizeof(float);
      std::vector<int32_t> rows;
      for (int r = msg; r < kRows; r += 3) rows.push_back((r * 5 + msg) % kRows);
      std::vector<int32_t> uniq;
      for (int32_t r : rows) {
        bool seen = false;
        for (int32_t u : uniq) seen |= u == r;
        if (!seen) uniq.push_back(r);
      }
      nrows = (int32_t)uniq.size();
      put(b, &num_tables, 4);
      put(b, &tid, 4);
      put(b, &usz, 8);
      put(b, &nrows, 4);
      for (int32_t r : uniq) {
        put(b, &r, 4);
        for (int c = 0; c < kCap; ++c) {
          float v = val(msg, r, c);
          put(b, &v, 4);
        }
      }
      server.ApplyOpLogUpdateVersion(b.data(), b.size(), 100 + (msg & 1), (uint32_t)(msg >> 1));
    }
    std::vector<int32_t> ids;
    for (int r = 0; r < kRows; ++r) ids.push_back(r);
    std::vector<uint8_t> out = server.SerializeRows(kTable, ids);
    FILE *f = fopen(argv[1], "wb");
    if (!f) return 3;
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
    std::printf("versions %d %d, %zu bytes\n", server.GetBgVersion(100), server.GetBgVersion(101), out.size());
  } catch (const psx::Error &e) {
    std::fprintf(stderr, "psx error: %s\n", e.what());
    return 1;
  }
  return 0;
}
