// psx_server.hpp — header-only C++ mirror of the reference server-apply interface over
// the C ABI (include/psx.h).  Method names and argument meaning follow
// src/petuum_ps/server/server.hpp (Server::Init, CreateTable, ApplyOpLogUpdateVersion,
// GetBgVersion) and configs.hpp (TableInfo); errors that the reference turns into glog
// CHECK aborts (server.cpp:124-126, serialized_oplog_reader.hpp:112) throw psx::Error.
//
// A maintainer swaps `petuum::Server` for `psx::Server` inside ServerThread
// (server_thread.hpp:90); see INTEGRATION.md.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "psx.h"

namespace psx {

class Error : public std::runtime_error {
 public:
  Error(psx_status s, const std::string &msg)
      : std::runtime_error(std::string(psx_status_string(s)) + ": " + msg), status(s) {}
  psx_status status;
};

// The TableInfo fields the apply path reads (configs.hpp:170-210) plus shard geometry.
struct TableInfo {
  int32_t row_kind = PSX_ROW_DENSE;   // DenseRow / SortedVectorMapRow / SparseRow
  int32_t dtype = PSX_F32;
  int64_t row_capacity = 0;
  bool oplog_dense_serialized = true;
  int64_t dense_row_oplog_capacity = 0;   // 0 -> row_capacity
  int64_t row_offset = 0;
  int64_t row_stride = 1;
  int64_t max_rows = 0;
  int64_t max_entries = 0;
  bool accum_importance = false;             // SSPAggr importance policies (server_table.cpp:26-47)
  int64_t server_push_row_upper_bound = 0;   // configs.hpp:181; 0 -> 100
  bool version_maintain = false;             // configs.hpp:207 (VersionDenseRowOpLog / VersionServerRow)
  int32_t row_oplog_type = 0;                // configs.hpp:35-40 (3: float16 dense records)
  bool row_bytes_f16 = false;                // DenseRowFloat16 rows: served as binary16
};

class Server {
 public:
  Server() = default;
  Server(const Server &) = delete;
  Server &operator=(const Server &) = delete;
  ~Server() {
    if (ctx_) psx_ctx_destroy(ctx_);
  }

  // Server::Init(server_id, bg_ids) (server.cpp:18-31), plus the GPU this shard lives on.
  void Init(int32_t server_id, const std::vector<int32_t> &bg_ids, int32_t device = 0) {
    Check(psx_ctx_create(device, server_id, &ctx_));
    for (int32_t bg : bg_ids) Check(psx_register_sender(ctx_, bg));
  }

  // Server::CreateTable(table_id, table_info) (server.cpp:33-44).
  void CreateTable(int32_t table_id, const TableInfo &ti) {
    psx_table_config c{};
    c.table_id = table_id;
    c.row_kind = ti.row_kind;
    c.dtype = ti.dtype;
    c.oplog_dense_serialized = ti.oplog_dense_serialized ? 1 : 0;
    c.row_capacity = ti.row_capacity;
    c.dense_row_oplog_capacity = ti.dense_row_oplog_capacity ? ti.dense_row_oplog_capacity : ti.row_capacity;
    c.row_offset = ti.row_offset;
    c.row_stride = ti.row_stride;
    c.max_rows = ti.max_rows;
    c.max_entries = ti.max_entries;
    c.accum_importance = ti.accum_importance ? 1 : 0;
    c.server_push_row_upper_bound = ti.server_push_row_upper_bound;
    c.version_maintain = ti.version_maintain ? 1 : 0;
    c.row_oplog_type = ti.row_oplog_type;
    c.row_bytes_f16 = ti.row_bytes_f16 ? 1 : 0;
    Check(psx_table_create(ctx_, &c));
  }

  // Server::ApplyOpLogUpdateVersion (server.hpp:46-48, server.cpp:120-179): the oplog
  // bytes are borrowed for the call only, as in the reference.  The call returns once they
  // are copied to HBM; the apply runs beside the next call's copy, and a failure only the
  // device sees surfaces at the next Sync() (psx.h, PSX_SEAM_ASYNC) — SetSeam(PSX_SEAM_SYNC)
  // settles every call before it returns.
  void ApplyOpLogUpdateVersion(const void *oplog, size_t oplog_size, int32_t bg_thread_id,
                               uint32_t version) {
    Check(psx_apply_stream(ctx_, oplog, oplog_size, bg_thread_id, version));
  }

  // Batched, device-resident form: n messages applied as n sequential calls.
  void ApplyOpLogsDevice(const std::vector<psx_stream> &msgs) {
    Check(psx_apply_streams_device(ctx_, msgs.data(), (int32_t)msgs.size()));
  }

  void Sync() { Check(psx_sync(ctx_)); }
  void SetSeam(int32_t mode) { Check(psx_ctx_set_seam(ctx_, mode)); }

  // Server::GetBgVersion (server.cpp:186-188).
  int32_t GetBgVersion(int32_t bg_thread_id) {
    int64_t v = 0;
    Check(psx_sender_version(ctx_, bg_thread_id, &v));
    return (int32_t)v;
  }

  // ServerRow::Serialize framed as RecordBuff records (server_row.hpp:65-71,
  // record_buff.hpp:41-53), for the rows listed.
  std::vector<uint8_t> SerializeRows(int32_t table_id, const std::vector<int32_t> &row_ids) {
    size_t cap = 1 << 16;
    for (;;) {
      std::vector<uint8_t> out(cap);
      size_t used = 0;
      psx_status s = psx_serialize_rows(ctx_, table_id, row_ids.data(), (int32_t)row_ids.size(), out.data(),
                                        cap, &used);
      if (s == PSX_ERR_BUFFER_TOO_SMALL) {
        cap *= 4;
        continue;
      }
      Check(s);
      out.resize(used);
      return out;
    }
  }

  // Server::CreateSendServerPushRowMsgs / ...Partial (server.cpp:189-420): the push body.
  std::vector<uint8_t> CreatePushBody(bool partial, bool clear_dirty = true) {
    size_t used = 0;
    auto fn = partial ? psx_serialize_partial : psx_serialize_dirty;
    psx_status s = fn(ctx_, nullptr, 0, &used, 0, 0);
    if (s != PSX_ERR_BUFFER_TOO_SMALL) Check(s);
    std::vector<uint8_t> out(used);
    if (used) Check(fn(ctx_, out.data(), used, &used, 0, clear_dirty ? 1 : 0));
    out.resize(used);
    return out;
  }

  // TableInfo.server_table_logic = AdaRevision: AdaRevisionServerTableLogic::Init
  // (adarevision_server_table_logic.cpp:19-36), before the table's first apply.
  void SetAdaRevision(int32_t table_id, const psx_adarevision_config &cfg) {
    Check(psx_table_set_adarevision(ctx_, table_id, &cfg));
  }

  // Server::RowSent (server.cpp:436-441), called by ServerThread after a row request
  // reply (server_thread.cpp:221).
  void RowSent(int32_t table_id, const std::vector<int32_t> &row_ids, int32_t num_clients) {
    Check(psx_row_sent(ctx_, table_id, row_ids.data(), (int32_t)row_ids.size(), num_clients));
  }

  // VersionServerRow::get_version for a row range (version_server_row.hpp:66).
  std::vector<uint64_t> RowVersions(int32_t table_id, int64_t first_row, int64_t num_rows) {
    std::vector<uint64_t> v((size_t)num_rows);
    Check(psx_row_versions(ctx_, table_id, first_row, num_rows, v.data()));
    return v;
  }

  psx_ctx *handle() const { return ctx_; }

 private:
  void Check(psx_status s) {
    if (s != PSX_OK) throw Error(s, ctx_ ? psx_last_error(ctx_) : "");
  }
  psx_ctx *ctx_ = nullptr;
};

}  // namespace psx
