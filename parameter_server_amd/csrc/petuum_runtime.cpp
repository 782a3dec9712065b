// petuum_runtime.cpp — the client runtime behind the petuum_ps App API
// (include/petuum_ps_common/...): libpetuum_ps.so.
//
// One process is one client (client id from TableGroupConfig) with num_comm_channels
// bg threads; channel ch's server shard is a psx context on this process's GPU owning the
// rows r with r % C == ch (GlobalContext::GetPartitionCommChannelIndex, context.hpp:291-293).
// The reference's threads collapse into calls made under one lock by the app threads:
//
//   Inc / BatchInc / DenseBatchInc   add into the table's oplog and into the cached row
//                                    (SSPConsistencyController, ssp_consistency_controller.cpp:98-187)
//   Clock                            one vector clock over the app threads (table_group.cpp:219-234);
//                                    when the process clock advances the "bg threads" pack every
//                                    table's oplog per shard (CreateOpLogMsgs + OpLogSerializer +
//                                    RowOpLogSerializer, abstract_bg_worker.cpp:590-689) into a
//                                    ClientSendOpLogMsg and hand it to its shard:
//                                    psx_handle_oplog_msg = ServerThread::HandleOpLogMsg's apply +
//                                    ClockUntil; on a new min clock the shard pushes
//                                    (psx_serialize_push) and the client resets its cached rows from
//                                    its body (SSPPushBgWorker::ApplyServerPushedRow,
//                                    ssp_push_bg_worker.cpp:70-122) and raises the system clock
//   Get                              SSPPush read (ssp_push_consistency_controller.cpp:70-120): wait
//                                    until the pushed system clock reaches clock - staleness, then the
//                                    cached row, or a row request: subscribe + serialize on the shard
//                                    (HandleRowRequest, server_thread.cpp:185-222) and insert
//
// PSX_TRACE_DIR=<dir> records every message handed to a shard and every push body it
// returns (the C1 test replays them through the CPU oracle).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <petuum_ps_common/include/abstract_server_table_logic.hpp>
#include <petuum_ps_common/include/ps_table_group.hpp>
#include <petuum_ps_common/util/stats.hpp>

#include "psx.h"

namespace petuum {
namespace runtime {
namespace {

[[noreturn]] void die(const std::string &msg) {
  // the reference aborts through glog CHECK; the runtime reports and aborts the same way
  std::fprintf(stderr, "petuum_ps runtime: %s\n", msg.c_str());
  std::abort();
}

void check(psx_ctx *ctx, psx_status st, const char *what) {
  if (st != PSX_OK)
    die(std::string(what) + ": " + psx_status_string(st) + " (" + (ctx ? psx_last_error(ctx) : "") + ")");
}

int vsize_of(int dt) { return (dt == PSX_F32 || dt == PSX_I32) ? 4 : 8; }

void add_value(int dt, uint8_t *acc, const void *u) {
  switch (dt) {
    case PSX_F32: *(float *)acc += *(const float *)u; break;
    case PSX_F64: *(double *)acc += *(const double *)u; break;
    case PSX_I32: *(int32_t *)acc += *(const int32_t *)u; break;
    default: *(int64_t *)acc += *(const int64_t *)u; break;
  }
}

bool is_zero(int dt, const uint8_t *p) {
  switch (dt) {
    case PSX_F32: return *(const float *)p == 0.0f;
    case PSX_F64: return *(const double *)p == 0.0;
    case PSX_I32: return *(const int32_t *)p == 0;
    default: return *(const int64_t *)p == 0;
  }
}

struct Shard {
  psx_ctx *ctx = nullptr;
  int32_t device = 0;
  int32_t bg_id = 0;
  uint32_t version = 0;      // the bg thread's message version (ssp_bg_worker.cpp:250-257)
  int32_t pushed_clock = 0;  // the clock of its last push (ServerPushRowMsg clock)
};

class Runtime;

class ClientTableImpl : public AbstractClientTable {
 public:
  ClientTableImpl(Runtime *rt, int32_t id, const ClientTableConfig &cfg, std::unique_ptr<AbstractRow> sample)
      : rt_(rt), id_(id), cfg_(cfg), sample_(std::move(sample)) {
    kind_ = sample_->psx_row_kind();
    dtype_ = sample_->psx_dtype();
    vsize_ = vsize_of(dtype_);
    oplog_cap_ = cfg_.table_info.dense_row_oplog_capacity ? cfg_.table_info.dense_row_oplog_capacity
                                                          : cfg_.table_info.row_capacity;
    dense_oplog_ = cfg_.table_info.row_oplog_type == RowOpLogType::kDenseRowOpLog;
    version_ = cfg_.table_info.version_maintain;
  }
  int32_t row_bytes_f16() const { return sample_->psx_row_bytes_f16(); }

  void RegisterThread() override {}
  void DeregisterThread() override {}
  void GetAsyncForced(int32_t row_id) override;
  void GetAsync(int32_t row_id) override { GetAsyncForced(row_id); }
  void WaitPendingAsyncGet() override {}
  void ThreadGet(int32_t row_id, ThreadRowAccessor *acc) override {
    RowAccessor a;
    Get(row_id, &a);
    acc->Set(Find(row_id));
  }
  void ThreadInc(int32_t r, int32_t c, const void *u) override { Inc(r, c, u); }
  void ThreadBatchInc(int32_t r, const int32_t *c, const void *u, int32_t n) override { BatchInc(r, c, u, n); }
  void ThreadDenseBatchInc(int32_t r, const void *u, int32_t st, int32_t n) override { DenseBatchInc(r, u, st, n); }
  void FlushThreadCache() override {}

  AbstractRow *Get(int32_t row_id, RowAccessor *acc) override;
  void Inc(int32_t row_id, int32_t col, const void *u) override { BatchInc(row_id, &col, u, 1); }
  void BatchInc(int32_t row_id, const int32_t *cols, const void *u, int32_t n) override;
  void DenseBatchInc(int32_t row_id, const void *u, int32_t index_st, int32_t n) override;
  void Clock() override {}
  int32_t get_row_type() const override { return cfg_.table_info.row_type; }

  // runtime side (under the runtime lock)
  std::shared_ptr<AbstractRow> Find(int32_t row_id) {
    std::lock_guard<std::mutex> g(mtx_);
    auto it = cache_.find(row_id);
    return it == cache_.end() ? nullptr : it->second;
  }
  void Insert(int32_t row_id, const uint8_t *data, size_t size);
  void Reset(int32_t row_id, const uint8_t *data, size_t size, int ch);
  void ReplayOplogLocked(int32_t row_id, AbstractRow *r);
  // RowOpLogSerializer::AppendRowOpLog for the rows of shard ch (r % C == ch), then clears them
  size_t SerializeOplog(int ch, int C, std::vector<uint8_t> *out, int32_t *num_rows);
  // Version tables: the end-of-version records a push produced for shard ch (taken)
  int32_t TakeEndOfVersion(int ch, std::vector<uint8_t> *out);
  bool version_maintain() const { return version_; }
  void set_logic(std::unique_ptr<AbstractServerTableLogic> l) { logic_ = std::move(l); }

  int32_t id() const { return id_; }
  int kind() const { return kind_; }
  int dtype() const { return dtype_; }
  const ClientTableConfig &cfg() const { return cfg_; }
  int64_t oplog_cap() const { return oplog_cap_; }

 private:
  Runtime *rt_;
  int32_t id_;
  ClientTableConfig cfg_;
  std::unique_ptr<AbstractRow> sample_;
  int kind_ = 0, dtype_ = 0, vsize_ = 4;
  int64_t oplog_cap_ = 0;
  bool dense_oplog_ = true;
  bool version_ = false;                                           // TableInfo.version_maintain
  std::unique_ptr<AbstractServerTableLogic> logic_;                // server_table_logic (runs on the device)
  std::mutex mtx_;                                                 // cache_ + oplogs
  std::unordered_map<int32_t, std::shared_ptr<AbstractRow>> cache_;   // process storage
  std::map<int32_t, std::vector<uint8_t>> dense_oplog_rows_;        // DenseRowOpLog V[cap]
  std::map<int32_t, std::map<int32_t, uint64_t>> sparse_oplog_rows_;   // SparseRowOpLog col -> V bits
  // Version tables (VersionDenseRowOpLog, version_dense_row_oplog.hpp:20-180): a row's oplog
  // lives on after it is sent (Reset zeroes it) and carries the version of the row the
  // server last pushed; rows touched since the last send (the oplog index).
  std::map<int32_t, uint64_t> oplog_version_;
  std::map<int32_t, bool> oplog_index_;
  std::map<int, std::vector<uint8_t>> eov_;                        // shard -> end-of-version records
  std::map<int, int32_t> eov_rows_;
  void AppendVersionRecord(std::vector<uint8_t> *out, int32_t row_id, const std::vector<uint8_t> &op,
                           uint64_t version, bool end_of_version);
};

class Runtime {
 public:
  explicit Runtime(const TableGroupConfig &cfg, bool table_access) : cfg_(cfg) {
    C_ = std::max(1, cfg.num_comm_channels_per_client);
    if (cfg.consistency_model != SSPPush && cfg.consistency_model != SSP)
      die("consistency models other than SSP/SSPPush are not provided by this runtime");
    // Every client's bg sender is registered on this process's shards, but only this
    // process's bg ever clocks them: with more clients the min clock would never advance
    // and the first Get after a Clock would wait forever.  Cross-process clients are not
    // provided (the reference reaches them over ZeroMQ tcp, out of scope).
    if (cfg.num_total_clients > 1)
      die("num_total_clients > 1 (clients in other processes) is not provided by this runtime");
    // Shard (comm channel) ch lives on devices_[ch % devices_.size()]: every visible GPU by
    // default, PSX_DEVICES="0,2,..." to choose them, PSX_DEVICE=<d> for one
    if (const char *d = std::getenv("PSX_DEVICES")) {
      for (const char *p = d; *p;) {
        devices_.push_back(std::atoi(p));
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
      }
    } else if (const char *d1 = std::getenv("PSX_DEVICE")) {
      devices_.push_back(std::atoi(d1));
    } else {
      int32_t nd = 0;
      check(nullptr, psx_device_count(&nd), "psx_device_count");
      for (int32_t i = 0; i < nd; ++i) devices_.push_back(i);
    }
    if (devices_.empty()) die("no devices for the server shards");
    shards_.resize(C_);
    for (int ch = 0; ch < C_; ++ch) {
      Shard &s = shards_[ch];
      s.device = devices_[ch % devices_.size()];
      check(nullptr, psx_ctx_create(s.device, cfg.client_id * 1000 + 1 + ch, &s.ctx), "psx_ctx_create");
      // thread ids: client * 1000 + 100 + channel for bg threads (context.hpp:410-414)
      for (int32_t client = 0; client < std::max(1, cfg.num_total_clients); ++client)
        check(s.ctx, psx_register_sender(s.ctx, client * 1000 + 100 + ch), "register sender");
      check(s.ctx, psx_set_num_clients(s.ctx, std::max(1, cfg.num_total_clients)), "set clients");
      s.bg_id = cfg.client_id * 1000 + 100 + ch;
    }
    if (const char *t = std::getenv("PSX_TRACE_DIR")) trace_dir_ = t;
    table_access_ = table_access;
    // num_local_app_threads counts the init thread (table_group.cpp:14-33)
    num_table_threads_ = std::max(1, table_access ? cfg.num_local_app_threads : cfg.num_local_app_threads - 1);
  }
  ~Runtime() {
    for (auto &s : shards_)
      if (s.ctx) psx_ctx_destroy(s.ctx);
    if (trace_index_) std::fclose(trace_index_);
  }

  bool CreateTable(int32_t id, const ClientTableConfig &c) {
    std::lock_guard<std::mutex> g(mtx_);
    if (tables_.count(id)) return false;
    std::unique_ptr<AbstractRow> sample(ClassRegistry<AbstractRow>::GetRegistry().CreateObject(c.table_info.row_type));
    if (!sample) die("row type " + std::to_string(c.table_info.row_type) + " not registered (RegisterRow)");
    if (sample->psx_row_kind() < 0 || sample->psx_dtype() < 0)
      die("row type " + std::to_string(c.table_info.row_type) + " has no MI355X server storage");
    if (c.process_cache_capacity == 0) die("process_cache_capacity must bound the table's row ids");
    const int32_t rot = c.table_info.row_oplog_type;
    if (rot != RowOpLogType::kDenseRowOpLog && rot != RowOpLogType::kSparseRowOpLog)
      die("row_oplog_type " + std::to_string(rot) + " is not provided by this runtime");
    if (rot == RowOpLogType::kSparseRowOpLog && c.table_info.oplog_dense_serialized &&
        sample->psx_row_kind() == PSX_ROW_DENSE)   // sparse_row_oplog.hpp:156-159
      die("Sparse OpLog does not support dense serialize");
    const bool version = c.table_info.version_maintain;
    if (version && (sample->psx_row_kind() != PSX_ROW_DENSE || rot != RowOpLogType::kDenseRowOpLog ||
                    !c.table_info.oplog_dense_serialized))
      die("version_maintain needs DenseRow tables with dense-serialized kDenseRowOpLog oplogs "
          "(VersionDenseRowOpLog, version_dense_row_oplog.hpp)");
    if (version && !c.no_oplog_replay)   // CHECK(no_oplog_replay), abstract_bg_worker.cpp:809-811
      die("version_maintain needs no_oplog_replay");
    // TableInfo.server_table_logic: the registered logic (ServerTable::ServerTable,
    // server_table.cpp:83-93) selects one of libpsx's device logics
    std::unique_ptr<AbstractServerTableLogic> logic;
    DeviceTableLogic dl;
    if (c.table_info.server_table_logic >= 0) {
      logic.reset(ClassRegistry<AbstractServerTableLogic>::GetRegistry().CreateObject(c.table_info.server_table_logic));
      if (!logic)
        die("server table logic " + std::to_string(c.table_info.server_table_logic) +
            " not registered (ClassRegistry<AbstractServerTableLogic>::AddCreator)");
      logic->Init(c.table_info, nullptr);
      dl = logic->GetDeviceLogic();
      if (dl.kind == DeviceTableLogicKind::kNone)
        die("server table logic " + std::to_string(c.table_info.server_table_logic) +
            " has no device implementation in libpsx (built in: AdaRevision)");
      if (dl.kind == DeviceTableLogicKind::kAdaRevision &&
          (sample->psx_row_kind() != PSX_ROW_DENSE || sample->psx_dtype() != PSX_F32 || rot != RowOpLogType::kDenseRowOpLog ||
           !c.table_info.oplog_dense_serialized))
        die("the AdaRevision logic runs on DenseRow<float> tables with dense-serialized kDenseRowOpLog oplogs");
    }
    auto t = std::make_unique<ClientTableImpl>(this, id, c, std::move(sample));
    const int64_t rows = (int64_t)c.process_cache_capacity;
    for (int ch = 0; ch < C_; ++ch) {
      psx_table_config pc{};
      pc.table_id = id;
      pc.row_kind = t->kind();
      pc.dtype = t->dtype();
      pc.oplog_dense_serialized = c.table_info.oplog_dense_serialized && t->kind() == PSX_ROW_DENSE ? 1 : 0;
      pc.row_capacity = (int64_t)std::max<size_t>(c.table_info.row_capacity, 1);
      pc.dense_row_oplog_capacity = t->oplog_cap();
      pc.row_offset = ch;
      pc.row_stride = C_;
      pc.max_rows = (rows - ch + C_ - 1) / C_;
      if (pc.max_rows < 1) pc.max_rows = 1;
      pc.max_entries = t->kind() == PSX_ROW_DENSE ? 0 : std::max<int64_t>(pc.row_capacity, 64);
      pc.server_push_row_upper_bound = (int64_t)c.table_info.server_push_row_upper_bound;
      pc.version_maintain = version ? 1 : 0;
      pc.row_bytes_f16 = t->row_bytes_f16();   // DenseRowFloat16: served as binary16
      check(shards_[ch].ctx, psx_table_create(shards_[ch].ctx, &pc), "psx_table_create");
      if (dl.kind == DeviceTableLogicKind::kAdaRevision) {
        psx_adarevision_config ac{};
        ac.init_step_size = dl.init_step_size;
        ac.gaussian_init = dl.gaussian_init ? 1 : 0;
        ac.old_grad_upper_bound = dl.old_grad_upper_bound;
        ac.push_clients = std::max(1, cfg_.num_total_clients);
        ac.max_snapshots_per_row = dl.max_snapshots_per_row;
        check(shards_[ch].ctx, psx_table_set_adarevision(shards_[ch].ctx, id, &ac), "AdaRevision logic");
      }
    }
    t->set_logic(std::move(logic));
    staleness_ = std::max(staleness_, c.table_info.table_staleness);
    table_order_.push_back(id);
    tables_[id] = std::move(t);
    return true;
  }

  ClientTableImpl *table(int32_t id) {
    auto it = tables_.find(id);
    if (it == tables_.end()) die("table " + std::to_string(id) + " not found (GetTableOrDie)");
    return it->second.get();
  }

  // TableGroup::RegisterThread (table_group.cpp:154-180): a vector-clock entry at clock 0,
  // then the register barrier over every table thread, so no thread's clock runs ahead of
  // a thread that has not registered yet
  int32_t RegisterThread(bool wait = true) {
    int32_t tid;
    {
      std::lock_guard<std::mutex> g(mtx_);
      tid = cfg_.client_id * 1000 + 200 + next_thread_++;   // kInitThreadIDOffset = 200
      thread_clock_[tid] = 0;
    }
    tls_thread_id_ = tid;
    tls_clock_ = 0;
    if (wait) ArriveRegisterBarrier();
    return tid;
  }
  void WaitThreadRegister() {
    if (table_access_) ArriveRegisterBarrier();
  }
  // The reference keeps a deregistered thread's clock in the vector clock.
  void DeregisterThread() {}

  // TableGroup::ClockConservative: the vector clock ticks; a new process clock (min over
  // the app threads) sends every table's oplog with is_clock (BgWorkers::ClockAllTables)
  void Clock() {
    std::lock_guard<std::mutex> g(mtx_);
    ++tls_clock_;
    thread_clock_[tls_thread_id_] = tls_clock_;
    AdvanceProcessClockLocked();
  }
  void GlobalBarrier() {
    for (int i = 0; i < staleness_ + 1; ++i) Clock();
  }

  int32_t staleness() const { return staleness_; }
  int32_t thread_clock() const { return tls_clock_; }

  // SSPPush Get gate: wait until the pushed system clock reaches `clock`
  void WaitSystemClock(int32_t clock) {
    std::unique_lock<std::mutex> l(clock_mtx_);
    clock_cv_.wait(l, [&] { return system_clock_ >= clock; });
  }

  // HandleRowRequest + ReplyRowRequest on the owning shard, then insert into the cache
  void FetchRow(ClientTableImpl *t, int32_t row_id) {
    std::lock_guard<std::mutex> g(mtx_);
    if (t->Find(row_id)) return;
    const int ch = row_id % C_;
    Shard &s = shards_[ch];
    const int32_t req[2] = {t->id(), row_id};
    Trace("req", ch, req_seq_, req, sizeof(req));
    check(s.ctx, psx_row_subscribe(s.ctx, t->id(), &row_id, 1, cfg_.client_id), "row request");
    std::vector<uint8_t> buf(1 << 16);
    size_t used = 0;
    for (;;) {
      psx_status st = psx_serialize_rows(s.ctx, t->id(), &row_id, 1, buf.data(), buf.size(), &used);
      if (st == PSX_ERR_BUFFER_TOO_SMALL) {
        buf.resize(buf.size() * 4);
        continue;
      }
      check(s.ctx, st, "row reply");
      break;
    }
    check(s.ctx, psx_row_sent(s.ctx, t->id(), &row_id, 1, 1), "RowSent");
    Trace("reply", ch, req_seq_++, buf.data(), used);
    if (used < 12) die("row request for " + std::to_string(row_id) + " returned no row");
    uint64_t size = 0;
    std::memcpy(&size, buf.data() + 4, 8);
    t->Insert(row_id, buf.data() + 12, (size_t)size);
  }

 private:
  void ArriveRegisterBarrier() {
    std::unique_lock<std::mutex> l(reg_mtx_);
    const int64_t gen = reg_gen_;
    if (++reg_arrived_ >= num_table_threads_) {
      reg_arrived_ = 0;
      ++reg_gen_;
      reg_cv_.notify_all();
      return;
    }
    reg_cv_.wait(l, [&] { return reg_gen_ != gen; });
  }

  void AdvanceProcessClockLocked() {
    if (thread_clock_.empty()) return;
    int32_t m = INT32_MAX;
    for (auto &kv : thread_clock_) m = std::min(m, kv.second);
    while (process_clock_ < m) {
      ++process_clock_;
      ClockAllTablesLocked(process_clock_);
    }
  }

  void Trace(const std::string &kind, int ch, int64_t seq, const void *p, size_t n) {
    if (trace_dir_.empty()) return;
    std::lock_guard<std::mutex> g(trace_mtx_);
    if (!trace_index_) trace_index_ = std::fopen((trace_dir_ + "/index.txt").c_str(), "w");
    const std::string name = kind + "_" + std::to_string(seq) + "_ch" + std::to_string(ch) + ".bin";
    FILE *f = std::fopen((trace_dir_ + "/" + name).c_str(), "wb");
    if (f) {
      if (n) std::fwrite(p, 1, n, f);
      std::fclose(f);
    }
    if (trace_index_) {
      std::fprintf(trace_index_, "%s %d %lld %s\n", kind.c_str(), ch, (long long)seq, name.c_str());
      std::fflush(trace_index_);
    }
  }

  // BgWorkers::ClockAllTables: every shard gets this client's message for the clock.  The
  // reference's server threads run concurrently; here the shards on distinct GPUs do (one
  // host thread per shard for the clock: a psx context is driven by one thread at a time),
  // shards sharing a GPU take their turn.
  void ClockAllTablesLocked(int32_t clock) {
    std::vector<std::vector<int>> by_dev;
    for (int ch = 0; ch < C_; ++ch) {
      size_t k = 0;
      while (k < by_dev.size() && shards_[by_dev[k][0]].device != shards_[ch].device) ++k;
      if (k == by_dev.size()) by_dev.emplace_back();
      by_dev[k].push_back(ch);
    }
    if (by_dev.size() == 1) {
      for (int ch = 0; ch < C_; ++ch) ClockShardLocked(ch, clock);
    } else {
      std::vector<std::thread> th;
      for (auto &chs : by_dev)
        th.emplace_back([this, chs, clock] {
          for (int ch : chs) ClockShardLocked(ch, clock);
        });
      for (auto &t : th) t.join();
    }
    int32_t sys = INT32_MAX;
    for (auto &s : shards_) sys = std::min(sys, s.pushed_clock);
    {
      std::lock_guard<std::mutex> g(clock_mtx_);
      system_clock_ = sys;
    }
    clock_cv_.notify_all();
  }

  void ClockShardLocked(int ch, int32_t clock) {
    {
      Shard &s = shards_[ch];
      // OpLogSerializer: tables in ascending id, empty ones omitted (oplog_serializer.hpp:12-37)
      std::vector<int32_t> ids(table_order_);
      std::sort(ids.begin(), ids.end());
      std::vector<uint8_t> payload(4, 0);
      int32_t ntab = 0;
      for (int32_t id : ids) {
        ClientTableImpl *t = tables_[id].get();
        std::vector<uint8_t> recs;
        int32_t nrows = 0;
        t->SerializeOplog(ch, C_, &recs, &nrows);
        if (!nrows) continue;
        ++ntab;
        uint8_t head[16];
        const uint64_t usz = (uint64_t)vsize_of(t->dtype());
        std::memcpy(head, &id, 4);
        std::memcpy(head + 4, &usz, 8);
        std::memcpy(head + 12, &nrows, 4);
        payload.insert(payload.end(), head, head + 16);
        payload.insert(payload.end(), recs.begin(), recs.end());
      }
      if (ntab) std::memcpy(payload.data(), &ntab, 4);
      else payload.clear();   // an empty message (abstract_bg_worker.cpp:670-682)
      // SendOpLogMsgs (abstract_bg_worker.cpp:651-689): the 41-byte header, is_clock
      psx_oplog_msg_header h{};
      h.avai_size = payload.size();
      h.is_clock = 1;
      h.client_id = cfg_.client_id;
      h.version = s.version++;
      h.bg_clock = clock;
      std::vector<uint8_t> msg(PSX_OPLOG_MSG_HEADER_BYTES + payload.size());
      psx_encode_oplog_header(&h, msg.data());
      if (!payload.empty()) std::memcpy(msg.data() + PSX_OPLOG_MSG_HEADER_BYTES, payload.data(), payload.size());
      Trace("msg", ch, msg_seq_++, msg.data(), msg.size());
      int32_t changed = 0;
      check(s.ctx, psx_handle_oplog_msg(s.ctx, msg.data(), msg.size(), s.bg_id, &changed), "HandleOpLogMsg");
      if (changed) PushLocked(ch, changed);
    }
  }

  // SSPPushServerThread::ServerPushRow + SSPPushBgWorker::ApplyServerPushedRow for this client
  void PushLocked(int ch, int32_t min_clock) {
    Shard &s = shards_[ch];
    const int C = std::max(1, cfg_.num_total_clients);
    std::vector<size_t> cap(C, 0), used(C, 0);
    psx_status st = psx_serialize_push(s.ctx, nullptr, cap.data(), used.data(), 0, 0);
    if (st != PSX_ERR_BUFFER_TOO_SMALL) check(s.ctx, st, "push size");
    std::vector<std::vector<uint8_t>> bodies(C);
    std::vector<void *> outs(C);
    for (int k = 0; k < C; ++k) {
      bodies[k].resize(std::max<size_t>(used[k], 4));
      outs[k] = bodies[k].data();
      cap[k] = bodies[k].size();
    }
    check(s.ctx, psx_serialize_push(s.ctx, outs.data(), cap.data(), used.data(), 0, 1), "push");
    std::vector<uint8_t> &mine = bodies[cfg_.client_id % C];
    mine.resize(used[cfg_.client_id % C]);
    Trace("push", ch, push_seq_++, mine.data(), mine.size());
    ApplyPushBody(mine, ch);
    s.pushed_clock = min_clock;
    SendEndOfVersionLocked(ch);
  }

  // The end-of-version records a push produced (version tables): the reference appends
  // them to the shard's serializer for the next message; they go out here as their own
  // message (is_clock false) ahead of it, which the server applies in the same order.
  void SendEndOfVersionLocked(int ch) {
    Shard &s = shards_[ch];
    std::vector<int32_t> ids(table_order_);
    std::sort(ids.begin(), ids.end());
    std::vector<uint8_t> payload(4, 0);
    int32_t ntab = 0;
    for (int32_t id : ids) {
      ClientTableImpl *t = tables_[id].get();
      if (!t->version_maintain()) continue;
      std::vector<uint8_t> recs;
      const int32_t nrows = t->TakeEndOfVersion(ch, &recs);
      if (!nrows) continue;
      ++ntab;
      uint8_t head[16];
      const uint64_t usz = (uint64_t)vsize_of(t->dtype());
      std::memcpy(head, &id, 4);
      std::memcpy(head + 4, &usz, 8);
      std::memcpy(head + 12, &nrows, 4);
      payload.insert(payload.end(), head, head + 16);
      payload.insert(payload.end(), recs.begin(), recs.end());
    }
    if (!ntab) return;
    std::memcpy(payload.data(), &ntab, 4);
    psx_oplog_msg_header h{};
    h.avai_size = payload.size();
    h.is_clock = 0;
    h.client_id = cfg_.client_id;
    h.version = s.version++;
    h.bg_clock = process_clock_;
    std::vector<uint8_t> msg(PSX_OPLOG_MSG_HEADER_BYTES + payload.size());
    psx_encode_oplog_header(&h, msg.data());
    std::memcpy(msg.data() + PSX_OPLOG_MSG_HEADER_BYTES, payload.data(), payload.size());
    Trace("msg", ch, msg_seq_++, msg.data(), msg.size());
    int32_t changed = 0;
    check(s.ctx, psx_handle_oplog_msg(s.ctx, msg.data(), msg.size(), s.bg_id, &changed), "HandleOpLogMsg (end of version)");
  }

  // SerializedRowReader walk (serialized_row_reader.hpp:30-100) over the host body
  void ApplyPushBody(const std::vector<uint8_t> &b, int ch) {
    if (b.size() < 4) return;
    size_t off = 0;
    int32_t table_id;
    std::memcpy(&table_id, b.data(), 4);
    off = 4;
    if (table_id == -2) return;
    while (off + 4 <= b.size()) {
      int32_t rid;
      std::memcpy(&rid, b.data() + off, 4);
      off += 4;
      if (rid == -1) {
        std::memcpy(&table_id, b.data() + off, 4);
        off += 4;
        continue;
      }
      if (rid == -2) return;
      uint64_t size;
      std::memcpy(&size, b.data() + off, 8);
      off += 8;
      auto it = tables_.find(table_id);
      if (it == tables_.end()) die("push for unknown table " + std::to_string(table_id));
      it->second->Reset(rid, b.data() + off, (size_t)size, ch);
      off += size;
    }
  }

  TableGroupConfig cfg_;
  int C_ = 1;

 public:
  // STATS_SERVER_ACCUM_APPLY_OPLOG_* of every shard context (psx_ctx_stats), summed
  ServerApplyStatsSum ServerApplyStats() {
    std::lock_guard<std::mutex> g(mtx_);
    ServerApplyStatsSum sum;
    for (auto &s : shards_) {
      psx_apply_stats st{};
      if (s.ctx && psx_ctx_stats(s.ctx, &st, 0) == PSX_OK) {
        sum.calls += st.calls;
        sum.messages += st.messages;
        sum.oplog_bytes += st.oplog_bytes;
        sum.settled_calls += st.settled_calls;
        sum.apply_sec += st.apply_sec;
      }
    }
    return sum;
  }

 private:
  std::vector<int32_t> devices_;
  std::vector<Shard> shards_;
  std::map<int32_t, std::unique_ptr<ClientTableImpl>> tables_;
  std::vector<int32_t> table_order_;
  int32_t staleness_ = 0;
  std::mutex mtx_;                              // bg work: oplog send, push apply, row requests
  std::map<int32_t, int32_t> thread_clock_;     // vector clock of the app threads
  int32_t next_thread_ = 0;
  int32_t process_clock_ = 0;
  std::mutex clock_mtx_;
  std::condition_variable clock_cv_;
  int32_t system_clock_ = 0;
  bool table_access_ = false;
  int32_t num_table_threads_ = 1;
  std::mutex reg_mtx_;
  std::condition_variable reg_cv_;
  int32_t reg_arrived_ = 0;
  int64_t reg_gen_ = 0;
  std::string trace_dir_;
  FILE *trace_index_ = nullptr;
  std::mutex trace_mtx_;
  std::atomic<int64_t> msg_seq_{0}, push_seq_{0}, req_seq_{0};

 public:
  static thread_local int32_t tls_thread_id_;
  static thread_local int32_t tls_clock_;
};

thread_local int32_t Runtime::tls_thread_id_ = 0;
thread_local int32_t Runtime::tls_clock_ = 0;

std::unique_ptr<Runtime> g_rt;

// ---- ClientTableImpl ------------------------------------------------------------------

AbstractRow *ClientTableImpl::Get(int32_t row_id, RowAccessor *acc) {
  if (row_id < 0 || (size_t)row_id >= cfg_.process_cache_capacity)
    die("row " + std::to_string(row_id) + " outside table " + std::to_string(id_));
  // SSPPushConsistencyController::Get (ssp_push_consistency_controller.cpp:70-120)
  const int32_t stalest = std::max(0, rt_->thread_clock() - cfg_.table_info.table_staleness);
  rt_->WaitSystemClock(stalest);
  std::shared_ptr<AbstractRow> r = Find(row_id);
  if (!r) {
    rt_->FetchRow(this, row_id);
    r = Find(row_id);
  }
  if (acc) acc->Set(r);
  return r.get();
}

void ClientTableImpl::GetAsyncForced(int32_t row_id) {
  if (!Find(row_id)) rt_->FetchRow(this, row_id);
}

void ClientTableImpl::BatchInc(int32_t row_id, const int32_t *cols, const void *u, int32_t n) {
  std::lock_guard<std::mutex> g(mtx_);
  const uint8_t *up = (const uint8_t *)u;
  if (dense_oplog_) {
    auto &op = dense_oplog_rows_[row_id];
    if (op.empty()) op.assign((size_t)oplog_cap_ * vsize_, 0);
    for (int32_t i = 0; i < n; ++i) {
      if (cols[i] < 0 || cols[i] >= oplog_cap_) die("column outside the dense row oplog");
      add_value(dtype_, op.data() + (size_t)cols[i] * vsize_, up + (size_t)i * vsize_);
    }
  } else {
    auto &op = sparse_oplog_rows_[row_id];
    for (int32_t i = 0; i < n; ++i) add_value(dtype_, (uint8_t *)&op[cols[i]], up + (size_t)i * vsize_);
  }
  // a version table's updates reach the cache only through the server
  // (SSPConsistencyController::BatchInc, ssp_consistency_controller.cpp:117-125)
  if (version_) {
    oplog_index_[row_id] = true;
    return;
  }
  auto it = cache_.find(row_id);   // the process cache sees the thread's own updates
  if (it != cache_.end()) it->second->ApplyBatchInc(cols, u, n);
}

void ClientTableImpl::DenseBatchInc(int32_t row_id, const void *u, int32_t index_st, int32_t n) {
  std::lock_guard<std::mutex> g(mtx_);
  const uint8_t *up = (const uint8_t *)u;
  if (index_st < 0 || index_st + n > oplog_cap_) die("dense batch outside the dense row oplog");
  if (dense_oplog_) {
    auto &op = dense_oplog_rows_[row_id];
    if (op.empty()) op.assign((size_t)oplog_cap_ * vsize_, 0);
    for (int32_t i = 0; i < n; ++i)
      add_value(dtype_, op.data() + (size_t)(index_st + i) * vsize_, up + (size_t)i * vsize_);
  } else {
    auto &op = sparse_oplog_rows_[row_id];
    for (int32_t i = 0; i < n; ++i) add_value(dtype_, (uint8_t *)&op[index_st + i], up + (size_t)i * vsize_);
  }
  if (version_) {
    oplog_index_[row_id] = true;
    return;
  }
  auto it = cache_.find(row_id);
  if (it != cache_.end()) it->second->ApplyDenseBatchInc(u, index_st, n);
}

// Updates not yet sent go back on top of a row the server just (re)sent
// (AbstractBgWorker::ApplyOpLogsAndInsertRow / ApplyServerPushedRow's replay,
// abstract_bg_worker.cpp:787-804); caller holds mtx_ and the row's write lock.
void ClientTableImpl::ReplayOplogLocked(int32_t row_id, AbstractRow *r) {
  if (cfg_.no_oplog_replay) return;
  auto d = dense_oplog_rows_.find(row_id);
  if (d != dense_oplog_rows_.end()) r->ApplyDenseBatchIncUnsafe(d->second.data(), 0, (int32_t)oplog_cap_);
  auto sp = sparse_oplog_rows_.find(row_id);
  if (sp != sparse_oplog_rows_.end())
    for (auto &kv : sp->second) r->ApplyIncUnsafe(kv.first, &kv.second);
}

void ClientTableImpl::Insert(int32_t row_id, const uint8_t *data, size_t size) {
  // version tables: the row bytes end with the row's uint64 version (ExtractRowVersion,
  // abstract_bg_worker.cpp:1032-1040); an inserted row leaves the oplog's version alone
  // (InsertNonexistentRow, :852-880)
  if (version_) {
    if (size < 8) die("version row reply without its version");
    size -= 8;
  }
  std::shared_ptr<AbstractRow> r(ClassRegistry<AbstractRow>::GetRegistry().CreateObject(cfg_.table_info.row_type));
  r->Init(cfg_.table_info.row_capacity);
  r->Deserialize(data, size);
  std::lock_guard<std::mutex> g(mtx_);
  r->GetWriteLock();
  ReplayOplogLocked(row_id, r.get());
  r->ReleaseWriteLock();
  cache_[row_id] = r;
}

void ClientTableImpl::Reset(int32_t row_id, const uint8_t *data, size_t size, int ch) {
  std::lock_guard<std::mutex> g(mtx_);
  uint64_t row_version = 0;
  if (version_) {
    if (size < 8) die("version row push without its version");
    size -= 8;
    std::memcpy(&row_version, data + size, 8);
  }
  auto it = cache_.find(row_id);
  if (it == cache_.end()) return;   // not cached: the reference drops it too
  AbstractRow *r = it->second.get();
  r->GetWriteLock();
  r->ResetRowData(data, size);
  ReplayOplogLocked(row_id, r);
  // UpdateExistingRow with version_maintain (abstract_bg_worker.cpp:807-823): a row that has
  // an oplog sends it now as the end of its version, then the oplog restarts empty at the
  // pushed row's version
  auto op = dense_oplog_rows_.find(row_id);
  if (version_ && op != dense_oplog_rows_.end()) {
    AppendVersionRecord(&eov_[ch], row_id, op->second, oplog_version_[row_id], true);
    ++eov_rows_[ch];
    std::fill(op->second.begin(), op->second.end(), 0);
    oplog_version_[row_id] = row_version;
  }
  r->ReleaseWriteLock();
}

// VersionDenseRowOpLog::SerializeDense: int32 row_id; V[cap]; uint64 version; bool
// end_of_version (version_dense_row_oplog.hpp:128-180)
void ClientTableImpl::AppendVersionRecord(std::vector<uint8_t> *out, int32_t row_id, const std::vector<uint8_t> &op,
                                          uint64_t version, bool end_of_version) {
  const size_t at = out->size();
  out->resize(at + 4 + op.size() + 9);
  std::memcpy(out->data() + at, &row_id, 4);
  std::memcpy(out->data() + at + 4, op.data(), op.size());
  std::memcpy(out->data() + at + 4 + op.size(), &version, 8);
  (*out)[at + 4 + op.size() + 8] = end_of_version ? 1 : 0;
}

int32_t ClientTableImpl::TakeEndOfVersion(int ch, std::vector<uint8_t> *out) {
  std::lock_guard<std::mutex> g(mtx_);
  auto it = eov_.find(ch);
  if (it == eov_.end() || it->second.empty()) return 0;
  out->insert(out->end(), it->second.begin(), it->second.end());
  it->second.clear();
  const int32_t n = eov_rows_[ch];
  eov_rows_[ch] = 0;
  return n;
}

size_t ClientTableImpl::SerializeOplog(int ch, int C, std::vector<uint8_t> *out, int32_t *num_rows) {
  std::lock_guard<std::mutex> g(mtx_);
  *num_rows = 0;
  const bool dense_ser = cfg_.table_info.oplog_dense_serialized && kind_ == PSX_ROW_DENSE;
  auto emit_sparse = [&](int32_t rid, const std::vector<std::pair<int32_t, const uint8_t *>> &nz) {
    // SerializeSparse: int32 n; int32 cols[n]; V vals[n], zeros dropped, ascending columns
    const int32_t n = (int32_t)nz.size();
    const size_t at = out->size();
    out->resize(at + 8 + (size_t)n * (4 + vsize_));
    std::memcpy(out->data() + at, &rid, 4);
    std::memcpy(out->data() + at + 4, &n, 4);
    for (int32_t i = 0; i < n; ++i) {
      std::memcpy(out->data() + at + 8 + (size_t)i * 4, &nz[i].first, 4);
      std::memcpy(out->data() + at + 8 + (size_t)n * 4 + (size_t)i * vsize_, nz[i].second, vsize_);
    }
    ++*num_rows;
  };
  if (version_) {
    // PrepareOpLogsNormalNoReplay (ssp_bg_worker.cpp:169-213): the rows in the oplog index,
    // each sent with its version and then Reset (zeroed, kept)
    for (auto it = oplog_index_.begin(); it != oplog_index_.end();) {
      if (it->first % C != ch) { ++it; continue; }
      auto &op = dense_oplog_rows_[it->first];
      AppendVersionRecord(out, it->first, op, oplog_version_[it->first], false);
      std::fill(op.begin(), op.end(), 0);
      ++*num_rows;
      it = oplog_index_.erase(it);
    }
    return out->size();
  }
  for (auto it = dense_oplog_rows_.begin(); it != dense_oplog_rows_.end();) {
    if (it->first % C != ch) { ++it; continue; }
    if (dense_ser) {   // SerializeDense: int32 row_id; V[cap] (dense_row_oplog.hpp:133-136)
      const size_t at = out->size();
      out->resize(at + 4 + it->second.size());
      std::memcpy(out->data() + at, &it->first, 4);
      std::memcpy(out->data() + at + 4, it->second.data(), it->second.size());
      ++*num_rows;
    } else {
      std::vector<std::pair<int32_t, const uint8_t *>> nz;
      for (int64_t c = 0; c < oplog_cap_; ++c)
        if (!is_zero(dtype_, it->second.data() + c * vsize_)) nz.push_back({(int32_t)c, it->second.data() + c * vsize_});
      emit_sparse(it->first, nz);   // a row whose updates cancel still sends {row_id, 0}
    }
    it = dense_oplog_rows_.erase(it);
  }
  for (auto it = sparse_oplog_rows_.begin(); it != sparse_oplog_rows_.end();) {
    if (it->first % C != ch) { ++it; continue; }
    std::vector<std::pair<int32_t, const uint8_t *>> nz;
    for (auto &kv : it->second)
      if (!is_zero(dtype_, (const uint8_t *)&kv.second)) nz.push_back({kv.first, (const uint8_t *)&kv.second});
    emit_sparse(it->first, nz);
    it = sparse_oplog_rows_.erase(it);
  }
  return out->size();
}

}  // namespace

// ---- the PSTableGroup entry points -----------------------------------------------------

int32_t Init(const TableGroupConfig &config, bool table_access) {
  if (g_rt) die("PSTableGroup::Init called twice");
  g_rt = std::make_unique<Runtime>(config, table_access);
  // the init thread's clock entry; it meets the others at WaitThreadRegister
  return table_access ? g_rt->RegisterThread(false) : config.client_id * 1000 + 200;
}
void ShutDown() { g_rt.reset(); }
bool CreateTable(int32_t table_id, const ClientTableConfig &config) { return g_rt->CreateTable(table_id, config); }
void CreateTableDone() {}
void WaitThreadRegister() { g_rt->WaitThreadRegister(); }
AbstractClientTable *GetTableOrDie(int32_t table_id) { return g_rt->table(table_id); }
int32_t RegisterThread() { return g_rt->RegisterThread(); }
void DeregisterThread() { g_rt->DeregisterThread(); }
void Clock() { g_rt->Clock(); }
void GlobalBarrier() { g_rt->GlobalBarrier(); }
ServerApplyStatsSum ServerApplyStats() { return g_rt ? g_rt->ServerApplyStats() : ServerApplyStatsSum{}; }

}  // namespace runtime
}  // namespace petuum
