// table.hpp — UpdateBatch, DenseUpdateBatch and Table<UPDATE>, the app-facing table API
// (src/petuum_ps_common/include/table.hpp:18-193).  Table is a light handle on the
// client table the runtime created (PSTableGroup::GetTableOrDie).
#pragma once

#include <cstdint>
#include <vector>

#include <petuum_ps_common/client/abstract_client_table.hpp>
#include <petuum_ps_common/include/row_access.hpp>

namespace petuum {

// A sparse batch of (column, update) pairs for one row.
template <typename UPDATE>
class UpdateBatch {
 public:
  UpdateBatch() = default;
  explicit UpdateBatch(size_t num_updates) : col_ids_(num_updates), updates_(num_updates) {}

  void Update(int32_t column_id, const UPDATE &update) {
    col_ids_.push_back(column_id);
    updates_.push_back(update);
  }
  void UpdateSet(int32_t idx, int32_t column_id, const UPDATE &update) {
    col_ids_[idx] = column_id;
    updates_[idx] = update;
  }
  const std::vector<int32_t> &GetColIDs() const { return col_ids_; }
  const UPDATE *GetUpdates() const { return updates_.data(); }
  int32_t GetBatchSize() const { return (int32_t)updates_.size(); }

 private:
  std::vector<int32_t> col_ids_;
  std::vector<UPDATE> updates_;
};

// Updates for the consecutive columns [index_st, index_st + num_updates); not initialized.
template <typename UPDATE>
class DenseUpdateBatch {
 public:
  DenseUpdateBatch(int32_t index_st, int32_t num_updates)
      : index_st_(index_st), num_updates_(num_updates), updates_(num_updates) {}

  UPDATE &operator[](int32_t index) { return updates_[index - index_st_]; }
  void *get_mem() { return updates_.data(); }
  const void *get_mem_const() const { return updates_.data(); }
  int32_t get_index_st() const { return index_st_; }
  int32_t get_num_updates() const { return num_updates_; }

 private:
  int32_t index_st_;
  int32_t num_updates_;
  std::vector<UPDATE> updates_;
};

template <typename UPDATE>
class Table {
 public:
  Table() = default;
  explicit Table(AbstractClientTable *system_table) : system_table_(system_table) {}

  void GetAsyncForced(int32_t row_id) { system_table_->GetAsyncForced(row_id); }
  void GetAsync(int32_t row_id) { system_table_->GetAsync(row_id); }
  void WaitPendingAsyncGet() { system_table_->WaitPendingAsyncGet(); }
  void ThreadGet(int32_t row_id, ThreadRowAccessor *row_accessor) { system_table_->ThreadGet(row_id, row_accessor); }
  void ThreadInc(int32_t row_id, int32_t column_id, UPDATE update) {
    system_table_->ThreadInc(row_id, column_id, &update);
  }
  void ThreadBatchInc(int32_t row_id, const UpdateBatch<UPDATE> &b) {
    system_table_->ThreadBatchInc(row_id, b.GetColIDs().data(), b.GetUpdates(), b.GetBatchSize());
  }
  void ThreadDenseBatchInc(int32_t row_id, const DenseUpdateBatch<UPDATE> &b) {
    system_table_->ThreadDenseBatchInc(row_id, b.get_mem_const(), b.get_index_st(), b.get_num_updates());
  }
  void FlushThreadCache() { system_table_->FlushThreadCache(); }

  // row_accessor keeps the cached row alive while it is read
  void Get(int32_t row_id, RowAccessor *row_accessor) { system_table_->Get(row_id, row_accessor); }

  template <typename ROW>
  const ROW &Get(int32_t row_id, RowAccessor *row_accessor = nullptr) {
    return *static_cast<ROW *>(system_table_->Get(row_id, row_accessor));
  }

  void Inc(int32_t row_id, int32_t column_id, UPDATE update) { system_table_->Inc(row_id, column_id, &update); }
  void BatchInc(int32_t row_id, const UpdateBatch<UPDATE> &b) {
    system_table_->BatchInc(row_id, b.GetColIDs().data(), b.GetUpdates(), b.GetBatchSize());
  }
  void DenseBatchInc(int32_t row_id, const DenseUpdateBatch<UPDATE> &b) {
    system_table_->DenseBatchInc(row_id, b.get_mem_const(), b.get_index_st(), b.get_num_updates());
  }
  int32_t get_row_type() const { return system_table_->get_row_type(); }

 private:
  AbstractClientTable *system_table_ = nullptr;
};

}  // namespace petuum
