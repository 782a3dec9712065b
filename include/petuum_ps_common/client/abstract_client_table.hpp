// abstract_client_table.hpp — the client table behind Table<UPDATE>
// (src/petuum_ps_common/client/abstract_client_table.hpp:17-45); implemented by the
// MI355X client runtime (parameter_server_amd/csrc/petuum_runtime.cpp).
#pragma once

#include <cstdint>

#include <petuum_ps_common/include/row_access.hpp>

namespace petuum {

class AbstractClientTable {
 public:
  virtual ~AbstractClientTable() {}

  virtual void RegisterThread() = 0;
  virtual void DeregisterThread() = 0;

  virtual void GetAsyncForced(int32_t row_id) = 0;
  virtual void GetAsync(int32_t row_id) = 0;
  virtual void WaitPendingAsyncGet() = 0;
  virtual void ThreadGet(int32_t row_id, ThreadRowAccessor *row_accessor) = 0;
  virtual void ThreadInc(int32_t row_id, int32_t column_id, const void *update) = 0;
  virtual void ThreadBatchInc(int32_t row_id, const int32_t *column_ids, const void *updates,
                              int32_t num_updates) = 0;
  virtual void ThreadDenseBatchInc(int32_t row_id, const void *updates, int32_t index_st, int32_t num_updates) = 0;
  virtual void FlushThreadCache() = 0;

  // Returns the row (kept alive by row_accessor).
  virtual AbstractRow *Get(int32_t row_id, RowAccessor *row_accessor) = 0;
  virtual void Inc(int32_t row_id, int32_t column_id, const void *update) = 0;
  virtual void BatchInc(int32_t row_id, const int32_t *column_ids, const void *updates, int32_t num_updates) = 0;
  virtual void DenseBatchInc(int32_t row_id, const void *updates, int32_t index_st, int32_t num_updates) = 0;

  virtual void Clock() = 0;
  virtual int32_t get_row_type() const = 0;
};

}  // namespace petuum
