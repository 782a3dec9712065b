// abstract_row.hpp — the row-type plugin interface (src/petuum_ps_common/include/abstract_row.hpp:14-126).
// A row type registered with PSTableGroup::RegisterRow<ROW>(id) implements it; the client
// runtime creates rows through the registry (ClassRegistry, util/class_register.hpp) and
// applies updates and pushed rows through these virtuals.  Rows built on NumericStoreRow
// (DenseRow, SortedVectorMapRow, SparseRow) also tell the runtime how the MI355X server
// stores them (psx_row_kind / psx_dtype, include/psx.h); a row type that cannot be
// stored by the device path is rejected at CreateTable.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>
// The reference's abstract_row.hpp includes <boost/thread.hpp> (abstract_row.hpp:3), and the
// apps use boost::barrier and std::atomic through petuum_ps.hpp without including them
// (apps/lda/src/lda_engine.hpp:54-62): carried the same way where boost is installed.
#if __has_include(<boost/thread.hpp>)
#include <boost/thread.hpp>
#endif

namespace petuum {

class AbstractRow {
 public:
  AbstractRow() = default;
  AbstractRow(const AbstractRow &) = delete;
  AbstractRow &operator=(const AbstractRow &) = delete;
  virtual ~AbstractRow() {}

  virtual void Init(size_t capacity) = 0;
  virtual AbstractRow *Clone() const = 0;
  virtual size_t get_update_size() const = 0;

  // Serialized bytes: what the server pushes for this row (ServerRow::Serialize).
  virtual size_t SerializedSize() const = 0;
  virtual size_t Serialize(void *bytes) const = 0;
  virtual void Deserialize(const void *data, size_t num_bytes) = 0;
  virtual void ResetRowData(const void *data, size_t num_bytes) = 0;

  virtual void GetWriteLock() const = 0;
  virtual void ReleaseWriteLock() const = 0;

  virtual double ApplyIncGetImportance(int32_t column_id, const void *update) = 0;
  virtual double ApplyBatchIncGetImportance(const int32_t *column_ids, const void *update_batch,
                                            int32_t num_updates) = 0;
  virtual double ApplyIncUnsafeGetImportance(int32_t column_id, const void *update) = 0;
  virtual double ApplyBatchIncUnsafeGetImportance(const int32_t *column_ids, const void *update_batch,
                                                  int32_t num_updates) = 0;
  virtual void ApplyInc(int32_t column_id, const void *update) = 0;
  virtual void ApplyBatchInc(const int32_t *column_ids, const void *update_batch, int32_t num_updates) = 0;
  virtual void ApplyIncUnsafe(int32_t column_id, const void *update) = 0;
  virtual void ApplyBatchIncUnsafe(const int32_t *column_ids, const void *update_batch, int32_t num_updates) = 0;
  virtual double ApplyDenseBatchIncGetImportance(const void *update_batch, int32_t index_st,
                                                 int32_t num_updates) = 0;
  virtual void ApplyDenseBatchInc(const void *update_batch, int32_t index_st, int32_t num_updates) = 0;
  virtual double ApplyDenseBatchIncUnsafeGetImportance(const void *update_batch, int32_t index_st,
                                                       int32_t num_updates) = 0;
  virtual void ApplyDenseBatchIncUnsafe(const void *update_batch, int32_t index_st, int32_t num_updates) = 0;

  // update1 (+|-)= update2, for oplog accumulation (no Init needed).
  virtual void AddUpdates(int32_t column_id, void *update1, const void *update2) const = 0;
  virtual void SubtractUpdates(int32_t column_id, void *update1, const void *update2) const = 0;

  virtual double GetImportance(int32_t column_id, const void *update, const void *value) const = 0;
  virtual double GetImportance(int32_t column_id, const void *update) const = 0;
  virtual double GetAccumImportance(const int32_t *column_ids, const void *update_batch,
                                    int32_t num_updates) const = 0;
  virtual double GetDenseAccumImportance(const void *update_batch, int32_t index_st,
                                         int32_t num_updates) const = 0;

  virtual void InitUpdate(int32_t column_id, void *zero) const = 0;
  virtual bool CheckZeroUpdate(const void *update) const = 0;

  // MI355X server storage of this row type: psx_row_kind and psx_dtype (include/psx.h),
  // -1 when the device path cannot store it.
  virtual int32_t psx_row_kind() const { return -1; }
  virtual int32_t psx_dtype() const { return -1; }
  // 1: the row's bytes are binary16 (DenseRowFloat16: psx_table_config.row_bytes_f16)
  virtual int32_t psx_row_bytes_f16() const { return 0; }
};

}  // namespace petuum
