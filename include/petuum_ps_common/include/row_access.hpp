// row_access.hpp — RowAccessor / ThreadRowAccessor (src/petuum_ps_common/include/row_access.hpp):
// a reference-counted handle keeping a cached row alive while the app reads it.
#pragma once

#include <memory>

#include <petuum_ps_common/include/abstract_row.hpp>

namespace petuum {

class RowAccessor {
 public:
  RowAccessor() = default;
  RowAccessor(const RowAccessor &) = delete;
  RowAccessor &operator=(const RowAccessor &) = delete;
  ~RowAccessor() { Clear(); }

  // Valid for the lifetime of this accessor.
  template <typename ROW>
  const ROW &Get() {
    return *static_cast<ROW *>(row_.get());
  }

  // runtime side
  void Set(std::shared_ptr<AbstractRow> row) { row_ = std::move(row); }
  void Clear() { row_.reset(); }
  AbstractRow *GetRowData() { return row_.get(); }

 private:
  std::shared_ptr<AbstractRow> row_;
};

class ThreadRowAccessor {
 public:
  ThreadRowAccessor() = default;
  ThreadRowAccessor(const ThreadRowAccessor &) = delete;
  ThreadRowAccessor &operator=(const ThreadRowAccessor &) = delete;

  template <typename ROW>
  const ROW &Get() {
    return *static_cast<ROW *>(row_.get());
  }

  void Set(std::shared_ptr<AbstractRow> row) { row_ = std::move(row); }

 private:
  std::shared_ptr<AbstractRow> row_;
};

}  // namespace petuum
