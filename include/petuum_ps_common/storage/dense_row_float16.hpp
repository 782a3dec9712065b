// dense_row_float16.hpp — DenseRowFloat16<V> (src/petuum_ps_common/storage/dense_row_float16.hpp:13
// of the reference), the row type apps/matrixfact's matrixfact_split16 registers
// (matrixfact_split16.cpp:47,560): values held and updated as V (float), the row's bytes
// binary16 — VectorStoreFloat16 (vector_store_float16.hpp:67-135) serializes every value
// through Float16Compressor::compress and resets from pushed rows through decompress.
// The MI355X server stores these rows as f32 and serves them in the same binary16 bytes
// (psx_table_config.row_bytes_f16; psx_serve.hip).  Float16Compressor lives in an
// unvendored third-party header (third_party/third_party.mk:281-290, no pinned version):
// float16_compressor.hpp here restates its published algorithm; parity unpinned.
#pragma once

#include <petuum_ps_common/storage/numeric_store_row.hpp>
#include <petuum_ps_common/util/float16_compressor.hpp>

namespace petuum {

// V must be float (vector_store_float16.hpp:12).  Init zeroes the row.
template <typename V>
class VectorStoreFloat16 {
 public:
  static constexpr int32_t kPsxKind = 0;   // PSX_ROW_DENSE (f32 on the server)
  void Init(size_t capacity) { data_.assign(capacity, V(0)); }
  size_t SerializedSize() const { return data_.size() * sizeof(uint16_t); }
  size_t Serialize(void *bytes) const {
    uint16_t *typed = static_cast<uint16_t *>(bytes);
    for (size_t i = 0; i < data_.size(); ++i) typed[i] = Float16Compressor::compress(data_[i]);
    return data_.size() * sizeof(uint16_t);
  }
  void Deserialize(const void *data, size_t num_bytes) {
    data_.resize(num_bytes / sizeof(uint16_t));
    ResetData(data, num_bytes);
  }
  // ResetData decompresses over the existing row (vector_store_float16.hpp:110-115)
  void ResetData(const void *data, size_t num_bytes) {
    const uint16_t *typed = static_cast<const uint16_t *>(data);
    const size_t n = std::min(data_.size(), num_bytes / sizeof(uint16_t));
    for (size_t i = 0; i < n; ++i) data_[i] = Float16Compressor::decompress(typed[i]);
  }
  V Get(int32_t col) const { return (size_t)col < data_.size() ? data_[col] : V(0); }
  void Inc(int32_t col, V delta) { data_[col] += delta; }
  V *GetPtr(int32_t col) { return data_.data() + col; }
  size_t get_capacity() const { return data_.size(); }
  void Copy(std::vector<V> *to) const { *to = data_; }
  void CopyToVector(std::vector<V> *to) const { *to = data_; }
  const void *GetDataPtr() const { return data_.data(); }

 private:
  std::vector<V> data_;
};

template <typename V>
using DenseRowFloat16Core = NumericStoreRow<VectorStoreFloat16, V>;

template <typename V>
class DenseRowFloat16 : public DenseRowFloat16Core<V> {
 public:
  DenseRowFloat16() {}
  ~DenseRowFloat16() {}

  AbstractRow *Clone() const override {
    std::lock_guard<std::mutex> g(this->mtx_);
    auto *r = new DenseRowFloat16<V>();
    r->store_ = this->store_;
    return r;
  }

  V operator[](int32_t col_id) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    return this->store_.Get(col_id);
  }

  // Bulk read.  Thread-safe.
  void CopyToVector(std::vector<V> *to) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    this->store_.Copy(to);
  }

  // not thread-safe
  const void *GetDataPtr() const { return this->store_.GetDataPtr(); }

  int32_t psx_row_bytes_f16() const override { return 1; }
};

}  // namespace petuum
