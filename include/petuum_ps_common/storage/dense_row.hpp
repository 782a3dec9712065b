// dense_row.hpp — DenseRow<V> (src/petuum_ps_common/storage/dense_row.hpp:16-41).
#pragma once
#include <petuum_ps_common/storage/numeric_store_row.hpp>

namespace petuum {

template <typename V>
class DenseRow : public NumericStoreRow<VectorStore, V> {
 public:
  AbstractRow *Clone() const override {
    std::lock_guard<std::mutex> g(this->mtx_);
    auto *r = new DenseRow<V>();
    std::vector<uint8_t> b(this->store_.SerializedSize());
    this->store_.Serialize(b.data());
    r->Deserialize(b.data(), b.size());
    return r;
  }
  V operator[](int32_t col_id) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    return this->store_.Get(col_id);
  }
  void CopyToVector(std::vector<V> *to) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    this->store_.CopyToVector(to);
  }
  void CopyToMem(void *to) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    this->store_.CopyToMem(to);
  }
  const void *GetDataPtr() const { return this->store_.GetDataPtr(); }
  size_t get_capacity() const { return this->store_.get_capacity(); }
};

}  // namespace petuum
