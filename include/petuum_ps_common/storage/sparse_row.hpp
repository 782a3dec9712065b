// sparse_row.hpp — SparseRow<V> (src/petuum_ps_common/storage/sparse_row.hpp): col -> V, zeros erased.
#pragma once
#include <petuum_ps_common/storage/numeric_store_row.hpp>

namespace petuum {

template <typename V>
class SparseRow : public NumericStoreRow<MapStore, V> {
 public:
  AbstractRow *Clone() const override {
    std::lock_guard<std::mutex> g(this->mtx_);
    auto *r = new SparseRow<V>();
    std::vector<uint8_t> b(this->store_.SerializedSize());
    this->store_.Serialize(b.data());
    r->Deserialize(b.data(), b.size());
    return r;
  }
  V operator[](int32_t col_id) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    return this->store_.Get(col_id);
  }
  void CopyToVector(std::vector<std::pair<int32_t, V>> *to) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    this->store_.Copy(to);
  }
};

}  // namespace petuum
