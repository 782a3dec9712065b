// sorted_vector_map_row.hpp — SortedVectorMapRow<V>
// (src/petuum_ps_common/storage/sorted_vector_map_row.hpp): entries kept in value order
// (LDA's word-topic rows).
#pragma once
#include <petuum_ps_common/storage/numeric_store_row.hpp>

namespace petuum {

template <typename V>
class SortedVectorMapRow : public NumericStoreRow<SortedVectorMapStore, V> {
 public:
  AbstractRow *Clone() const override {
    std::lock_guard<std::mutex> g(this->mtx_);
    auto *r = new SortedVectorMapRow<V>();
    std::vector<uint8_t> b(this->store_.SerializedSize());
    this->store_.Serialize(b.data());
    r->Deserialize(b.data(), b.size());
    return r;
  }
  V operator[](int32_t col_id) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    return this->store_.Get(col_id);
  }
  void CopyToVector(std::vector<Entry<V>> *to) const {
    std::lock_guard<std::mutex> g(this->mtx_);
    this->store_.CopyToVector(to);
  }
  size_t num_entries() const {
    std::lock_guard<std::mutex> g(this->mtx_);
    return this->store_.num_entries();
  }
};

}  // namespace petuum
