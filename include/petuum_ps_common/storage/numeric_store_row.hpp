// numeric_store_row.hpp — the client-side rows of the App API: a numeric row over one of
// three stores, with the reference's store semantics (the same ones the MI355X server
// kernels and the oracle implement):
//   VectorStore<V>          V[capacity], Inc adds in place            (vector_store.hpp:64-118)
//   SortedVectorMapStore<V> Entry<V>[n] kept in the reference's value order: a new key is
//                           appended and moves back past strictly smaller values, an added
//                           key stays where it is, a key reaching 0 is removed
//                                                                       (sorted_vector_map_store.hpp:175-337)
//   MapStore<V>             col -> V, a key reaching 0 is erased      (map_store.hpp:45-121)
// Serialize/Deserialize use the server's row bytes (V[cap]; Entry<V>[n]; {int32, V}[n]),
// so a pushed row resets a cached row exactly (ResetRowData, numeric_store_row.hpp:142-145).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include <petuum_ps_common/include/abstract_row.hpp>
#include <petuum_ps_common/storage/entry.hpp>

namespace petuum {

// psx_dtype (include/psx.h) of a value type: f32 0, f64 1, i32 2, i64 3.
template <typename V> struct PsxDtype { static constexpr int32_t value = -1; };
template <> struct PsxDtype<float> { static constexpr int32_t value = 0; };
template <> struct PsxDtype<double> { static constexpr int32_t value = 1; };
template <> struct PsxDtype<int32_t> { static constexpr int32_t value = 2; };
template <> struct PsxDtype<int64_t> { static constexpr int32_t value = 3; };

template <typename V>
class VectorStore {
 public:
  static constexpr int32_t kPsxKind = 0;   // PSX_ROW_DENSE
  void Init(size_t capacity) { data_.assign(capacity, V(0)); }
  size_t SerializedSize() const { return data_.size() * sizeof(V); }
  size_t Serialize(void *bytes) const {
    if (!data_.empty()) std::memcpy(bytes, data_.data(), data_.size() * sizeof(V));
    return data_.size() * sizeof(V);
  }
  void Deserialize(const void *data, size_t num_bytes) {
    data_.resize(num_bytes / sizeof(V));
    if (num_bytes) std::memcpy(data_.data(), data, num_bytes);
  }
  // VectorStore::ResetData copies over the existing row (vector_store.hpp:89-91)
  void ResetData(const void *data, size_t num_bytes) {
    if (num_bytes > data_.size() * sizeof(V)) data_.resize(num_bytes / sizeof(V));
    if (num_bytes) std::memcpy(data_.data(), data, num_bytes);
  }
  V Get(int32_t col) const { return (size_t)col < data_.size() ? data_[col] : V(0); }
  void Inc(int32_t col, V delta) { data_[col] += delta; }
  V *GetPtr(int32_t col) { return data_.data() + col; }
  size_t get_capacity() const { return data_.size(); }
  void CopyToVector(std::vector<V> *to) const { *to = data_; }
  void CopyToMem(void *to) const {
    if (!data_.empty()) std::memcpy(to, data_.data(), data_.size() * sizeof(V));
  }
  const void *GetDataPtr() const { return data_.data(); }

 private:
  std::vector<V> data_;
};

template <typename V>
class SortedVectorMapStore {
 public:
  static constexpr int32_t kPsxKind = 1;   // PSX_ROW_SORTED_MAP
  void Init(size_t capacity) {
    entries_.clear();
    entries_.reserve(capacity);
  }
  size_t SerializedSize() const { return entries_.size() * sizeof(Entry<V>); }
  size_t Serialize(void *bytes) const {
    const size_t n = entries_.size() * sizeof(Entry<V>);
    if (n) std::memcpy(bytes, entries_.data(), n);
    return n;
  }
  void Deserialize(const void *data, size_t num_bytes) {
    entries_.resize(num_bytes / sizeof(Entry<V>));
    if (num_bytes) std::memcpy(entries_.data(), data, num_bytes);
  }
  void ResetData(const void *data, size_t num_bytes) { Deserialize(data, num_bytes); }
  V Get(int32_t col) const {
    for (const auto &e : entries_)
      if (e.first == col) return e.second;
    return V(0);
  }
  void Inc(int32_t col, V delta) {
    if (delta == V(0)) return;
    size_t i = 0;
    while (i < entries_.size() && entries_[i].first != col) ++i;
    if (i == entries_.size()) {
      Entry<V> e;
      std::memset(&e, 0, sizeof(e));
      e.first = col;
      e.second = delta;
      // the new entry lands after the last entry whose value is not strictly smaller
      size_t p = entries_.size();
      while (p > 0 && entries_[p - 1].second < delta) --p;
      entries_.insert(entries_.begin() + p, e);
      return;
    }
    entries_[i].second += delta;                   // no re-sort of a found key
    if (entries_[i].second == V(0)) entries_.erase(entries_.begin() + i);
  }
  size_t num_entries() const { return entries_.size(); }
  void CopyToVector(std::vector<Entry<V>> *to) const { *to = entries_; }

 private:
  std::vector<Entry<V>> entries_;
};

template <typename V>
class MapStore {
 public:
  static constexpr int32_t kPsxKind = 2;   // PSX_ROW_MAP
  void Init(size_t) { data_.clear(); }
  size_t SerializedSize() const { return data_.size() * (sizeof(int32_t) + sizeof(V)); }
  size_t Serialize(void *bytes) const {
    uint8_t *p = static_cast<uint8_t *>(bytes);
    for (const auto &kv : data_) {
      std::memcpy(p, &kv.first, sizeof(int32_t));
      std::memcpy(p + sizeof(int32_t), &kv.second, sizeof(V));
      p += sizeof(int32_t) + sizeof(V);
    }
    return data_.size() * (sizeof(int32_t) + sizeof(V));
  }
  void Deserialize(const void *data, size_t num_bytes) {
    data_.clear();
    const uint8_t *p = static_cast<const uint8_t *>(data);
    for (size_t k = 0; k < num_bytes / (sizeof(int32_t) + sizeof(V)); ++k) {
      int32_t c;
      V v;
      std::memcpy(&c, p, sizeof(c));
      std::memcpy(&v, p + sizeof(c), sizeof(V));
      data_[c] = v;
      p += sizeof(int32_t) + sizeof(V);
    }
  }
  void ResetData(const void *data, size_t num_bytes) { Deserialize(data, num_bytes); }
  V Get(int32_t col) const {
    auto it = data_.find(col);
    return it == data_.end() ? V(0) : it->second;
  }
  void Inc(int32_t col, V delta) {
    V &x = data_[col];
    x += delta;
    if (x == V(0)) data_.erase(col);
  }
  void Copy(std::vector<std::pair<int32_t, V>> *to) const { to->assign(data_.begin(), data_.end()); }

 private:
  std::map<int32_t, V> data_;
};

// NumericStoreRow<Store, V>: the AbstractRow every numeric row type shares.  Importance
// is NSSumImpCalc's (ns_sum_imp_calc.hpp:42-98): dense sum |u/v| (|u| where v = 0),
// sparse sum |u|.
template <template <typename> class StoreType, typename V>
class NumericStoreRow : public AbstractRow {
 public:
  void Init(size_t capacity) override { store_.Init(capacity); }
  size_t get_update_size() const override { return sizeof(V); }
  size_t SerializedSize() const override { return store_.SerializedSize(); }
  size_t Serialize(void *bytes) const override { return store_.Serialize(bytes); }
  void Deserialize(const void *data, size_t num_bytes) override { store_.Deserialize(data, num_bytes); }
  void ResetRowData(const void *data, size_t num_bytes) override { store_.ResetData(data, num_bytes); }
  void GetWriteLock() const override { mtx_.lock(); }
  void ReleaseWriteLock() const override { mtx_.unlock(); }

  double ApplyIncGetImportance(int32_t c, const void *u) override {
    std::lock_guard<std::mutex> g(mtx_);
    return ApplyIncUnsafeGetImportance(c, u);
  }
  double ApplyBatchIncGetImportance(const int32_t *c, const void *u, int32_t n) override {
    std::lock_guard<std::mutex> g(mtx_);
    return ApplyBatchIncUnsafeGetImportance(c, u, n);
  }
  double ApplyIncUnsafeGetImportance(int32_t c, const void *u) override {
    const V d = *static_cast<const V *>(u);
    store_.Inc(c, d);
    return std::fabs((double)d);
  }
  double ApplyBatchIncUnsafeGetImportance(const int32_t *c, const void *u, int32_t n) override {
    double imp = 0;
    for (int32_t i = 0; i < n; ++i) imp += ApplyIncUnsafeGetImportance(c[i], static_cast<const V *>(u) + i);
    return imp;
  }
  void ApplyInc(int32_t c, const void *u) override { ApplyIncGetImportance(c, u); }
  void ApplyBatchInc(const int32_t *c, const void *u, int32_t n) override { ApplyBatchIncGetImportance(c, u, n); }
  void ApplyIncUnsafe(int32_t c, const void *u) override { ApplyIncUnsafeGetImportance(c, u); }
  void ApplyBatchIncUnsafe(const int32_t *c, const void *u, int32_t n) override {
    ApplyBatchIncUnsafeGetImportance(c, u, n);
  }
  double ApplyDenseBatchIncGetImportance(const void *u, int32_t st, int32_t n) override {
    std::lock_guard<std::mutex> g(mtx_);
    return ApplyDenseBatchIncUnsafeGetImportance(u, st, n);
  }
  void ApplyDenseBatchInc(const void *u, int32_t st, int32_t n) override {
    ApplyDenseBatchIncGetImportance(u, st, n);
  }
  double ApplyDenseBatchIncUnsafeGetImportance(const void *u, int32_t st, int32_t n) override {
    const V *d = static_cast<const V *>(u);
    double imp = 0;
    for (int32_t i = 0; i < n; ++i) {
      const double old = (double)store_.Get(st + i);
      imp += std::fabs(old == 0.0 ? (double)d[i] : (double)d[i] / old);
      store_.Inc(st + i, d[i]);
    }
    return imp;
  }
  void ApplyDenseBatchIncUnsafe(const void *u, int32_t st, int32_t n) override {
    ApplyDenseBatchIncUnsafeGetImportance(u, st, n);
  }

  void AddUpdates(int32_t, void *u1, const void *u2) const override {
    *static_cast<V *>(u1) += *static_cast<const V *>(u2);
  }
  void SubtractUpdates(int32_t, void *u1, const void *u2) const override {
    *static_cast<V *>(u1) -= *static_cast<const V *>(u2);
  }
  double GetImportance(int32_t, const void *u, const void *v) const override {
    const double x = (double)*static_cast<const V *>(v), d = (double)*static_cast<const V *>(u);
    return std::fabs(x == 0.0 ? d : d / x);
  }
  double GetImportance(int32_t c, const void *u) const override {
    const V v = store_.Get(c);
    return GetImportance(c, u, &v);
  }
  double GetAccumImportance(const int32_t *c, const void *u, int32_t n) const override {
    double imp = 0;
    for (int32_t i = 0; i < n; ++i) imp += GetImportance(c[i], static_cast<const V *>(u) + i);
    return imp;
  }
  double GetDenseAccumImportance(const void *u, int32_t st, int32_t n) const override {
    double imp = 0;
    for (int32_t i = 0; i < n; ++i) imp += GetImportance(st + i, static_cast<const V *>(u) + i);
    return imp;
  }
  void InitUpdate(int32_t, void *zero) const override { *static_cast<V *>(zero) = V(0); }
  bool CheckZeroUpdate(const void *u) const override { return *static_cast<const V *>(u) == V(0); }

  int32_t psx_row_kind() const override { return StoreType<V>::kPsxKind; }
  int32_t psx_dtype() const override { return PsxDtype<V>::value; }

 protected:
  mutable std::mutex mtx_;
  StoreType<V> store_;
};

}  // namespace petuum
