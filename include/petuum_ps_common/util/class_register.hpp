// class_register.hpp — ClassRegistry<BaseClass> (src/petuum_ps_common/util/class_register.hpp:13-57):
// the row-type plugin registry.  PSTableGroup::RegisterRow<ROW>(id) adds a creator for ROW
// under id; tables create their rows from TableInfo.row_type through it.
#pragma once

#include <cstdint>
#include <map>
#include <mutex>

namespace petuum {

template <typename BaseClass, typename ImplClass>
BaseClass *CreateObj() {
  return new ImplClass;
}

template <typename BaseClass>
class ClassRegistry {
 public:
  typedef BaseClass *(*CreateFunc)();

  static ClassRegistry<BaseClass> &GetRegistry() {
    static ClassRegistry<BaseClass> registry;
    return registry;
  }

  void AddCreator(int32_t key, CreateFunc creator) {
    std::lock_guard<std::mutex> g(mtx_);
    creators_[key] = creator;
  }

  void SetDefaultCreator(CreateFunc creator) { default_creator_ = creator; }

  // nullptr for an unknown key without a default creator
  BaseClass *CreateObject(int32_t key) {
    std::lock_guard<std::mutex> g(mtx_);
    auto it = creators_.find(key);
    if (it != creators_.end()) return it->second();
    return default_creator_ ? default_creator_() : nullptr;
  }

  bool Has(int32_t key) {
    std::lock_guard<std::mutex> g(mtx_);
    return creators_.count(key) != 0;
  }

 private:
  std::mutex mtx_;
  std::map<int32_t, CreateFunc> creators_;
  CreateFunc default_creator_ = nullptr;
};

}  // namespace petuum
