// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
#include <unordered_map>
namespace boost {
template <class K, class V, class H = std::hash<K>, class E = std::equal_to<K>>
using unordered_map = std::unordered_map<K, V, H, E>;
}  // namespace boost
