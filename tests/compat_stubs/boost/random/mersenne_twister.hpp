// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
#include <cstdint>
namespace boost {
class mt19937 {
 public:
  typedef uint32_t result_type;
  mt19937();
  explicit mt19937(uint32_t seed);
  void seed(uint32_t s);
  result_type operator()();
  static constexpr result_type min() { return 0; }
  static constexpr result_type max() { return 0xffffffffu; }
};
namespace random { using boost::mt19937; }
}  // namespace boost
