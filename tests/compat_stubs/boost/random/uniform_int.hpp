// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
namespace boost {
template <class T = int>
class uniform_int {
 public:
  typedef T result_type;
  typedef T input_type;
  explicit uniform_int(T lo = 0, T hi = 9);
  template <class Engine> T operator()(Engine &e);
};
}  // namespace boost
