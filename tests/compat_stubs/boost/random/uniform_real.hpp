// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
namespace boost {
template <class T = double>
class uniform_real {
 public:
  typedef T result_type;
  typedef T input_type;
  explicit uniform_real(T lo = T(0), T hi = T(1));
  template <class Engine> T operator()(Engine &e);
};
}  // namespace boost
