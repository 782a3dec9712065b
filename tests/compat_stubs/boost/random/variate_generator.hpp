// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
namespace boost {
template <class Engine, class Distribution>
class variate_generator {
 public:
  typedef typename Distribution::result_type result_type;
  variate_generator(Engine e, Distribution d);
  result_type operator()();
};
}  // namespace boost
