// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
namespace boost {
namespace math {
template <class T> T lgamma(T x);
template <class T> T digamma(T x);
template <class T> T tgamma(T x);
}  // namespace math
}  // namespace boost
