// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
namespace boost {
class noncopyable {
 protected:
  noncopyable() {}
  ~noncopyable() {}
 private:
  noncopyable(const noncopyable &);
  noncopyable &operator=(const noncopyable &);
};
}  // namespace boost
