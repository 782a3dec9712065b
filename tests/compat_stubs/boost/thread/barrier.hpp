// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps).
#pragma once
namespace boost {
class barrier {
 public:
  explicit barrier(unsigned int count);
  bool wait();
};
}  // namespace boost
