// Declaration stub of glog for tests/test_app_compile.py only (`g++ -fsyntax-only` of the
// reference's app sources against include/).  Not shipped, not linked.
#pragma once
#include <ostream>

namespace google {
void InitGoogleLogging(const char *argv0);
void InstallFailureSignalHandler();
extern int COUNTER;   // LOG_EVERY_N's occurrence count
struct PsxStubLog {
  std::ostream &stream();
};
}  // namespace google

#define LOG(severity) ::google::PsxStubLog().stream()
#define VLOG(level) ::google::PsxStubLog().stream()
#define LOG_IF(severity, cond) ::google::PsxStubLog().stream()
#define LOG_EVERY_N(severity, n) ::google::PsxStubLog().stream()
#define DLOG(severity) ::google::PsxStubLog().stream()
#define CHECK(cond) ((void)(cond), ::google::PsxStubLog().stream())
#define PSX_STUB_CHECK2_(a, b) ((void)(a), (void)(b), ::google::PsxStubLog().stream())
#define CHECK_EQ(a, b) PSX_STUB_CHECK2_(a, b)
#define CHECK_NE(a, b) PSX_STUB_CHECK2_(a, b)
#define CHECK_LT(a, b) PSX_STUB_CHECK2_(a, b)
#define CHECK_LE(a, b) PSX_STUB_CHECK2_(a, b)
#define CHECK_GT(a, b) PSX_STUB_CHECK2_(a, b)
#define CHECK_GE(a, b) PSX_STUB_CHECK2_(a, b)
#define CHECK_NOTNULL(p) (p)
#define DCHECK(cond) CHECK(cond)
#define DCHECK_EQ(a, b) CHECK_EQ(a, b)
#define DCHECK_NE(a, b) CHECK_NE(a, b)
#define DCHECK_LT(a, b) CHECK_LT(a, b)
#define DCHECK_LE(a, b) CHECK_LE(a, b)
#define DCHECK_GT(a, b) CHECK_GT(a, b)
#define DCHECK_GE(a, b) CHECK_GE(a, b)
