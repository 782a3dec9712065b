// Declaration stub of gflags for tests/test_app_compile.py only: enough for the
// reference's app sources to pass `g++ -fsyntax-only` against include/.  Not shipped, not
// linked, not a gflags implementation.
#pragma once
#include <cstdint>
#include <string>

#define PSX_STUB_FLAG_(type, name) extern type FLAGS_##name
#define DECLARE_int32(name) PSX_STUB_FLAG_(int32_t, name)
#define DECLARE_int64(name) PSX_STUB_FLAG_(int64_t, name)
#define DECLARE_uint32(name) PSX_STUB_FLAG_(uint32_t, name)
#define DECLARE_uint64(name) PSX_STUB_FLAG_(uint64_t, name)
#define DECLARE_bool(name) PSX_STUB_FLAG_(bool, name)
#define DECLARE_double(name) PSX_STUB_FLAG_(double, name)
#define DECLARE_string(name) PSX_STUB_FLAG_(std::string, name)
#define DEFINE_int32(name, v, help) int32_t FLAGS_##name = (v)
#define DEFINE_int64(name, v, help) int64_t FLAGS_##name = (v)
#define DEFINE_uint32(name, v, help) uint32_t FLAGS_##name = (v)
#define DEFINE_uint64(name, v, help) uint64_t FLAGS_##name = (v)
#define DEFINE_bool(name, v, help) bool FLAGS_##name = (v)
#define DEFINE_double(name, v, help) double FLAGS_##name = (v)
#define DEFINE_string(name, v, help) std::string FLAGS_##name = (v)

#include <vector>
namespace google {
struct CommandLineFlagInfo {
  std::string name, type, description, current_value, default_value, filename;
  bool has_validator_fn = false;
  bool is_default = true;
};
void GetAllFlags(std::vector<CommandLineFlagInfo> *out);
void ParseCommandLineFlags(int *argc, char ***argv, bool remove_flags);
void SetUsageMessage(const std::string &usage);
void ShutDownCommandLineFlags();
}  // namespace google
namespace gflags = google;
