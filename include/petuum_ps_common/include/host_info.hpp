// host_info.hpp — one line of a machine file (id ip port), src/petuum_ps_common/include/host_info.hpp.
#pragma once
#include <cstdint>
#include <string>

namespace petuum {

struct HostInfo {
  HostInfo() = default;
  HostInfo(int32_t id_, std::string ip_, std::string port_) : id(id_), ip(std::move(ip_)), port(std::move(port_)) {}
  int32_t id = 0;
  std::string ip;
  std::string port;
};

}  // namespace petuum
