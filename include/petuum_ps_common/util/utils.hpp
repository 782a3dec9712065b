// utils.hpp — the string-to-config helpers petuum_ps.hpp pulls in (src/petuum_ps_common/util/utils.hpp,
// utils.cpp:55-171): apps and their flag parsing turn gflags strings into TableGroupConfig /
// TableInfo enums with these.  An unknown name aborts, as the reference's LOG(FATAL) does.
// GetHostInfos / GetServerIDsFromHostMap read the machine file InitTableGroupConfig names
// (--hostfile); the hosts are recorded in the config, the ZeroMQ transport that would
// connect them is out of scope — shards are contexts in this process.
#pragma once

#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <string>
#include <vector>

#include <petuum_ps_common/include/configs.hpp>

namespace petuum {
namespace utils_detail {
[[noreturn]] inline void fatal(const char *what, const std::string &name) {
  std::fprintf(stderr, "petuum: unknown %s \"%s\"\n", what, name.c_str());
  std::abort();
}
}  // namespace utils_detail

// One "id ip port" line per host (utils.cpp:15-35); a missing file leaves the map empty.
inline void GetHostInfos(std::string server_file, std::map<int32_t, HostInfo> *host_map) {
  std::ifstream input(server_file.c_str());
  std::string line;
  while (std::getline(input, line)) {
    const size_t pos = line.find_first_of("\t ");
    const size_t pos_ip = line.find_first_of("\t ", pos + 1);
    const int32_t id = std::atoi(line.substr(0, pos).c_str());
    host_map->insert(std::make_pair(id, HostInfo(id, line.substr(pos + 1, pos_ip - pos - 1),
                                                 line.substr(pos_ip + 1))));
  }
}

// Every host but the name node (id 0), in id order (utils.cpp:38-52).
inline void GetServerIDsFromHostMap(std::vector<int32_t> *server_ids, const std::map<int32_t, HostInfo> &host_map) {
  server_ids->clear();
  for (const auto &h : host_map)
    if (h.first != 0) server_ids->push_back(h.first);
}

inline UpdateSortPolicy GetUpdateSortPolicy(const std::string &p) {
  if (p == "Random") return Random;
  if (p == "FIFO") return FIFO;
  if (p == "RelativeMagnitude") return RelativeMagnitude;
  if (p == "FIFO_N_RegMag") return FIFO_N_ReMag;   // the reference's spelling of the flag value (utils.cpp:62)
  if (p == "FixedOrder") return FixedOrder;
  utils_detail::fatal("update sort policy", p);
}

inline ConsistencyModel GetConsistencyModel(const std::string &m) {
  if (m == "SSPPush") return SSPPush;
  if (m == "SSP") return SSP;
  if (m == "SSPAggr") return SSPAggr;
  utils_detail::fatal("consistency model", m);
}

inline OpLogType GetOpLogType(const std::string &t) {
  if (t == "Sparse") return Sparse;
  if (t == "AppendOnly") return AppendOnly;
  if (t == "Dense") return Dense;
  utils_detail::fatal("oplog type", t);
}

inline AppendOnlyOpLogType GetAppendOnlyOpLogType(const std::string &t) {
  if (t == "Inc") return Inc;
  if (t == "BatchInc") return BatchInc;
  if (t == "DenseBatchInc") return DenseBatchInc;
  utils_detail::fatal("append-only oplog type", t);
}

inline ProcessStorageType GetProcessStroageType(const std::string &t) {   // (sic), utils.hpp:33
  if (t == "BoundedDense") return BoundedDense;
  if (t == "BoundedSparse") return BoundedSparse;
  utils_detail::fatal("process storage type", t);
}

// +-inf -> +-FLT_MAX (utils.cpp:137-147); RestoreInfNaN also maps NaN to 0.01 (:149-160).
inline float RestoreInf(float x) { return std::isinf(x) ? (x > 0 ? FLT_MAX : -FLT_MAX) : x; }
inline float RestoreInfNaN(float x) { return std::isnan(x) ? 0.01f : RestoreInf(x); }

}  // namespace petuum
