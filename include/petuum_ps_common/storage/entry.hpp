// entry.hpp — Entry<V>{first, second} of sorted/map rows (src/petuum_ps_common/storage/entry.hpp:16-20);
// its C++ layout (8 bytes, or 16 with 4 pad bytes for 8-byte V) is the serialized row format.
#pragma once
#include <cstdint>

namespace petuum {

template <typename V>
struct Entry {
  int32_t first;
  V second;
};

}  // namespace petuum
