// constants.hpp — the petuum_ps constants apps include
// (src/petuum_ps_common/include/constants.hpp:1-17 of the reference): same names and values.
// kMaxPendingMsgs / kMaxPendingAcks bound the reference's message tracker (flow control,
// msg_tracker.cpp); the MI355X runtime hands messages to its shards in-process and does not
// use them.
#pragma once

#include <cstddef>
#include <cstdint>

namespace petuum {

const size_t kNumBitsPerByte = 8;
const size_t k1_Mi = 1024 * 1024;
const size_t k1_Ki = 1024;
const float kCuckooExpansionFactor = 1.428;

const size_t kOneThousand = 1000;

const uint64_t kMaxPendingMsgs = 200;
const uint64_t kMaxPendingAcks = 40;

}  // namespace petuum
