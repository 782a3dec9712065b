// float16_compressor.hpp — Float16Compressor, the binary16 codec DenseRowFloat16 and the
// kDenseRowOpLogFloat16 oplog call (vector_store_float16.hpp:94-115,
// dense_row_oplog_float16.hpp:135-157).  The reference fetches it unpinned from the network
// (third_party/third_party.mk:281-290) and does not vendor it; this restates the published
// public-domain algorithm of that class, bit for bit the same as libpsx's device and host
// forms (psx_device.hpp f32_to_half_fc, psx_runtime.cpp) and the oracle's
// (orc_float_to_half): compress truncates the mantissa (round toward zero), makes values
// below the smallest normal half subnormal through a float x 2^37 -> int conversion,
// values above 65504 infinity, and keeps NaN payloads; decompress is exact.  Parity
// unpinned: no reference test holds a compressed value.
#pragma once

#include <cstdint>
#include <cstring>

class Float16Compressor {
 public:
  static uint16_t compress(float value) {
    const int32_t infN = 0x7F800000, maxN = 0x477FE000, minN = 0x38800000;
    const int32_t infC = infN >> 13, nanN = (infC + 1) << 13, maxC = maxN >> 13, minC = minN >> 13;
    const int32_t subC = 0x003FF, maxD = infC - maxC - 1, minD = minC - subC - 1;
    uint32_t u;
    std::memcpy(&u, &value, 4);
    uint32_t sign = u & 0x80000000u;
    int32_t v = (int32_t)(u ^ sign);
    sign >>= 16;
    float mag, mul;
    const int32_t mulN = 0x52000000;   // 2^37
    std::memcpy(&mag, &v, 4);
    std::memcpy(&mul, &mulN, 4);
    const int32_t sub = minN > v ? (int32_t)(mul * mag) : 0;
    v ^= (sub ^ v) & -(int32_t)(minN > v);
    v ^= (infN ^ v) & -(int32_t)((infN > v) & (v > maxN));
    v ^= (nanN ^ v) & -(int32_t)((nanN > v) & (v > infN));
    v = (int32_t)((uint32_t)v >> 13);
    v ^= ((v - maxD) ^ v) & -(int32_t)(v > maxC);
    v ^= ((v - minD) ^ v) & -(int32_t)(v > subC);
    return (uint16_t)(((uint32_t)v | sign) & 0xffffu);
  }

  static float decompress(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, bits;
    if (e == 0x1f) {
      bits = sign | 0x7f800000u | (m << 13);
    } else if (e != 0) {
      bits = sign | ((e + 112u) << 23) | (m << 13);
    } else if (m == 0) {
      bits = sign;
    } else {   // subnormal half: normalise
      uint32_t k = 0;
      while (!(m & 0x400u)) {
        m <<= 1;
        ++k;
      }
      bits = sign | ((113u - k) << 23) | ((m & 0x3ffu) << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
  }
};
