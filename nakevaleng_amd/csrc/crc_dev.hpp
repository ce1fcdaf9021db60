// crc_dev.hpp -- CRC-32/IEEE (Go hash/crc32 ChecksumIEEE: reflected, poly
// 0xEDB88320, init and final XOR 0xFFFFFFFF) building blocks shared by the
// checksum kernels (crc.hip) and the leaf kernel's verify form (kernels.hip).
// Slicing-by-4: one 32-bit little-endian word per step, four lookups into
// 256-entry tables that the kernels stage in LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nkv {

struct CrcTables {
    uint32_t t[4][256];
};

constexpr CrcTables make_crc_tables() {
    CrcTables r{};
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
        r.t[0][i] = c;
    }
    for (int k = 1; k < 4; ++k)
        for (uint32_t i = 0; i < 256; ++i) r.t[k][i] = (r.t[k - 1][i] >> 8) ^ r.t[0][r.t[k - 1][i] & 0xFFu];
    return r;
}

// tab: this lane's copy (LDS base + lane % C), C copies interleaved
template <int C>
__device__ __forceinline__ uint32_t crc_lut(const uint32_t* tab, int k, uint32_t e) {
    return tab[(uint32_t(k) * 256u + e) * C];
}

template <int C>
__device__ __forceinline__ uint32_t crc_word(uint32_t crc, uint32_t w, const uint32_t* tab) {
    const uint32_t x = crc ^ w;
    return crc_lut<C>(tab, 3, x & 0xFFu) ^ crc_lut<C>(tab, 2, (x >> 8) & 0xFFu) ^
           crc_lut<C>(tab, 1, (x >> 16) & 0xFFu) ^ crc_lut<C>(tab, 0, x >> 24);
}

template <int C>
__device__ __forceinline__ uint32_t crc_byte(uint32_t crc, uint32_t b, const uint32_t* tab) {
    return crc_lut<C>(tab, 0, (crc ^ b) & 0xFFu) ^ (crc >> 8);
}

}  // namespace nkv
