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

// a ^ b ^ c in one v_bitop3_b32 (the backend leaves xor chains as two-input v_xor)
__device__ __forceinline__ uint32_t crc_xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// The same step carried in x = crc ^ w form: from this word's x and the next
// word, the next x (six VALU: four byte indices, two three-input XORs, and no
// separate crc ^ w); crc_x_last gives the crc after the last word.
template <int C>
__device__ __forceinline__ uint32_t crc_x_next(uint32_t x, uint32_t w_next, const uint32_t* tab) {
    return crc_xor3(crc_xor3(crc_lut<C>(tab, 3, x & 0xFFu), crc_lut<C>(tab, 2, (x >> 8) & 0xFFu),
                     crc_lut<C>(tab, 1, (x >> 16) & 0xFFu)),
                crc_lut<C>(tab, 0, x >> 24), w_next);
}
template <int C>
__device__ __forceinline__ uint32_t crc_x_last(uint32_t x, const uint32_t* tab) {
    return crc_xor3(crc_lut<C>(tab, 3, x & 0xFFu), crc_lut<C>(tab, 2, (x >> 8) & 0xFFu),
                crc_lut<C>(tab, 1, (x >> 16) & 0xFFu)) ^
           crc_lut<C>(tab, 0, x >> 24);
}

// 16 little-endian words (one 64-byte block) in x form
template <int C>
__device__ __forceinline__ uint32_t crc_block16(uint32_t crc, const uint32_t w[16], const uint32_t* tab) {
    uint32_t x = crc ^ w[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) x = crc_x_next<C>(x, w[i], tab);
    return crc_x_last<C>(x, tab);
}

template <int C>
__device__ __forceinline__ uint32_t crc_quad(uint32_t crc, uint4 v, const uint32_t* tab) {
    return crc_x_last<C>(crc_x_next<C>(crc_x_next<C>(crc_x_next<C>(crc ^ v.x, v.y, tab), v.z, tab), v.w, tab), tab);
}

template <int C>
__device__ __forceinline__ uint32_t crc_byte(uint32_t crc, uint32_t b, const uint32_t* tab) {
    return crc_lut<C>(tab, 0, (crc ^ b) & 0xFFu) ^ (crc >> 8);
}

__device__ __forceinline__ uint32_t crc_wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, uint32_t(__shfl_xor(int(v), o)));
    return __builtin_amdgcn_readfirstlane(v);
}

// CRC-32/IEEE of [s, s + len) (finalised).  Every lane of the wave calls it
// (dead lanes with len 0).
// SW: the word steps run in the byte-swapped domain against swtab (slot k =
// bswap(T[3 - k]), k_leaf_verify's layout); tab then needs only T[0] (bytes).
template <int C, bool SW = false>
__device__ __forceinline__ uint32_t crc_span(const uint8_t* s, uint64_t len, const uint32_t* tab,
                                             const uint32_t* swtab = nullptr) {
    uint32_t crc = 0xFFFFFFFFu;
    const uint64_t sa = uint64_t(reinterpret_cast<uintptr_t>(s));
    const uint64_t ea = sa + len;
    const uint64_t s4 = (sa + 3) & ~uint64_t(3);
    const uint64_t e4 = ea & ~uint64_t(3);
    const uint64_t hb = s4 < ea ? s4 : ea;
    for (uint64_t a = sa; a < hb; ++a) crc = crc_byte<C>(crc, s[a - sa], tab);
    const uint64_t A = s4 & ~uint64_t(63);
    const uint32_t nch = e4 > s4 ? uint32_t((e4 - A + 63) >> 6) : 0u;
    const uint32_t nmax = crc_wave_max(nch);
    // s + (A - sa): stays a global pointer (no integer-to-pointer cast)
    const uint4* q = reinterpret_cast<const uint4*>(s + (A - sa));
    for (uint32_t c = 0; c < nmax; ++c) {
        if (c < nch) {
            uint4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = q[4 * c + i];
            const uint32_t w[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                                    v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
            const uint64_t b0 = A + 64ull * c;
            if (b0 >= s4 && b0 + 64 <= e4) {
                if constexpr (SW) {
                    uint32_t be[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j) be[j] = __builtin_bswap32(w[j]);
                    crc = __builtin_bswap32(crc_block16<C>(__builtin_bswap32(crc), be, swtab));
                } else {
                    crc = crc_block16<C>(crc, w, tab);
                }
            } else {
                const uint64_t lo = s4 > b0 ? (s4 - b0) >> 2 : 0;
                const uint64_t hi = e4 - b0 >= 64 ? 16 : (e4 - b0) >> 2;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t u = SW ? __builtin_bswap32(crc_x_last<C>(__builtin_bswap32(crc ^ w[j]), swtab))
                                          : crc_word<C>(crc, w[j], tab);
                    crc = (uint64_t(j) >= lo && uint64_t(j) < hi) ? u : crc;
                }
            }
        }
    }
    const uint64_t tb = e4 > hb ? e4 : hb;
    for (uint64_t a = tb; a < ea; ++a) crc = crc_byte<C>(crc, s[a - sa], tab);
    return ~crc;
}

}  // namespace nkv
