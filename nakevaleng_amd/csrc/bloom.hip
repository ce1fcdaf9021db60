// bloom.hip -- the SSTable filter build on gfx950.
//
// Reference: core/sstable/sstable.go:49-56 (makeFilter: bloomfilter.New(n, 0.01),
// Insert(key) per record key), ds/bloomfilter/bloomfilter.go:28-39 (k hash
// functions seeded t, t+1, ..), :76-91 (Insert: bit murmur3(seed_j, key) % M,
// Contents[idx / 8] |= 1 << (idx % 8)), :93-111 (Query).  The hash is
// spaolacci/murmur3 v1.1.0 Sum32 = MurmurHash3_x86_32.
//
// One lane per key.  The key's 4-byte little-endian blocks come from aligned
// dword loads funnelled by the key's byte offset (v_alignbyte), so any
// alignment works and no load touches a dword without a key byte.  The block
// mix (k *= c1, rotl 15, *= c2) does not depend on the seed, so it is done once
// per block and shared by all k hash states, which are kept in registers (up
// to kBloomMaxK per pass over the key).  idx = h % M by Lemire's fastmod (one
// 64-bit multiply + one 64x32 high multiply, exact for every 32-bit h).
// Contents is addressed as little-endian 32-bit words: byte idx/8 bit idx%8 is
// word idx/32 bit idx%32, set with one atomicOr.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "internal.hpp"

namespace nkv {

constexpr int kBloomBlock = 256;
constexpr int kBloomMaxK = 16;

__device__ __forceinline__ uint32_t mm_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ __forceinline__ uint32_t mm_fmix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

__device__ __forceinline__ uint32_t mm_block(uint32_t k) {
    k *= 0xcc9e2d51u;
    k = mm_rotl(k, 15);
    return k * 0x1b873593u;
}

// Lemire fastmod: a % d with M = 2^64 / d rounded up (M = 0 for d = 1).
__device__ __forceinline__ uint32_t fastmod_u32(uint32_t a, uint64_t M, uint32_t d) {
    const uint64_t low = M * a;
    return uint32_t(__umul64hi(low, uint64_t(d)));
}

__device__ __forceinline__ uint64_t bl_ld_le64(const uint8_t* p) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v |= uint64_t(p[i]) << (8 * i);
    return v;
}

// h[j] = MurmurHash3_x86_32(key, seed0 + j0 + j) before the final length xor
// and fmix, for j < nk (<= kBloomMaxK).
__device__ __forceinline__ void mm_states(const uint8_t* key, uint64_t len, uint32_t seed, int nk,
                                          uint32_t h[kBloomMaxK]) {
#pragma unroll
    for (int j = 0; j < kBloomMaxK; ++j) h[j] = seed + uint32_t(j);
    const uint32_t s = uint32_t(reinterpret_cast<uintptr_t>(key)) & 3u;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(key - s);  // stays a global pointer
    const uint64_t nb = len >> 2;
    const uint32_t nxt = s != 0u;  // the dword after q[i] holds key bytes only when s > 0
    for (uint64_t i = 0; i < nb; ++i) {
        const uint32_t k = mm_block(__builtin_amdgcn_alignbyte(q[i + nxt], q[i], s));
#pragma unroll
        for (int j = 0; j < kBloomMaxK; ++j)
            if (j < nk) h[j] = mm_rotl(h[j] ^ k, 13) * 5u + 0xe6546b64u;
    }
    const uint32_t r = uint32_t(len & 3u);
    if (r) {
        // bytes 4nb .. 4nb+r-1: in q[nb] and, if s + r > 4, q[nb + 1]
        const uint32_t w0 = q[nb];
        const uint32_t w1 = s + r > 4u ? q[nb + 1] : w0;
        const uint32_t t = __builtin_amdgcn_alignbyte(w1, w0, s) & (0xFFFFFFFFu >> (8 * (4 - r)));
        const uint32_t k = mm_block(t);
#pragma unroll
        for (int j = 0; j < kBloomMaxK; ++j)
            if (j < nk) h[j] ^= k;
    }
}

// MODE 0: key i at base + off[i], len[i].  MODE 1: key of the record at
// base + off[i] (at +30, KeySize at +14), checked against stream_len (err).
// QUERY: out[i] = every bit set; else set the bits.
template <int MODE, bool QUERY>
__global__ __launch_bounds__(kBloomBlock) void k_bloom(const uint8_t* __restrict__ base,
                                                       const uint64_t* __restrict__ off,
                                                       const uint64_t* __restrict__ len, uint64_t stream_len,
                                                       uint64_t n, uint32_t m, uint64_t M, uint32_t k,
                                                       uint32_t seed0, uint32_t* __restrict__ bits,
                                                       uint8_t* __restrict__ out, unsigned int* __restrict__ err) {
    const uint64_t i = uint64_t(blockIdx.x) * kBloomBlock + threadIdx.x;
    if (i >= n) return;
    const uint8_t* key;
    uint64_t L;
    if (MODE == 0) {
        key = base + off[i];
        L = len[i];
    } else {
        const uint64_t r = off[i];
        if (r + 30 > stream_len) {
            atomicOr(err, 1u);
            return;
        }
        L = bl_ld_le64(base + r + 14);
        if (L > stream_len - r - 30) {
            atomicOr(err, 1u);
            return;
        }
        key = base + r + 30;
    }
    bool hit = true;
    for (uint32_t j0 = 0; j0 < k; j0 += kBloomMaxK) {
        const int nk = int(min(k - j0, uint32_t(kBloomMaxK)));
        uint32_t h[kBloomMaxK];
        mm_states(key, L, seed0 + j0, nk, h);
#pragma unroll
        for (int j = 0; j < kBloomMaxK; ++j) {
            if (j < nk) {
                const uint32_t idx = fastmod_u32(mm_fmix(h[j] ^ uint32_t(L)), M, m);
                if (QUERY) hit = hit && ((bits[idx >> 5] >> (idx & 31u)) & 1u);
                else atomicOr(bits + (idx >> 5), 1u << (idx & 31u));
            }
        }
    }
    if (QUERY) out[i] = hit ? 1 : 0;
}

static uint64_t fastmod_magic(uint32_t d) { return ~uint64_t(0) / d + 1; }

hipError_t launch_bloom(int mode, bool query, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                        uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0, uint32_t* bits,
                        uint8_t* out, unsigned int* err, hipStream_t s) {
    if (n == 0 || k == 0) return hipSuccess;
    const dim3 grid(uint32_t((n + kBloomBlock - 1) / kBloomBlock)), block(kBloomBlock);
    const uint64_t M = fastmod_magic(m);
#define NKV_BLOOM_LAUNCH(MD, Q) \
    hipLaunchKernelGGL((k_bloom<MD, Q>), grid, block, 0, s, base, off, len, stream_len, n, m, M, k, seed0, bits, out, err)
    if (mode == 0) {
        if (query) NKV_BLOOM_LAUNCH(0, true);
        else NKV_BLOOM_LAUNCH(0, false);
    } else {
        if (query) NKV_BLOOM_LAUNCH(1, true);
        else NKV_BLOOM_LAUNCH(1, false);
    }
#undef NKV_BLOOM_LAUNCH
    return hipGetLastError();
}

}  // namespace nkv
