// sha1_dev.hpp -- per-lane SHA-1 compression for gfx950 (CDNA4).
//
// One lane owns one message (one Merkle leaf or one parent node): SHA-1 is a
// serial chain inside a message, so the parallelism is
// across lanes, 64 messages per wavefront.  Every round is 5 VALU ops on gfx950:
//   rotl5, rotl30      -> v_alignbit_b32
//   Ch / Parity / Maj  -> ONE v_bitop3_b32 (gfx950's 3-input truth-table op;
//                         truth tables 0xCA / 0x96 / 0xE8, src0/1/2 = 0xF0/0xCC/0xAA)
//   5-term sum         -> 2 x v_add3_u32 (round constant in an SGPR)
// and each schedule word is 3 ops (v_bitop3 xor3 + v_xor + v_alignbit), each
// input word 1 v_perm_b32 byte swap: 613 VALU per 64-byte block in total.
// The arithmetic is FIPS 180-4 SHA-1, the function Go's crypto/sha1 computes
// for ds/merkletree/merklenode.go:27-34 and merkletree.go:44-46.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nkv {

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, 32u - n);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t b, uint32_t c, uint32_t d) {
    return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);  // b ? c : d
}
__device__ __forceinline__ uint32_t maj(uint32_t b, uint32_t c, uint32_t d) {
    return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);
}

// Big-endian word made of bytes [s, s+4) of the little-endian byte pair lo,hi
// (lo = bytes 0..3, hi = bytes 4..7), s in 0..3: one v_perm_b32 with a per-lane
// selector from be_sel(s).  Fuses the unaligned funnel shift and the byte swap.
__device__ __forceinline__ uint32_t be_sel(uint32_t s) {
    return ((s + 0u) << 24) | ((s + 1u) << 16) | ((s + 2u) << 8) | (s + 3u);
}
__device__ __forceinline__ uint32_t be_word(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// v_add3_u32 as an opaque (but non-volatile, freely schedulable) instruction,
// so the association below survives instruction selection.
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t add3k(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

__device__ __forceinline__ void sha1_init(uint32_t h[5]) {
    h[0] = 0x67452301u;
    h[1] = 0xEFCDAB89u;
    h[2] = 0x98BADCFEu;
    h[3] = 0x10325476u;
    h[4] = 0xC3D2E1F0u;
}

// One 64-byte block; w[] holds the 16 big-endian message words and is
// clobbered (it becomes the rolling schedule).
__device__ __forceinline__ void sha1_compress(uint32_t h[5], uint32_t w[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) {
            f = ch(b, c, d);
            k = 0x5A827999u;
        } else if (t < 40) {
            f = xor3(b, c, d);
            k = 0x6ED9EBA1u;
        } else if (t < 60) {
            f = maj(b, c, d);
            k = 0x8F1BBCDCu;
        } else {
            f = xor3(b, c, d);
            k = 0xCA62C1D6u;
        }
        // e + W + K does not depend on this round's a/b, so the critical path
        // through a round is two ops (rotl5 or f, then one add3)
        const uint32_t ewk = add3k(e, wt, k);
        const uint32_t tmp = add3(rotl(a, 5), f, ewk);
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
}

// rotl(x, 1) of a wave-uniform x on the scalar unit.  Written as shifts in C,
// the compiler recognises the rotate and selects v_alignbit (vector-only) plus
// a v_readfirstlane back; s_lshl1_add_u32 adds the carried-out bit instead.
__device__ __forceinline__ uint32_t srotl1(uint32_t x) {
    uint32_t r, t;
    asm("s_lshr_b32 %1, %2, 31\n\ts_lshl1_add_u32 %0, %2, %1" : "=s"(r), "=&s"(t) : "s"(x) : "scc");
    return r;
}

// A block whose 16 message words are the same in every lane (wave-uniform:
// the padding block of values of one length that is a multiple of 64): the
// schedule and W + K run on the scalar unit, which idles beside the VALU, so
// the block costs the 400 round ops (e + W + K: one v_add with an SGPR
// operand) instead of 613 VALU.
__device__ __forceinline__ void sha1_compress_uniform(uint32_t h[5], uint32_t w[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = srotl1(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15]);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) {
            f = ch(b, c, d);
            k = 0x5A827999u;
        } else if (t < 40) {
            f = xor3(b, c, d);
            k = 0x6ED9EBA1u;
        } else if (t < 60) {
            f = maj(b, c, d);
            k = 0x8F1BBCDCu;
        } else {
            f = xor3(b, c, d);
            k = 0xCA62C1D6u;
        }
        uint32_t wk, ewk;  // W + K on the scalar unit, + e in one v_add with an SGPR operand
        asm("s_add_u32 %0, %1, %2" : "=s"(wk) : "s"(wt), "s"(k) : "scc");
        asm("v_add_u32 %0, %1, %2" : "=v"(ewk) : "s"(wk), "v"(e));
        const uint32_t tmp = add3(rotl(a, 5), f, ewk);
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
}

// The padding block of a value whose length L (wave-uniform) is a multiple of
// 64: 0x80, zeros, the 64-bit big-endian bit length (FIPS 180-4 5.1.1).
__device__ __forceinline__ void sha1_pad_uniform(uint32_t h[5], uint64_t L) {
    const uint64_t bits = L << 3;
    uint32_t w[16];
    w[0] = 0x80000000u;
#pragma unroll
    for (int j = 1; j < 14; ++j) w[j] = 0u;
    w[14] = uint32_t(bits >> 32);
    w[15] = uint32_t(bits);
    sha1_compress_uniform(h, w);
}

// Parent node of the Merkle tree (ds/merkletree/merkletree.go:44-46):
// SHA-1(left || right) for a pair (40-byte message), SHA-1(left) for a lone
// node whose sibling is the empty pad (20-byte message).  Children are given
// as their SHA-1 state words, which are exactly the big-endian message words.
// A wave with no lone node (all but at most one wave of a level) takes the
// pair form with its padding words as constants, which the compiler folds
// into the schedule; only a wave holding the level's lone node selects the
// message words per lane.
__device__ __forceinline__ void sha1_parent(const uint32_t l[5], const uint32_t r[5], bool lone,
                                            uint32_t out[5]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = l[i];
    sha1_init(out);
    if (!__any(lone)) {
#pragma unroll
        for (int i = 0; i < 5; ++i) w[5 + i] = r[i];
        w[10] = 0x80000000u;
#pragma unroll
        for (int i = 11; i < 15; ++i) w[i] = 0u;
        w[15] = 320u;
        sha1_compress(out, w);
        return;
    }
    if (lone) {
        w[5] = 0x80000000u;
#pragma unroll
        for (int i = 6; i < 15; ++i) w[i] = 0u;
        w[15] = 160u;
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) w[5 + i] = r[i];
        w[10] = 0x80000000u;
#pragma unroll
        for (int i = 11; i < 15; ++i) w[i] = 0u;
        w[15] = 320u;
    }
    sha1_compress(out, w);
}

}  // namespace nkv
