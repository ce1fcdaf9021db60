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
        if (!header_in(r, stream_len)) {
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

// ---------------------------------------------------------------------------
// Range-privatised insert.  A filter's n*k bit updates land on m bits at
// random: device-scope atomicOr on one shared array runs at ~24 G updates/s.
// Instead the bit space is cut into 32768-bit ranges (4 KiB of LDS each) and
// the updates are grouped by range with a counting sort (per-tile counts, one
// column scan, a scatter that recomputes the hashes), then one workgroup per
// range sets its bits with LDS atomics and ORs its 1024 words into the filter
// (it is their only writer).
constexpr uint32_t kBloomRangeShift = 15;
constexpr uint32_t kBloomRangeWords = (1u << kBloomRangeShift) / 32;
constexpr uint32_t kBloomMaxRanges = 4096;  // LDS counters of a tile
constexpr int kBloomTileKeys = 8;           // keys per thread of a tile

// key i: pointer and length (MODE 1: the record's key, header checked)
template <int MODE>
__device__ __forceinline__ bool bloom_key(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                                          uint64_t stream_len, uint64_t i, const uint8_t** key, uint64_t* L) {
    if (MODE == 0) {
        *key = base + off[i];
        *L = len[i];
        return true;
    }
    const uint64_t r = off[i];
    if (!header_in(r, stream_len)) return false;
    const uint64_t l = bl_ld_le64(base + r + 14);
    if (l > stream_len - r - 30) return false;
    *key = base + r + 30;
    *L = l;
    return true;
}

// fn(idx) for the k bit indices of key i
template <int MODE, class F>
__device__ __forceinline__ void bloom_indices(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                                              uint64_t stream_len, uint64_t i, uint32_t m, uint64_t M, uint32_t k,
                                              uint32_t seed0, unsigned int* err, F fn) {
    const uint8_t* key;
    uint64_t L;
    if (!bloom_key<MODE>(base, off, len, stream_len, i, &key, &L)) {
        if (err) atomicOr(err, 1u);
        return;
    }
    for (uint32_t j0 = 0; j0 < k; j0 += kBloomMaxK) {
        const int nk = int(min(k - j0, uint32_t(kBloomMaxK)));
        uint32_t h[kBloomMaxK];
        mm_states(key, L, seed0 + j0, nk, h);
#pragma unroll
        for (int j = 0; j < kBloomMaxK; ++j)
            if (j < nk) fn(fastmod_u32(mm_fmix(h[j] ^ uint32_t(L)), M, m));
    }
}

template <int MODE>
__global__ __launch_bounds__(kBloomBlock) void k_bloom_count(const uint8_t* __restrict__ base,
                                                             const uint64_t* __restrict__ off,
                                                             const uint64_t* __restrict__ len, uint64_t stream_len,
                                                             uint64_t n, uint32_t m, uint64_t M, uint32_t k,
                                                             uint32_t seed0, uint32_t nranges, uint32_t tiles,
                                                             uint32_t* __restrict__ hist, unsigned int* err) {
    __shared__ uint32_t cnt[kBloomMaxRanges];
    for (uint32_t r = threadIdx.x; r < nranges; r += kBloomBlock) cnt[r] = 0u;
    __syncthreads();
    const uint64_t t0 = uint64_t(blockIdx.x) * kBloomBlock * kBloomTileKeys;
    for (int q = 0; q < kBloomTileKeys; ++q) {
        const uint64_t i = t0 + uint64_t(q) * kBloomBlock + threadIdx.x;
        if (i < n)
            bloom_indices<MODE>(base, off, len, stream_len, i, m, M, k, seed0, err,
                                [&](uint32_t idx) { atomicAdd(&cnt[idx >> kBloomRangeShift], 1u); });
    }
    __syncthreads();
    // range-major, so one exclusive scan gives every (range, tile) slot's first
    // update position and range r's updates are [hist[r * tiles], hist[(r + 1) * tiles])
    for (uint32_t r = threadIdx.x; r < nranges; r += kBloomBlock) hist[uint64_t(r) * tiles + blockIdx.x] = cnt[r];
}

template <int MODE>
__global__ __launch_bounds__(kBloomBlock) void k_bloom_scatter(const uint8_t* __restrict__ base,
                                                               const uint64_t* __restrict__ off,
                                                               const uint64_t* __restrict__ len,
                                                               uint64_t stream_len, uint64_t n, uint32_t m, uint64_t M,
                                                               uint32_t k, uint32_t seed0, uint32_t nranges,
                                                               uint32_t tiles, const uint32_t* __restrict__ hist,
                                                               uint32_t* __restrict__ upd) {
    __shared__ uint32_t cur[kBloomMaxRanges];
    for (uint32_t r = threadIdx.x; r < nranges; r += kBloomBlock) cur[r] = hist[uint64_t(r) * tiles + blockIdx.x];
    __syncthreads();
    const uint64_t t0 = uint64_t(blockIdx.x) * kBloomBlock * kBloomTileKeys;
    for (int q = 0; q < kBloomTileKeys; ++q) {
        const uint64_t i = t0 + uint64_t(q) * kBloomBlock + threadIdx.x;
        if (i < n)
            bloom_indices<MODE>(base, off, len, stream_len, i, m, M, k, seed0, nullptr,
                                [&](uint32_t idx) { upd[atomicAdd(&cur[idx >> kBloomRangeShift], 1u)] = idx; });
    }
}

__global__ __launch_bounds__(kBloomBlock) void k_bloom_apply(const uint32_t* __restrict__ upd,
                                                             const uint32_t* __restrict__ hist, uint32_t tiles,
                                                             uint32_t words, uint32_t* __restrict__ bits) {
    __shared__ uint32_t w[kBloomRangeWords];
    const uint32_t r = blockIdx.x;
    for (uint32_t t = threadIdx.x; t < kBloomRangeWords; t += kBloomBlock) w[t] = 0u;
    __syncthreads();
    // hist holds one word past the last range: the total
    const uint32_t lo = hist[uint64_t(r) * tiles], hi = hist[uint64_t(r + 1) * tiles];
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kBloomBlock) {
        const uint32_t idx = upd[i];
        atomicOr(&w[(idx >> 5) & (kBloomRangeWords - 1)], 1u << (idx & 31u));
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < kBloomRangeWords; t += kBloomBlock) {
        const uint64_t g = uint64_t(r) * kBloomRangeWords + t;
        if (g < words && w[t]) bits[g] |= w[t];  // range r's words have no other writer
    }
}

uint64_t bloom_ranges_scratch_words(uint64_t n, uint32_t m, uint32_t k) {
    const uint64_t nranges = (uint64_t(m) + (1u << kBloomRangeShift) - 1) >> kBloomRangeShift;
    const uint64_t tiles = (n + uint64_t(kBloomBlock) * kBloomTileKeys - 1) / (uint64_t(kBloomBlock) * kBloomTileKeys);
    if (nranges > kBloomMaxRanges || n * k > 0xFFFFFFFFull) return 0;  // the atomic kernel serves these
    const uint64_t h = tiles * nranges + 1;
    return h + scan_sums_words(h) + n * k;
}

hipError_t launch_bloom_ranges(int mode, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                               uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0,
                               uint32_t* bits, unsigned int* err, uint32_t* scratch, hipStream_t s) {
    if (n == 0 || k == 0) return hipSuccess;
    const uint32_t nranges = (m + (1u << kBloomRangeShift) - 1) >> kBloomRangeShift;
    const uint64_t tiles = (n + uint64_t(kBloomBlock) * kBloomTileKeys - 1) / (uint64_t(kBloomBlock) * kBloomTileKeys);
    const uint64_t hn = tiles * nranges + 1;
    uint32_t* hist = scratch;
    uint32_t* sums = hist + hn;
    uint32_t* upd = sums + scan_sums_words(hn);
    const uint64_t M = fastmod_magic(m);
    const uint32_t words = (m + 31) / 32;
    const uint32_t T = uint32_t(tiles);
    hipError_t e = hipMemsetAsync(hist + hn - 1, 0, 4, s);  // the appended zero: the scan leaves the total there
    if (e != hipSuccess) return e;
    if (mode == 0)
        hipLaunchKernelGGL(k_bloom_count<0>, dim3(T), dim3(kBloomBlock), 0, s, base, off, len, stream_len, n, m, M, k,
                           seed0, nranges, T, hist, err);
    else
        hipLaunchKernelGGL(k_bloom_count<1>, dim3(T), dim3(kBloomBlock), 0, s, base, off, len, stream_len, n, m, M, k,
                           seed0, nranges, T, hist, err);
    if ((e = scan_exclusive_u32(hist, hn, sums, s)) != hipSuccess) return e;
    if (mode == 0)
        hipLaunchKernelGGL(k_bloom_scatter<0>, dim3(T), dim3(kBloomBlock), 0, s, base, off, len, stream_len, n, m, M,
                           k, seed0, nranges, T, hist, upd);
    else
        hipLaunchKernelGGL(k_bloom_scatter<1>, dim3(T), dim3(kBloomBlock), 0, s, base, off, len, stream_len, n, m, M,
                           k, seed0, nranges, T, hist, upd);
    hipLaunchKernelGGL(k_bloom_apply, dim3(nranges), dim3(kBloomBlock), 0, s, upd, hist, T, words, bits);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Staged insert (NKV_OPT_BLOOM_PATH 2): each key is loaded and hashed once.  A
// tile of kBloomBlock x kpt keys hashes into LDS (a thread-major list of its
// updates, counted per range), counting-sorts them by range inside LDS, and
// writes the sorted list contiguously to its own stage area, with per-range
// counts and starts (range-major over tiles).  One workgroup per range then
// reads its segment of every tile and sets its bits in LDS.  The range path
// above hashes every key twice (count, scatter) and scatters 4-byte updates
// one by one across the whole update array.
constexpr uint32_t kStageLdsWords = 16384 - 64;  // 64 KiB of dynamic LDS, less the scan's words
constexpr int kApplyBlock = 1024;

__device__ __forceinline__ uint32_t bloom_block_exclusive(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = uint32_t(__shfl_up(int(x), o));
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBloomBlock / 64; ++w) {
        if (w < wave) before += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

template <int MODE>
__global__ __launch_bounds__(kBloomBlock) void k_bloom_stage(const uint8_t* __restrict__ base,
                                                             const uint64_t* __restrict__ off,
                                                             const uint64_t* __restrict__ len, uint64_t stream_len,
                                                             uint64_t n, uint32_t m, uint64_t M, uint32_t k,
                                                             uint32_t seed0, uint32_t nranges, uint32_t tiles,
                                                             uint32_t kpt, uint32_t* __restrict__ stage,
                                                             uint32_t* __restrict__ tcount,
                                                             uint32_t* __restrict__ tstart, unsigned int* err) {
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t wsum[kBloomBlock / 64];
    const uint32_t per = kpt * k;  // update slots per thread
    uint32_t* A = lds;                            // thread-major, per slots each
    uint32_t* B = A + per * kBloomBlock;          // sorted by range
    uint32_t* cnt = B + per * kBloomBlock;        // nranges counts, then cursors
    for (uint32_t r = threadIdx.x; r < nranges; r += kBloomBlock) cnt[r] = 0u;
    __syncthreads();
    uint32_t* mine = A + threadIdx.x * per;
    uint32_t na = 0;
    const uint64_t t0 = uint64_t(blockIdx.x) * kBloomBlock * kpt;
    for (uint32_t q = 0; q < kpt; ++q) {
        const uint64_t i = t0 + uint64_t(q) * kBloomBlock + threadIdx.x;
        if (i < n)
            bloom_indices<MODE>(base, off, len, stream_len, i, m, M, k, seed0, err, [&](uint32_t idx) {
                mine[na++] = idx;
                atomicAdd(&cnt[idx >> kBloomRangeShift], 1u);
            });
    }
    __syncthreads();
    // exclusive scan of the counts: thread t owns a contiguous run of ranges
    const uint32_t run = (nranges + kBloomBlock - 1) / kBloomBlock;
    const uint32_t r0 = threadIdx.x * run, r1 = min(r0 + run, nranges);
    uint32_t mysum = 0;
    for (uint32_t r = r0; r < r1; ++r) mysum += cnt[r];
    uint32_t total;
    uint32_t at = bloom_block_exclusive(mysum, wsum, &total);
    for (uint32_t r = r0; r < r1; ++r) {
        const uint32_t c = cnt[r];
        tcount[uint64_t(r) * tiles + blockIdx.x] = c;
        tstart[uint64_t(r) * tiles + blockIdx.x] = at;
        cnt[r] = at;  // becomes the range's cursor
        at += c;
    }
    __syncthreads();
    for (uint32_t j = 0; j < na; ++j) {
        const uint32_t idx = mine[j];
        B[atomicAdd(&cnt[idx >> kBloomRangeShift], 1u)] = idx;
    }
    __syncthreads();
    uint32_t* dst = stage + uint64_t(blockIdx.x) * per * kBloomBlock;
    for (uint32_t j = threadIdx.x; j < total; j += kBloomBlock) dst[j] = B[j];
}

// one workgroup per range: a thread per tile reads that tile's segment
// (unrolled, so several loads are in flight) into the LDS bitmap
__global__ __launch_bounds__(kApplyBlock) void k_bloom_apply_staged(const uint32_t* __restrict__ stage,
                                                                    uint32_t tile_slots,
                                                                    const uint32_t* __restrict__ tcount,
                                                                    const uint32_t* __restrict__ tstart,
                                                                    uint32_t tiles, uint32_t words,
                                                                    uint32_t* __restrict__ bits) {
    __shared__ uint32_t w[kBloomRangeWords];
    const uint32_t r = blockIdx.x;
    for (uint32_t t = threadIdx.x; t < kBloomRangeWords; t += kApplyBlock) w[t] = 0u;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < tiles; t += kApplyBlock) {
        const uint32_t c = tcount[uint64_t(r) * tiles + t];
        const uint32_t* seg = stage + uint64_t(t) * tile_slots + tstart[uint64_t(r) * tiles + t];
        uint32_t j = 0;
        for (; j + 4 <= c; j += 4) {
            const uint32_t a = seg[j], b = seg[j + 1], d = seg[j + 2], e = seg[j + 3];
            atomicOr(&w[(a >> 5) & (kBloomRangeWords - 1)], 1u << (a & 31u));
            atomicOr(&w[(b >> 5) & (kBloomRangeWords - 1)], 1u << (b & 31u));
            atomicOr(&w[(d >> 5) & (kBloomRangeWords - 1)], 1u << (d & 31u));
            atomicOr(&w[(e >> 5) & (kBloomRangeWords - 1)], 1u << (e & 31u));
        }
        for (; j < c; ++j) {
            const uint32_t a = seg[j];
            atomicOr(&w[(a >> 5) & (kBloomRangeWords - 1)], 1u << (a & 31u));
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < kBloomRangeWords; t += kApplyBlock) {
        const uint64_t g = uint64_t(r) * kBloomRangeWords + t;
        if (g < words && w[t]) bits[g] |= w[t];  // range r's words have no other writer
    }
}

// keys per thread of a staged tile: two update lists (per slots each) and the
// range counters fit the 64 KiB of dynamic LDS; 0 = not applicable
static uint32_t bloom_stage_kpt(uint32_t k, uint32_t nranges) {
    if (k == 0 || nranges >= kStageLdsWords) return 0u;
    const uint32_t kpt = (kStageLdsWords - nranges) / 2 / (uint32_t(kBloomBlock) * k);
    return kpt < 32u ? kpt : 32u;
}

uint64_t bloom_staged_scratch_words(uint64_t n, uint32_t m, uint32_t k) {
    const uint64_t nranges = (uint64_t(m) + (1u << kBloomRangeShift) - 1) >> kBloomRangeShift;
    if (nranges > kBloomMaxRanges) return 0;
    const uint32_t kpt = bloom_stage_kpt(k, uint32_t(nranges));
    if (kpt == 0) return 0;  // the range or atomic path serves these
    const uint64_t tiles = (n + uint64_t(kBloomBlock) * kpt - 1) / (uint64_t(kBloomBlock) * kpt);
    return tiles * kpt * k * kBloomBlock + 2 * tiles * nranges;
}

hipError_t launch_bloom_staged(int mode, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                               uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0,
                               uint32_t* bits, unsigned int* err, uint32_t* scratch, hipStream_t s) {
    if (n == 0 || k == 0) return hipSuccess;
    const uint32_t nranges = (m + (1u << kBloomRangeShift) - 1) >> kBloomRangeShift;
    const uint32_t kpt = bloom_stage_kpt(k, nranges);
    const uint64_t tiles = (n + uint64_t(kBloomBlock) * kpt - 1) / (uint64_t(kBloomBlock) * kpt);
    const uint32_t slots = kpt * k * kBloomBlock;
    uint32_t* stage = scratch;
    uint32_t* tcount = stage + tiles * slots;
    uint32_t* tstart = tcount + tiles * nranges;
    const uint64_t M = fastmod_magic(m);
    const uint32_t words = (m + 31) / 32;
    const uint32_t T = uint32_t(tiles);
    const size_t lds = (size_t(2) * slots + nranges) * sizeof(uint32_t);
    if (mode == 0)
        hipLaunchKernelGGL(k_bloom_stage<0>, dim3(T), dim3(kBloomBlock), lds, s, base, off, len, stream_len, n, m, M,
                           k, seed0, nranges, T, kpt, stage, tcount, tstart, err);
    else
        hipLaunchKernelGGL(k_bloom_stage<1>, dim3(T), dim3(kBloomBlock), lds, s, base, off, len, stream_len, n, m, M,
                           k, seed0, nranges, T, kpt, stage, tcount, tstart, err);
    hipLaunchKernelGGL(k_bloom_apply_staged, dim3(nranges), dim3(kApplyBlock), 0, s, stage, slots, tcount, tstart, T,
                       words, bits);
    return hipGetLastError();
}

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
