// kernels.hip -- gfx950 kernels of the Merkle step of SSTable build.
//
//   K1  k_leaf        NewLeaf over many values (merklenode.go:27-34), one lane
//                     per leaf, 64 leaves per wavefront (level 0 only).
//   K1q k_leaf_queue  the same for ragged, length-sorted batches (work queue).
//   K1v k_leaf_verify the compaction read: record checksum check + NewLeaf.
//   K2w k_reduce2     build() levels (merkletree.go:31-64) two at a time at
//                     full lane use, while a level holds >= 64 Ki nodes.
//   K2  k_reduce      the rest: a 256-node slab of one level reduced up to 8
//                     levels in LDS per launch.
//   K3  k_bfs_image   Serialize() byte image (merkletree.go:67-92,
//                     merklenode.go:37-63) at closed-form offsets.
//   K0  k_locate      value offset/length of each serialized core/record
//                     (record.go:191-199): value = rec + 30 + KeySize.
//   Ks  k_small_tree  a whole small tree (n <= 1024) and its image in one launch.
//       k_fill        splitmix64 synthetic bytes (bench/test input only).
//
// Node storage ("nodes" buffer): every level, bottom-up, level-major; level L
// holds ceil(n / 2^L) 20-byte digests in Go byte order (big-endian words);
// level 0 is the leaves, the last digest is the root.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "crc_dev.hpp"
#include "internal.hpp"
#include "nkv_merkle.h"
#include "sha1_dev.hpp"

namespace nkv {

// experiment builds only (tools/build_exp.sh -D...), never the product library
#ifndef NKV_EXP_REC
#define NKV_EXP_REC 0
#endif
#ifndef NKV_EXP_NOTAIL
#define NKV_EXP_NOTAIL 0
#endif
#ifndef NKV_EXP_PARTIAL_REDUCE
#define NKV_EXP_PARTIAL_REDUCE 0  // 1: subtree_reduce with only the live lanes active (the round-5 form)
#endif
#ifndef NKV_EXP_FIXEDHDR
#define NKV_EXP_FIXEDHDR 0
#endif

#ifdef NKV_DIAG
// Diagnostic build only (tools/diag_timeline.py): per-wave s_memtime /
// s_memrealtime stamps, never part of an output.
__device__ unsigned long long* g_diag = nullptr;
#define NKV_STAMP(slot)                                                                 \
    do {                                                                                \
        if (g_diag && (threadIdx.x & 63) == 0) {                                        \
            const size_t w_ = size_t(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);   \
            g_diag[w_ * 8 + 2 * (slot)] = __builtin_amdgcn_s_memrealtime();             \
            g_diag[w_ * 8 + 2 * (slot) + 1] = __builtin_amdgcn_s_memtime();             \
        }                                                                               \
    } while (0)
#else
#define NKV_STAMP(slot) \
    do {                \
    } while (0)
#endif

// Clock probe (NKV_TIMING_CLOCK; bench.py's sclk_mhz).  Each wave of a leaf
// kernel adds its lifetime in shader-clock cycles (s_memtime) and in 100 MHz
// reference ticks (s_memrealtime) to slot[0] / slot[1] and counts itself in
// slot[2] (slot = g_clk + 32 (workgroup % 8)); the host divides the sums: the
// shader clock the kernel's waves ran at, weighted by their lifetimes.  Off
// (g_clk null) it costs one uniform load.
__device__ unsigned long long* g_clk = nullptr;
struct ClockProbe {
    unsigned long long* p;
    uint64_t c0 = 0, r0 = 0;
    __device__ __forceinline__ ClockProbe() : p(g_clk) {
        if (p) {
            c0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
        }
    }
    __device__ __forceinline__ void end() const {
        if (p) {
            const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            if ((threadIdx.x & 63) == 0) {  // 8 slots on their own 256-B lines: little contention
                unsigned long long* q = p + 32 * (blockIdx.x & 7);
                atomicAdd(q, (unsigned long long)(c1 - c0));
                atomicAdd(q + 1, (unsigned long long)(r1 - r0));
                atomicAdd(q + 2, 1ull);
            }
        }
    }
};

hipError_t set_clock_probe(unsigned long long* p, hipStream_t s) {
    (void)s;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_clk), &p, sizeof(p));
}

// KeySize and ValueSize (header bytes 14..29, record.go:191-199) of the
// record at p, from two or three aligned 8-byte loads and a funnel shift
// instead of sixteen byte loads (one line request per lane per load rather
// than one per byte).  The third load is issued only when the fields are
// not 8-byte aligned; it then holds byte 29, so every load stays inside an
// aligned word that holds a header byte (no page can be crossed).
__device__ __forceinline__ void ld_header_sizes(const uint8_t* p, uint64_t& ks, uint64_t& vs) {
#if NKV_EXP_FIXEDHDR
    // traffic experiment only (wrong for any other shape): the bench's 16-B
    // keys and 4,050-B values without reading the header line
    (void)p;
    ks = 16;
    vs = 4050;
    return;
#endif
    // pointer arithmetic on p (not an integer-to-pointer cast) keeps the global
    // address space: global_load, not flat_load
    const uint8_t* f = p + 14;
    const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(f) & 7u);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(f - mis);
    const uint32_t sh = mis * 8u;
    const uint64_t q0 = q[0], q1 = q[1];
    const uint64_t q2 = sh ? q[2] : 0ull;
    ks = sh ? (q0 >> sh) | (q1 << (64u - sh)) : q0;
    vs = sh ? (q1 >> sh) | (q2 << (64u - sh)) : q1;
}

// ---------------------------------------------------------------------------
// Block fold: leaves the workgroup's min / max / or / sum in thread 0.  Grid
// results go through per-workgroup partials and a fold launch (k_locate_fold)
// or, in the records entries, the pass flags below.
__device__ __forceinline__ void block_fold(uint32_t& lo, uint32_t& hi, uint32_t& flag, unsigned long long& sum) {
    __shared__ uint32_t s_lo[kBlock / 64], s_hi[kBlock / 64], s_fl[kBlock / 64];
    __shared__ unsigned long long s_sum[kBlock / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, uint32_t(__shfl_xor(int(lo), o)));
        hi = max(hi, uint32_t(__shfl_xor(int(hi), o)));
        flag |= uint32_t(__shfl_xor(int(flag), o));
        sum += __shfl_xor(sum, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_lo[w] = lo;
        s_hi[w] = hi;
        s_fl[w] = flag;
        s_sum[w] = sum;
    }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 1; k < kBlock / 64; ++k) {
            lo = min(lo, s_lo[k]);
            hi = max(hi, s_hi[k]);
            flag |= s_fl[k];
            sum += s_sum[k];
        }
}

// Pass flags (internal.hpp kPassFlagWords): block 0 resets the set the next
// call uses; a workgroup raises this call's deferred / bad-header words with
// one atomic each, skipped once another workgroup has raised them.
__device__ __forceinline__ void pass_flags_reset(uint32_t* f) {
    if (blockIdx.x == 0 && threadIdx.x < kPassFlagWords) f[threadIdx.x] = (threadIdx.x & ~1u) == 6u ? ~0u : 0u;
}
__device__ __forceinline__ void pass_flag_raise(uint32_t* f, uint32_t v) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != v) atomicOr(f, v);
}

// SHA-1 compressions of a len-byte message (FIPS 180-4 padding: + 0x80 + 8 B)
__device__ __forceinline__ uint64_t compressions(uint64_t len) { return (len + 8) / 64 + 1; }

// Value offset of a record k_leaf_records already hashed (the length-sorted
// pass that follows it skips the value).
constexpr uint64_t kDone = ~uint64_t(0);

// CRC tables for k_leaf_verify (crc.hip keeps its own copy: no relocatable
// device code, so each translation unit defines its constants)
__constant__ CrcTables c_crc_leaf = make_crc_tables();

constexpr uint32_t kLenBuckets = 640;  // counting-sort buckets (len_bucket_desc)
constexpr int kSortItems = 16;         // values per thread of a sort tile
constexpr uint64_t kSortTile = uint64_t(kBlock) * kSortItems;

// ---------------------------------------------------------------------------
// tree shape helpers (device side; host side mirrors them in capi.cpp)

__device__ __forceinline__ uint64_t lvl_count(uint64_t n, int L) {
    return L == 0 ? n : ((n - 1) >> L) + 1;  // ceil(n / 2^L), n >= 1
}

__device__ __forceinline__ uint64_t lvl_start(uint64_t n, int L) {
    uint64_t s = 0;
    for (int j = 0; j < L; ++j) s += lvl_count(n, j);
    return s;
}

__device__ __forceinline__ void store_digest(uint8_t* nodes, uint64_t idx, const uint32_t h[5]) {
    uint32_t* p = reinterpret_cast<uint32_t*>(nodes + 20ull * idx);
#pragma unroll
    for (int k = 0; k < 5; ++k) p[k] = bswap32(h[k]);
}

__device__ __forceinline__ void load_digest(const uint8_t* nodes, uint64_t idx, uint32_t h[5]) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(nodes + 20ull * idx);
#pragma unroll
    for (int k = 0; k < 5; ++k) h[k] = bswap32(p[k]);
}

// ---------------------------------------------------------------------------
// Subtree reduce inside one 256-thread workgroup.
//
// lds[k][t] holds word k of the node at index lo + t of level j0 (t < 256).
// Levels j0+1 .. jmax are computed; each level's nodes are written to the
// global nodes buffer.  Node i of level j is SHA-1(c[2i] || c[2i+1]) when
// 2i+1 < n_{j-1}, else SHA-1(c[2i]) (the empty pad, merkletree.go:32-34).
template <int B>
__device__ __forceinline__ void subtree_reduce(uint32_t (*lds)[B], uint64_t n, int j0, int jmax, uint64_t lo,
                               uint8_t* nodes) {
    const int tid = threadIdx.x;
    uint64_t nprev = lvl_count(n, j0);
    uint64_t start_cur = lvl_start(n, j0) + nprev;
    uint64_t lo_prev = lo;
    int span = B;
    for (int j = j0 + 1; j <= jmax; ++j) {
        const uint64_t ncur = ((nprev - 1) >> 1) + 1;
        const uint64_t lo_cur = lo_prev >> 1;
        span >>= 1;
        // lanes [0, live) build this level's parents; every lane of a wave that
        // has one takes part (a lane past live rebuilds the last parent and
        // drops it): a wave with few active lanes computes up to 35 % slower on
        // some CUs, and the narrow top levels are a lone-wave chain
        // (sha1_value_all_lanes, tools/svc_shape.hip)
        const int live = ncur > lo_cur ? int(min<uint64_t>(uint64_t(span), ncur - lo_cur)) : 0;
        const bool act = tid < live;
        uint32_t out[5];
        __syncthreads();
        if (NKV_EXP_PARTIAL_REDUCE ? act : (tid & ~63) < live) {
            const int t = min(tid, live - 1);
            uint32_t l[5], r[5];
            const bool lone = (2 * (lo_cur + uint64_t(t)) + 1) >= nprev;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                l[k] = lds[k][2 * t];
                r[k] = lone ? 0u : lds[k][2 * t + 1];
            }
            sha1_parent(l, r, lone, out);
        }
        __syncthreads();
        if (act) {
#pragma unroll
            for (int k = 0; k < 5; ++k) lds[k][tid] = out[k];
            store_digest(nodes, start_cur + lo_cur + tid, out);
        }
        nprev = ncur;
        start_cur += ncur;
        lo_prev = lo_cur;
    }
}

// ---------------------------------------------------------------------------
// K1: leaf SHA-1.
//
// Each lane hashes the value p[0 .. len).  Full 64-byte blocks are streamed
// with a one-block register prefetch; the 1-2 padding blocks are built from
// the remaining 0..63 bytes (FIPS 180-4 5.1.1).  A 16-byte aligned wave takes
// 4 x global_load_dwordx4 per block; otherwise each lane reads the five
// aligned 16-byte chunks that cover its 64 bytes and funnels them with
// v_perm_b32 (never touching an aligned chunk that holds no value byte, so it
// cannot step onto an unmapped page).

__device__ __forceinline__ void be16_from_raw(const uint4 c[4], uint32_t w[16]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        w[4 * q + 0] = bswap32(c[q].x);
        w[4 * q + 1] = bswap32(c[q].y);
        w[4 * q + 2] = bswap32(c[q].z);
        w[4 * q + 3] = bswap32(c[q].w);
    }
}

// d[0..19]: 20 little-endian dwords of the aligned 80-byte window; s = byte
// shift 0..15 of the stream start inside it.  Produces 16 big-endian words.
__device__ __forceinline__ void be16_funnel(const uint32_t d[20], uint32_t s, uint32_t w[16]) {
    // Dword select by k = s >> 2 in two v_perm_b32 steps (a plain ?: on the
    // array would be folded into a dynamically indexed private array).
    const uint32_t k = s >> 2;
    const uint32_t sel = be_sel(s & 3u);
    const uint32_t sel1 = (k & 1u) ? 0x07060504u : 0x03020100u;
    const uint32_t sel2 = (k & 2u) ? 0x07060504u : 0x03020100u;
    uint32_t m1[19];
#pragma unroll
    for (int j = 0; j < 19; ++j) m1[j] = __builtin_amdgcn_perm(d[j + 1], d[j], sel1);
    uint32_t m2[17];
#pragma unroll
    for (int j = 0; j < 17; ++j) m2[j] = __builtin_amdgcn_perm(m1[j + 2], m1[j], sel2);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = be_word(m2[j + 1], m2[j], sel);
}

__device__ __forceinline__ void load_window(const uint8_t* p, uint32_t avail, uint32_t d[20]) {
    // p: stream start; avail: value bytes available from p (>= 1 unless empty).
    // p - s (not an integer-to-pointer cast) keeps the global address space,
    // so these stay global_load_dwordx4 rather than flat loads
    const uint32_t s = uint32_t(reinterpret_cast<uintptr_t>(p) & 15);
    const uint4* q = reinterpret_cast<const uint4*>(p - s);
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (avail > 0 && uint32_t(16 * c) < s + avail) v = q[c];
        d[4 * c + 0] = v.x;
        d[4 * c + 1] = v.y;
        d[4 * c + 2] = v.z;
        d[4 * c + 3] = v.w;
    }
}

// ALIGNED: the caller guarantees p is 16-byte aligned (host-checked base and
// stride, or host-packed values); otherwise a wave-uniform test picks the path.
struct NoRaw;
template <bool ALIGNED, class Hook = NoRaw>
__device__ __forceinline__ void sha1_tail(const uint8_t* p, uint64_t len, uint32_t h[5], Hook hook = Hook{});

// The 1-2 padding blocks: rem = len % 64 value bytes, 0x80, zeros, 64-bit
// big-endian bit length (FIPS 180-4 5.1.1).  h holds the state after the full
// blocks.
// hook.tail(w, rem): the tail block's big-endian words before the padding is
// applied (rem = len % 64 value bytes), for k_leaf_verify's checksum.
template <bool ALIGNED, class Hook>
__device__ __forceinline__ void sha1_tail(const uint8_t* p, uint64_t len, uint32_t h[5], Hook hook) {
    uint32_t w[16];
    const uint64_t nfull = len >> 6;
    const uint32_t rem = uint32_t(len & 63);
    const uint64_t bits = len << 3;
    // A wave-level step issues every instruction whatever the exec mask, so the
    // branches below are taken on wave votes: a wave whose values are all
    // whole blocks (every 4 KiB SSTable value) pays neither the byte loads and
    // masking nor a second compression that no lane needs.
    if (__all(rem == 0u)) {
        w[0] = 0x80000000u;
#pragma unroll
        for (int j = 1; j < 14; ++j) w[j] = 0u;
        w[14] = uint32_t(bits >> 32);
        w[15] = uint32_t(bits);
        sha1_compress(h, w);
        return;
    }
    const uint8_t* pt = p + 64 * nfull;
    if (ALIGNED) {
        const uint4* q = reinterpret_cast<const uint4*>(pt);
        uint4 c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = (uint32_t(16 * i) < rem) ? q[i] : make_uint4(0u, 0u, 0u, 0u);
        be16_from_raw(c, w);
    } else {
        uint32_t d[20];
#if NKV_EXP_NOTAIL
        // traffic experiment only (wrong digests): no load of the tail window
#pragma unroll
        for (int k = 0; k < 20; ++k) d[k] = 0u;
#else
        load_window(pt, rem, d);
#endif
        be16_funnel(d, uint32_t(reinterpret_cast<uintptr_t>(pt) & 15), w);
    }
    hook.tail(w, rem);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int v = int(rem) - 4 * j;  // value bytes inside word j
        uint32_t m = v >= 4 ? 0xFFFFFFFFu : (v <= 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * v)));
        uint32_t x = w[j] & m;
        if (v >= 0 && v < 4) x |= 0x80u << (24 - 8 * v);
        w[j] = x;
    }
    const bool two = rem >= 56;
    if (!two) {
        w[14] = uint32_t(bits >> 32);
        w[15] = uint32_t(bits);
    }
    sha1_compress(h, w);
    if (__any(two)) {
        uint32_t h2[5];
#pragma unroll
        for (int j = 0; j < 14; ++j) w[j] = 0u;
        w[14] = uint32_t(bits >> 32);
        w[15] = uint32_t(bits);
#pragma unroll
        for (int i = 0; i < 5; ++i) h2[i] = h[i];
        sha1_compress(h2, w);
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] = two ? h2[i] : h[i];
    }
}

// Full 64-byte blocks of the 64 values owned by one wavefront, streamed
// HBM -> LDS with LDS-DMA (global_load_lds_dwordx4: no VGPR staging, fully
// used 64-byte runs per request), one 4 KiB stage per block, wave-private.
//
// Stage layout: value j's block at wbuf + 64 j, its 16-byte chunk q stored
// at chunk slot q ^ ((j >> 2) & 3), so the four ds_read_b128 of a block are
// bank-conflict free (every 16-lane ds_read_b128 group hits 16 distinct
// 16-byte bank slots).  DMA instruction k (k = 0..3) fills values
// 16k .. 16k+15: lane l loads chunk (l & 3) ^ ((l >> 4) & 3) of value
// 16k + (l >> 2), which lands at wbuf + 1024 k + 16 l -- exactly its slot.
//
// src[k] = chunk address of block 0 for this lane's DMA role k; nf[k] = full
// blocks of that value (0 for a dead lane).  my_nfull: this lane's own value.
// Wave reductions by ds_swizzle (xor pattern in the instruction, within each
// 32-lane half) and two readlanes: no lane-index VGPRs, which __shfl_xor
// computes once and the compiler then keeps live through a whole kernel.
template <int X>
__device__ __forceinline__ uint32_t swz_xor(uint32_t v) {
    return uint32_t(__builtin_amdgcn_ds_swizzle(int(v), (X << 10) | 0x1F));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, swz_xor<1>(v));
    v = max(v, swz_xor<2>(v));
    v = max(v, swz_xor<4>(v));
    v = max(v, swz_xor<8>(v));
    v = max(v, swz_xor<16>(v));
    return max(uint32_t(__builtin_amdgcn_readlane(int(v), 0)), uint32_t(__builtin_amdgcn_readlane(int(v), 32)));
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, swz_xor<1>(v));
    v = min(v, swz_xor<2>(v));
    v = min(v, swz_xor<4>(v));
    v = min(v, swz_xor<8>(v));
    v = min(v, swz_xor<16>(v));
    return min(uint32_t(__builtin_amdgcn_readlane(int(v), 0)), uint32_t(__builtin_amdgcn_readlane(int(v), 32)));
}

template <int X>
__device__ __forceinline__ uint64_t min_swz64(uint64_t v) {
    const uint64_t u = (uint64_t(swz_xor<X>(uint32_t(v >> 32))) << 32) | swz_xor<X>(uint32_t(v));
    return u < v ? u : v;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    v = min_swz64<1>(v);
    v = min_swz64<2>(v);
    v = min_swz64<4>(v);
    v = min_swz64<8>(v);
    v = min_swz64<16>(v);
    const uint64_t a = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), 0))) << 32) |
                       uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), 0));
    const uint64_t b = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), 32))) << 32) |
                       uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), 32));
    return a < b ? a : b;
}

// issue(b) starts the four DMA instructions of block b (each lane for its DMA
// role); nmax = the wave's largest full-block count (wave-uniform).  raw(c, w)
// sees each of this lane's blocks as loaded (four little-endian quads) and as
// the 16 big-endian words SHA-1 takes (k_leaf_verify checksums them there);
// be(w), for the stages that only form the big-endian words.
struct NoRaw {
    __device__ __forceinline__ void operator()(const uint4*, const uint32_t*) const {}
    __device__ __forceinline__ void be(const uint32_t*) const {}
    __device__ __forceinline__ void tail(const uint32_t*, uint32_t) const {}
};

template <class Issue, class Raw = NoRaw>
__device__ __forceinline__ void sha1_blocks_lds(const uint8_t* wbuf, uint32_t nmax, uint32_t my_nfull,
                                                Issue issue, uint32_t h[5], Raw raw = Raw{}) {
    const int lane = threadIdx.x & 63;
    const uint4* rd = reinterpret_cast<const uint4*>(wbuf + 64 * lane);
    const uint32_t swz = (uint32_t(lane) >> 2) & 3u;
    uint32_t w[16];
    if (nmax == 0) return;
    issue(0u);
    for (uint32_t b = 0; b < nmax; ++b) {
        // block b's DMA has landed.  Explicit: the compiler's own LDS-DMA wait
        // depends on its alias analysis of the stage (a second __shared__
        // object in the kernel once made it drop this wait).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint4 c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = rd[q ^ swz];
        be16_from_raw(c, w);
        if (b + 1 < nmax) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // stage reads done before refill
            issue(b + 1);
        }
        if (b < my_nfull) {
            raw(c, w);
            sha1_compress(h, w);
        }
    }
}

// Full blocks in runs of S blocks: each lane loads S*64 contiguous bytes of its
// value (4S x global_load_dwordx4) before compressing them, so every request
// stream touches a DRAM page for a longer run.
template <int S>
__device__ __forceinline__ void sha1_blocks_runs(const uint8_t* p, uint32_t nfull, uint32_t h[5]) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint32_t w[16];
    uint32_t b = 0;
    for (; b + S <= nfull; b += S) {
        uint4 c[4 * S];
#pragma unroll
        for (int i = 0; i < 4 * S; ++i) c[i] = q[4 * b + i];
#pragma unroll
        for (int j = 0; j < S; ++j) {
            be16_from_raw(c + 4 * j, w);
            sha1_compress(h, w);
        }
    }
    for (; b < nfull; ++b) {
        uint4 c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = q[4 * b + i];
        be16_from_raw(c, w);
        sha1_compress(h, w);
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ds_read_b128_asm(uint32_t addr) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
    return v;
}
template <int OFF>
__device__ __forceinline__ u32x4 ds_read_b128_off(uint32_t addr) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
    return v;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Pipelined ring over VALUE-relative chunks: chunk c of a value is its bytes
// [64c, 64c + 64), fetched by LDS-DMA from the value's own (unaligned) address,
// so the LDS row already holds block c and no funnel is needed (16 v_perm
// byte swaps per block instead of 52).  Only full blocks are fetched, so every
// byte read belongs to the value.  A lane past its value's last block re-reads
// that block (a value with none re-reads another of the wave), so each issue is four
// wave-instructions.  Window b = chunk b; at block b the ring holds chunks
// b+1 .. b+R, and vmcnt(4 (R-1)) before reading window b+1 lets chunks
// b+2 .. b+R fly (R-1 blocks of lookahead).
// sink(b, w): block b's 16 big-endian words (clobbered), every lane, every
// b < the wave's longest value (sha1_blocks_ring_vc compresses the lane's own)
template <int R, class Sink>
__device__ __forceinline__ void ring_vc_blocks(uint8_t* wbuf, const uint8_t* p, uint32_t my_nfull, Sink&& sink) {
    static_assert(R >= 2 && R <= 4, "ring depth");
    const int lane = threadIdx.x & 63;
    // DMA role k of this lane: chunk (lane & 3) of value 16 k + (lane >> 2),
    // which lands at wbuf + 1024 k + 16 lane = row 64 j + 16 (lane & 3): rows
    // unswizzled, so a lane reads its window at one base + immediate offsets
    // (the 4-way bank conflicts cost LDS cycles the VALU-bound loop has spare)
    const uint32_t dq = uint32_t(lane) & 3u;
    const uint32_t nmax = wave_max_u32(my_nfull);
    if (nmax == 0) return;
    // wave base: the lowest value address among lanes with a full block
    const uint64_t pa = reinterpret_cast<uintptr_t>(p);
    const uint64_t wb = wave_min_u64(my_nfull ? pa : ~uint64_t(0));
    const uint32_t minfull = wave_min_u32(my_nfull ? my_nfull : 0xFFFFFFFFu);
    const uint32_t wb_nfull = wave_max_u32(my_nfull && pa == wb ? my_nfull : 0u);
    uint64_t relk[4];
    uint32_t lastk[4];  // byte offset of the role value's last full block
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = 16 * k + (lane >> 2);
        const uint64_t aj = uint64_t(__shfl(int64_t(pa), j));
        const uint32_t nj = uint32_t(__shfl(int(my_nfull), j));
        // a role whose value has no full block re-reads the wave base's value
        relk[k] = (nj ? aj - wb : 0ull) + 16u * dq;
        lastk[k] = 64u * ((nj ? nj : wb_nfull) - 1u);
    }
    const uint8_t* base = reinterpret_cast<const uint8_t*>(wb);
    const bool near = __all(relk[0] + lastk[0] <= 0xFFFFFFFFull && relk[1] + lastk[1] <= 0xFFFFFFFFull &&
                            relk[2] + lastk[2] <= 0xFFFFFFFFull && relk[3] + lastk[3] <= 0xFFFFFFFFull);
    uint32_t rel[4], lastabs[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rel[k] = uint32_t(relk[k]);
        lastabs[k] = uint32_t(relk[k]) + lastk[k];
    }
    // Chunk c: while every live value still has block c (c < minfull) the
    // offsets are the per-role constants rel[k] from the uniform base + 64 c
    // (saddr-form DMA, no VALU); past that, each role clamps to its value's
    // last full block (a lane past its value re-reads it).  Waves whose values
    // lie more than 4 GiB apart take 64-bit addresses throughout.
    // buffer descriptor over [wb, wb + 4 GiB): the uniform chunk offset rides
    // in soffset, so the in-range issue has no VALU at all
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), short(0), int(0xFFFFFFFF), 0x00020000);
    auto issue = [&](uint32_t c) {
        uint8_t* dst = wbuf + 4096 * (c % R);
        const uint32_t cb = 64u * c;
        if (near && c < minfull) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void*)(dst + 1024 * k), 16, rel[k],
                    int(cb), 0, 0);
        } else if (near) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void*)(dst + 1024 * k), 16,
                    min(rel[k] + cb, lastabs[k]), 0, 0, 0);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_global_load_lds(base + (relk[k] + min(cb, lastk[k])), dst + 1024 * k, 16, 0, 0);
        }
    };
    const uint32_t row = uint32_t(reinterpret_cast<uintptr_t>(wbuf)) + 64u * uint32_t(lane);
    auto read_window = [&](uint32_t b, u32x4 v[4]) {
        const uint32_t s0 = row + 4096u * (b % R);  // one VALU; the chunks at immediate offsets
        v[0] = ds_read_b128_off<0>(s0);
        v[1] = ds_read_b128_off<16>(s0);
        v[2] = ds_read_b128_off<32>(s0);
        v[3] = ds_read_b128_off<48>(s0);
    };
    // block b from cur while window b+1 lands in nxt; the loop below runs it
    // twice per iteration with the roles swapped, so no window is copied
    auto step = [&](uint32_t b, u32x4 cur[4], u32x4 nxt[4]) {
        issue(b + R);
        wait_vmcnt<4 * (R - 1)>();
        read_window(b + 1, nxt);
        uint4 c4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c4[q] = make_uint4(cur[q].x, cur[q].y, cur[q].z, cur[q].w);
        uint32_t w[16];
        be16_from_raw(c4, w);
        sink(b, w);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nxt[0]), "+v"(nxt[1]), "+v"(nxt[2]), "+v"(nxt[3]) : : "memory");
    };
#pragma unroll
    for (uint32_t c = 0; c < uint32_t(R); ++c) issue(c);
    wait_vmcnt<4 * (R - 1)>();
    u32x4 wa[4], wb4[4];
    read_window(0u, wa);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wa[0]), "+v"(wa[1]), "+v"(wa[2]), "+v"(wa[3]) : : "memory");
    uint32_t b = 0;
    for (; b + 2 <= nmax; b += 2) {
        step(b, wa, wb4);
        step(b + 1, wb4, wa);
    }
    if (b < nmax) step(b, wa, wb4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int R>
__device__ __forceinline__ void sha1_blocks_ring_vc(uint8_t* wbuf, const uint8_t* p, uint32_t my_nfull,
                                                    uint32_t h[5]) {
    ring_vc_blocks<R>(wbuf, p, my_nfull, [&](uint32_t b, uint32_t w[16]) {
        // the live lanes only: compressing in every lane (into a copy a lane
        // past its value drops) measured no faster on configs[2] and ran the
        // clock 1-2 % lower (profiles/r06_ab_ring_lanes.txt): its sorted groups
        // keep waves nearly full, unlike the small trees (sha1_value_all_lanes)
        if (b < my_nfull) sha1_compress(h, w);
    });
}

// The 80-byte window stage for values that are not 64-byte aligned and whose
// full-block counts are equal across the wave (records of one size whose
// offsets mod 64 differ).  Block b of a value at o = p & 63 lies in the five
// aligned quads from (p & ~15) + 64 b; five LDS-DMA instructions per block
// fetch them for all 64 values (quad g = 64 k + l of instruction k is quad
// g % 5 of value g / 5; quads past o + 63 are clamped to the last needed one,
// so every request is aligned, inside one line, and inside a line that holds
// bytes of the value's block).  Value j's row is 80 contiguous bytes at wbuf +
// 80 j, and the lane reads its 64-byte window with four byte-unaligned
// ds_read_b128 at 80 j + (o & 15): no register funnel, 16 v_perm per block as
// in the aligned path.  The addresses are a 32-bit offset per role from a
// wave-uniform base plus the uniform 64 b (the wave's rows must lie within 4
// GiB of the base).  Stage: 5 KiB per wave (eight waves per SIMD fit the 160 KiB
// LDS).  Returns false, doing nothing, when the wave does not qualify; the
// caller then runs the value-relative stream.
__device__ __forceinline__ bool sha1_blocks_pair(uint8_t* wbuf, const uint8_t* p, bool live, uint32_t my_nfull,
                                                 uint32_t h[5]) {
    constexpr int kDma = 5;  // DMA instructions per block
    constexpr uint32_t kRow = 80u;
    const int lane = threadIdx.x & 63;
    const uint32_t nmax = wave_max_u32(live ? my_nfull : 0u);
    if (nmax == 0) return true;  // no live value has a full block
    if (!__all(!live || my_nfull == nmax)) return false;
    const uint64_t a = reinterpret_cast<uintptr_t>(p) & ~uint64_t(63);
    const uint64_t wb = wave_min_u64(live ? a : ~uint64_t(0));
    const uint64_t rel = live ? a - wb : 0u;
    if (!__all(rel + 64ull * (uint64_t(nmax) + 1ull) <= 0xFFFFFFFFull)) return false;
    const uint32_t o = live ? uint32_t(reinterpret_cast<uintptr_t>(p) & 63u) : 0u;
    const uint8_t* base = reinterpret_cast<const uint8_t*>(wb);
    // lane 0 is live whenever any lane is (dead lanes are the grid's tail), so
    // dead values' roles re-read lane 0's quads into their unused rows
    uint32_t voff[kDma];
#pragma unroll
    for (int k = 0; k < kDma; ++k) {
        const uint32_t g = 64u * uint32_t(k) + uint32_t(lane);
        const int j = int(g / 5u);
        const uint32_t qi = g - 5u * uint32_t(j);
        const bool lj = __shfl(int(live), j) != 0;
        const uint32_t src = lj ? uint32_t(j) : 0u;
        const uint32_t rj = uint32_t(__shfl(int(uint32_t(rel)), int(src)));
        const uint32_t oj = uint32_t(__shfl(int(o), int(src)));
        const uint32_t qlast = (oj + 63u) >> 4;
        voff[k] = rj + 16u * min((oj >> 4) + qi, qlast);
    }
    auto issue = [&](uint32_t b) {
        const uint32_t cb = 64u * b;
#pragma unroll
        for (int k = 0; k < kDma; ++k) __builtin_amdgcn_global_load_lds(base + (voff[k] + cb), wbuf + 1024 * k, 16, 0, 0);
    };
    const uint32_t rd = uint32_t(reinterpret_cast<uintptr_t>(wbuf)) + kRow * uint32_t(lane) + (o & 15u);
    issue(0u);
    for (uint32_t b = 0; b < nmax; ++b) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ds_read_b128_asm(rd + 16u * uint32_t(q));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) : : "memory");
        if (b + 1 < nmax) issue(b + 1);
        uint4 c4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c4[q] = make_uint4(v[q].x, v[q].y, v[q].z, v[q].w);
        uint32_t w[16];
        be16_from_raw(c4, w);
        if (live) sha1_compress(h, w);
    }
    return true;
}

// LOAD 11: values that share one misalignment o = (address mod 64) != 0
// across the wave (Data-table records of one size: Value at rec + 30 + KeySize,
// record.go:191-199).  Each lane streams its value's 64-byte ALIGNED segments
// straight into registers, in order, once: block b's window is bytes
// [o, o + 64) of segments b, b + 1, so segment b + 1 is loaded for block b and
// kept for block b + 1 (two register sets swap roles; the loop is unrolled by
// two).  The L2 then sees every 128-byte line requested by one lane in two
// consecutive blocks, as for 64-byte aligned values, where the window stages
// (LOAD 8/9/10) request each line in three consecutive blocks and the line
// falls out of the 4 MiB L2 in between (records form).
// The funnel is the 16 v_perm_b32 byte swaps the aligned path runs anyway: o is
// wave-uniform, so the dword offset o >> 2 selects one of 16 straight-line
// register patterns (scalar branch) and the byte offset o & 3 is the v_perm
// selector (an SGPR).  Every segment loaded holds a byte of the value's full
// blocks, so no load steps past the value's last full block (no page beyond
// the buffer is touched).  No LDS.  Returns false (and does nothing) when the
// wave's live values do not share o, or o == 0.
template <int Q>
__device__ __forceinline__ void funnel_q(const uint32_t a[16], const uint32_t b[16], uint32_t sel, uint32_t w[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int j = Q + i;  // dword j of the 32-dword pair (a, b): the window's dword i
        const uint32_t lo = j < 16 ? a[j] : b[j - 16];
        const uint32_t hi = j + 1 < 16 ? a[j + 1] : b[j - 15];
        w[i] = be_word(hi, lo, sel);
    }
}

__device__ __forceinline__ void funnel_u(uint32_t q, const uint32_t a[16], const uint32_t b[16], uint32_t sel,
                                         uint32_t w[16]) {
    switch (q) {
        case 0: funnel_q<0>(a, b, sel, w); break;
        case 1: funnel_q<1>(a, b, sel, w); break;
        case 2: funnel_q<2>(a, b, sel, w); break;
        case 3: funnel_q<3>(a, b, sel, w); break;
        case 4: funnel_q<4>(a, b, sel, w); break;
        case 5: funnel_q<5>(a, b, sel, w); break;
        case 6: funnel_q<6>(a, b, sel, w); break;
        case 7: funnel_q<7>(a, b, sel, w); break;
        case 8: funnel_q<8>(a, b, sel, w); break;
        case 9: funnel_q<9>(a, b, sel, w); break;
        case 10: funnel_q<10>(a, b, sel, w); break;
        case 11: funnel_q<11>(a, b, sel, w); break;
        case 12: funnel_q<12>(a, b, sel, w); break;
        case 13: funnel_q<13>(a, b, sel, w); break;
        case 14: funnel_q<14>(a, b, sel, w); break;
        default: funnel_q<15>(a, b, sel, w); break;
    }
}

__device__ __forceinline__ void load_seg(const uint4* s, uint32_t r[16]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = s[q];
        r[4 * q + 0] = v.x;
        r[4 * q + 1] = v.y;
        r[4 * q + 2] = v.z;
        r[4 * q + 3] = v.w;
    }
}

// LINES: whole 128-byte lines into registers when the values' segments start
// lines (the caller's kernel must afford ~86 VGPRs: k_leaf_records runs 5
// waves per SIMD); else the LDS-DMA stage or 64-byte register segments.
template <class Hook = NoRaw, bool LINES = false>
__device__ __forceinline__ bool sha1_blocks_shift(uint8_t* wbuf, const uint8_t* p, bool live, uint32_t my_nfull,
                                                  uint32_t h[5], Hook hook = Hook{}) {
    const uint32_t o = live ? uint32_t(reinterpret_cast<uintptr_t>(p) & 63u) : 0u;
    // lane 0 is live whenever any lane is (dead lanes are the grid's tail)
    const uint32_t o0 = __builtin_amdgcn_readfirstlane(o);
    if (o0 == 0u || !__all(!live || o == o0)) return false;
    const uint32_t nmax = wave_max_u32(live ? my_nfull : 0u);
    if (nmax == 0) return true;
    const uint32_t q = o0 >> 2;
    const uint32_t sel = be_sel(o0 & 3u);
    uint32_t a[16], b[16], w[16];
    // Whole 128-byte lines into registers: when every live value's segment 0
    // starts a line and the block counts are equal, each lane loads its aligned
    // lines (two segments, eight 16-byte loads) once, no LDS.  Three segment
    // sets rotate over four blocks: block k takes segments k and k + 1.  Every
    // line loaded holds a needed segment, so no load leaves the value's pages.
    if (LINES && __all(!live || my_nfull == nmax) &&
        __all(!live || ((reinterpret_cast<uintptr_t>(p) - o) & 64u) == 0u)) {
        const uint4* seg = reinterpret_cast<const uint4*>(live ? p - o : p);
        uint32_t c[16];
        auto line = [&](uint32_t sg, uint32_t x[16], uint32_t y[16]) {
            if (live) {
                load_seg(seg + 4 * sg, x);
                load_seg(seg + 4 * (sg + 1), y);
            }
        };
        auto block = [&](const uint32_t lo[16], const uint32_t hi[16]) {
            funnel_u(q, lo, hi, sel, w);
            if (live) {
                hook.be(w);
                sha1_compress(h, w);
            }
            asm volatile("" ::: "memory");  // the next line's loads stay after this compress
        };
#if NKV_EXP_REC == 1
        // experiment: four segment sets, each line issued one block before
        // the block that first needs it (4 waves per SIMD)
        uint32_t d[16];
        line(0u, a, b);
        if (nmax >= 2) line(2u, c, d);
        for (uint32_t k = 0; k < nmax; k += 4) {
            block(a, b);  // k, k + 1
            if (k + 1 >= nmax) break;
            block(b, c);  // k + 1, k + 2
            if (k + 2 >= nmax) break;
            if (k + 4 <= nmax) line(k + 4, a, b);
            block(c, d);  // k + 2, k + 3
            if (k + 3 >= nmax) break;
            block(d, a);  // k + 3, k + 4
            if (k + 4 >= nmax) break;
            if (k + 6 <= nmax) line(k + 6, c, d);
        }
        return true;
#elif NKV_EXP_REC == 2
        // experiment: three segment sets, each 64-byte segment issued one block
        // before the block that first needs it (the two halves of a line are
        // requested one block apart)
        auto segl = [&](uint32_t sg, uint32_t x[16]) {
            if (live && sg <= nmax) load_seg(seg + 4 * sg, x);
        };
        segl(0u, a);
        segl(1u, b);
        for (uint32_t k = 0; k < nmax; k += 3) {
            segl(k + 2, c);
            block(a, b);  // k, k + 1
            if (k + 1 >= nmax) break;
            segl(k + 3, a);
            block(b, c);  // k + 1, k + 2
            if (k + 2 >= nmax) break;
            segl(k + 4, b);
            block(c, a);  // k + 2, k + 3
        }
        return true;
#else
        line(0u, a, b);
        for (uint32_t k = 0; k < nmax; k += 4) {
            block(a, b);  // segments k, k + 1
            if (k + 1 >= nmax) break;
            line(k + 2, a, c);
            block(b, a);  // k + 1, k + 2
            if (k + 2 >= nmax) break;
            block(a, c);  // k + 2, k + 3
            if (k + 3 >= nmax) break;
            line(k + 4, a, b);
            block(c, a);  // k + 3, k + 4
        }
        return true;
#endif
    }
    if (wbuf && __all(!live || my_nfull == nmax)) {
        // Equal block counts: the segments go HBM -> LDS by LDS-DMA, one segment
        // of lookahead, in k_leaf's aligned stage layout (value j's segment at
        // wbuf + 64 j, chunks XOR-swizzled; sha1_blocks_lds), then into the
        // register pair.  32-bit offsets from a wave-uniform base (one VGPR per
        // DMA role) keep the register pair and the schedule within 64 VGPRs.
        const uint64_t sa = reinterpret_cast<uintptr_t>(p) - o;
        const uint64_t wb = wave_min_u64(live ? sa : ~uint64_t(0));
        const uint64_t rel = live ? sa - wb : 0u;
        if (__all(rel + 64ull * (uint64_t(nmax) + 1ull) <= 0xFFFFFFFFull)) {
            const int lane = threadIdx.x & 63;
            const uint8_t* base = reinterpret_cast<const uint8_t*>(wb);
            const uint32_t cq = (uint32_t(lane) & 3u) ^ ((uint32_t(lane) >> 4) & 3u);
            uint32_t voff[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                // dead values' roles re-read lane 0's segments into unused rows
                const int j = 16 * k + (lane >> 2);
                const bool lj = __shfl(int(live), j) != 0;
                voff[k] = uint32_t(__shfl(int(uint32_t(rel)), lj ? j : 0)) + 16u * cq;
            }
            auto issue = [&](uint32_t sg) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    __builtin_amdgcn_global_load_lds(base + (voff[k] + 64u * sg), wbuf + 1024 * k, 16, 0, 0);
            };
            // chunk c of this lane's segment sits at (wbuf + 64 lane) + 16 (c ^ swz)
            // = rd0 ^ 16 c with rd0 = wbuf + 64 lane + 16 swz (64-B aligned rows).
            // One address VGPR, the other three are recomputed per read (the
            // asm hides rd0 from hoisting: four live addresses spill at 64 VGPRs)
            const uint32_t rd0 = uint32_t(reinterpret_cast<uintptr_t>(wbuf)) + 64u * uint32_t(lane) +
                                 16u * ((uint32_t(lane) >> 2) & 3u);
            auto take = [&](uint32_t r[16]) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                uint32_t ra = rd0;
                asm volatile("" : "+v"(ra));
                u32x4 v[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) v[c] = ds_read_b128_asm(ra ^ (16u * uint32_t(c)));
                // stage read before its refill; the in/out operands keep the
                // registers from being used before the wait
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) : : "memory");
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    r[4 * c + 0] = v[c].x;
                    r[4 * c + 1] = v[c].y;
                    r[4 * c + 2] = v[c].z;
                    r[4 * c + 3] = v[c].w;
                }
            };
            // segments 0 .. nmax (block k's window spans segments k and k + 1)
            issue(0u);
            take(a);
            issue(1u);
            // sched_barrier: no instruction crosses a phase boundary, so the
            // scheduler cannot overlap one block's compression with the next
            // block's reads and funnel (two windows live at 64 VGPRs spill)
            for (uint32_t k = 0; k < nmax; k += 2) {
                take(b);  // segment k + 1
                if (k + 2 <= nmax) issue(k + 2);
                funnel_u(q, a, b, sel, w);
                __builtin_amdgcn_sched_barrier(0);
                if (live) {
                    hook.be(w);
                    sha1_compress(h, w);
                }
                __builtin_amdgcn_sched_barrier(0);
                if (k + 1 >= nmax) break;
                take(a);  // segment k + 2
                if (k + 3 <= nmax) issue(k + 3);
                funnel_u(q, b, a, sel, w);
                __builtin_amdgcn_sched_barrier(0);
                if (live) {
                    hook.be(w);
                    sha1_compress(h, w);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            return true;
        }
    }
    // p - o, not an integer-to-pointer cast: stays in the global address space
    const uint4* seg = reinterpret_cast<const uint4*>(live ? p - o : p);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        a[i] = 0u;
        b[i] = 0u;
    }
    if (my_nfull) load_seg(seg, a);
    for (uint32_t k = 0; k < nmax; k += 2) {
        // block k: segments k (a) and k + 1 (b)
        if (k < my_nfull) load_seg(seg + 4 * (k + 1), b);
        funnel_u(q, a, b, sel, w);
        if (k < my_nfull) {
            hook.be(w);
            sha1_compress(h, w);
        }
        // keep each load after the previous compress: hoisted above it, a
        // segment set would be live through the compress and spill at 64 VGPRs
        // (the other resident waves cover the load latency)
        asm volatile("" ::: "memory");
        if (k + 1 >= nmax) break;
        // block k + 1: segments k + 1 (b) and k + 2 (a)
        if (k + 1 < my_nfull) load_seg(seg + 4 * (k + 2), a);
        funnel_u(q, b, a, sel, w);
        if (k + 1 < my_nfull) {
            hook.be(w);
            sha1_compress(h, w);
        }
        asm volatile("" ::: "memory");
    }
    return true;
}

// The full blocks of a wave's 64 values at any addresses (wbuf: the wave's
// 5 KiB of LDS): the segment stage when the values share their offset mod 64,
// else the 80-byte window stage when their full-block counts are equal, else
// the value-relative stream.  k_leaf's LOAD 11 for MODE 1 and k_leaf_records.
template <bool LINES = false>
__device__ __forceinline__ void sha1_blocks_any(uint8_t* wbuf, const uint8_t* p, bool live, uint32_t my_nfull,
                                                uint32_t h[5]) {
    if (sha1_blocks_shift<NoRaw, LINES>(wbuf, p, live, my_nfull, h)) return;
    if (sha1_blocks_pair(wbuf, p, live, my_nfull, h)) return;
    const int lane = threadIdx.x & 63;
    const uint32_t q = (uint32_t(lane) & 3u) ^ ((uint32_t(lane) >> 4) & 3u);
    const uint8_t* src[4];
    uint32_t nf[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = 16 * k + (lane >> 2);
        const uint64_t pj = uint64_t(__shfl(int64_t(reinterpret_cast<uintptr_t>(p)), j));
        src[k] = reinterpret_cast<const uint8_t*>(pj) + 16 * q;
        nf[k] = uint32_t(__shfl(int(my_nfull), j));
    }
    auto issue = [&](uint32_t b) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (b < nf[k]) __builtin_amdgcn_global_load_lds(src[k] + 64ull * b, wbuf + 1024 * k, 16, 0, 0);
    };
    sha1_blocks_lds(wbuf, wave_max_u32(my_nfull), my_nfull, issue, h);
}


// MODE 0: value i at base + i*stride, length L.  MODE 1: base + off[i], len[i].
// perm (MODE 1 only, nullable): lane i hashes leaf perm[i]; a pass after
// k_leaf_records skips the values it hashed (off == kDone).
// No tree level is fused here: a wave-level step costs a whole SHA-1
// instruction stream however few lanes it keeps, so levels built inside the
// leaf kernel (6 per wave, or the workgroup's last wave finishing its 256-leaf
// subtree) cost 3-7 % of a 4 KiB leaf launch, more than k_reduce2 at full lane
// use plus its launch.
// LOAD 4: 16-byte aligned values in 128-byte runs straight into registers
// (sha1_blocks_runs<2>: eight global_load_dwordx4 per lane, every 128-byte line
// fetched once by one lane; 65 VGPRs, 7 waves per SIMD).  LOAD 11: values at
// any address, each wave by the first stage that fits it: the segment stage
// when its values share their offset mod 64 (sha1_blocks_shift), the 80-byte
// window stage when their full-block counts are equal (sha1_blocks_pair), else
// the value-relative LDS-DMA stream (sha1_blocks_lds).  The other load paths
// measured in rounds 1-2 (LDS-DMA stage for aligned values, direct and
// non-temporal loads, 256-byte runs, line-pair stage, runs at each value's own
// address, deep register prefetch) lost their A/Bs and are gone.
constexpr int kRunsWaves = 4;  // launch bound of the LOAD 4 kernel
template <int MODE, int LOAD>
__global__ __launch_bounds__(kBlock, LOAD == 4 ? kRunsWaves : kLeafWavesPerSimd) void k_leaf(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
    uint64_t stride, uint64_t L, const uint32_t* __restrict__ perm, uint64_t n, uint8_t* __restrict__ nodes,
    Gate gate) {
    static_assert(LOAD == 4 || LOAD == 11, "leaf load path");
    // LOAD 11: four wave-private 5 KiB stages (the window stage's 80-byte rows)
    __shared__ __attribute__((aligned(16))) uint8_t smem[LOAD == 11 ? kBlock * 80 : 16];
    if (!gate.open()) return;
    NKV_STAMP(0);
    const ClockProbe clk;
    const uint64_t g = blockIdx.x;
    const uint64_t t = g * kBlock + threadIdx.x;
    uint32_t h[5] = {0u, 0u, 0u, 0u, 0u};
    uint64_t leaf = t;
    // a length-sorted batch after k_leaf_records skips the values it hashed
    const bool live = t < n && (MODE == 0 || !perm || off[perm[t]] != kDone);
    const uint8_t* p = nullptr;
    uint64_t ln = 0;
    if (live) {
        if (MODE == 0) {
            p = base + t * stride;
            ln = L;
        } else {
            leaf = perm ? uint64_t(perm[t]) : t;
            p = base + off[leaf];
            ln = len[leaf];
        }
    }
    sha1_init(h);
    if constexpr (LOAD == 4) {
        if (live) {
            sha1_blocks_runs<2>(p, uint32_t(ln >> 6), h);
            // one length for all: a whole-block length's padding block is the
            // same message in every lane (its schedule on the scalar unit)
            if (MODE == 0 && (L & 63) == 0) sha1_pad_uniform(h, L);
            else sha1_tail<true>(p, ln, h);
            store_digest(nodes, leaf, h);
        }
    } else {
        // wave-cooperative stages of the full blocks, then the tail.  Every
        // stage reads only full blocks' bytes, so nothing past a value is read.
        const int lane = threadIdx.x & 63;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        uint8_t* wbuf = smem + 5120 * wave;
        const uint32_t q = (uint32_t(lane) & 3u) ^ ((uint32_t(lane) >> 4) & 3u);
        const uint32_t my_nfull = live ? uint32_t(ln >> 6) : 0u;
        bool staged = sha1_blocks_shift(wbuf, p, live, my_nfull, h);
        if (!staged) staged = sha1_blocks_pair(wbuf, p, live, my_nfull, h);
        if (staged) {
            // done (wave-uniform)
        } else if (MODE == 0) {
            // value j of this wave at wave_base + j * stride (32-bit offsets:
            // saddr-form DMA, one VGPR of addressing)
            const uint64_t first = g * kBlock + 64 * uint64_t(wave);
            const uint8_t* wave_base = base + first * stride;
            const uint32_t nvalid = first < n ? uint32_t(min(uint64_t(64), n - first)) : 0u;
            const uint32_t off0 = uint32_t(lane >> 2) * uint32_t(stride) + 16u * q;
            const uint32_t kstep = 16u * uint32_t(stride);
            const uint32_t nmax = nvalid ? uint32_t(L >> 6) : 0u;
            auto issue = [&](uint32_t b) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (uint32_t(16 * k + (lane >> 2)) < nvalid)
                        __builtin_amdgcn_global_load_lds(wave_base + (off0 + k * kstep + 64u * b),
                                                         wbuf + 1024 * k, 16, 0, 0);
            };
            sha1_blocks_lds(wbuf, nmax, my_nfull, issue, h);
        } else {
            const uint8_t* src[4];
            uint32_t nf[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 16 * k + (lane >> 2);
                const uint64_t pj = uint64_t(__shfl(int64_t(reinterpret_cast<uintptr_t>(p)), j));
                src[k] = reinterpret_cast<const uint8_t*>(pj) + 16 * q;
                nf[k] = uint32_t(__shfl(int(my_nfull), j));
            }
            auto issue = [&](uint32_t b) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (b < nf[k])
                        __builtin_amdgcn_global_load_lds(src[k] + 64ull * b, wbuf + 1024 * k, 16, 0, 0);
            };
            sha1_blocks_lds(wbuf, wave_max_u32(my_nfull), my_nfull, issue, h);
        }
        if constexpr (MODE == 1) {
            // reload the value's place instead of keeping it live through the
            // register stage (its two 16-dword segment sets need the VGPRs)
            asm volatile("" ::: "memory");
            if (live) {
                leaf = perm ? uint64_t(perm[t]) : t;
                p = base + off[leaf];
                ln = len[leaf];
            }
        }
        if (live) {
            sha1_tail<false>(p, ln, h);
            store_digest(nodes, leaf, h);
        }
    }
    clk.end();
    NKV_STAMP(1);
    NKV_STAMP(2);
#ifdef NKV_DIAG
    if (g_diag && (threadIdx.x & 63) == 0) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        const size_t w_ = size_t(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
        g_diag[w_ * 8 + 6] = (uint64_t(xcc) << 32) | hw;
    }
#endif
}

// k_leaf_verify's block hook: the CRC steps over the 16 big-endian words SHA-1
// takes, with the state byte-swapped (cs = bswap(crc)) against byte-swapped
// tables stored in reverse order (slot k = bswap(T[3 - k]), crc_dev.hpp), so
// the same x-form step indexes the right bytes and no extra byte swap runs.
// (Spreading the 16 steps over the rounds, one per one or two rounds, ran
// 0.3 % faster and 6 % slower: the lookups' latency is not what bounds it.)
struct CrcBE {
    uint32_t& cs;
    const uint32_t* swtab;
    const uint32_t* tab0;  // T[0], for the last 0-3 bytes
    __device__ __forceinline__ void be(const uint32_t* w) { cs = crc_block16<1>(cs, w, swtab); }
    __device__ __forceinline__ void operator()(const uint4*, const uint32_t* w) { be(w); }
    // the first nb (<= 64) bytes held by 16 big-endian words: whole words in
    // the swapped domain, then the 0-3 bytes of the partial word
    __device__ __forceinline__ void span(const uint32_t* w, uint32_t nb) {
        const uint32_t nfw = nb >> 2;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t u = crc_x_last<1>(cs ^ w[i], swtab);
            cs = uint32_t(i) < nfw ? u : cs;
        }
        uint32_t pw = 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i) pw = uint32_t(i) == nfw ? w[i] : pw;
        uint32_t crc = __builtin_bswap32(cs);
        for (uint32_t b = 0; b < (nb & 3u); ++b) crc = crc_byte<1>(crc, (pw >> (24u - 8u * b)) & 0xFFu, tab0);
        cs = __builtin_bswap32(crc);
    }
    // the value's last rem (< 64) bytes, from the words sha1_tail loaded
    __device__ __forceinline__ void tail(const uint32_t* w, uint32_t rem) { span(w, rem); }
};

// K1v: the compaction read of a Data table in one pass.  For every record it
// checks record.Deserialize's checksum (record.go:163-169: crc32.ChecksumIEEE
// of Key ++ Value against the stored Crc) and computes NewLeaf(Value)
// (merklenode.go:27-34), reading each byte once.  The value-relative LDS-DMA
// stream of k_leaf (LOAD 8) feeds both: each 64-byte block's 16 little-endian
// words step the CRC (slicing-by-4 from one LDS table copy) before the byte
// swap feeds SHA-1.  The key, which precedes the value, and the value's tail
// are checksummed bytewise from global memory.  SHA-1 is VALU-bound and leaves
// the LDS nearly idle, so the lookups ride along.  A record whose header points
// outside the stream sets stats[2] and gets the digest of an empty value, as
// in nkv_tree_from_records_dev.
//
// The header parse is k_locate's, so no separate locate pass runs.  policy
// (as k_leaf_records): 0 hashes every wave here; 1 (auto) hashes the waves
// whose value block counts are narrow by the plan rule and defers the others;
// 2 defers all.  A deferred wave only checksums its records here (crc_span
// over Key ++ Value, the CRC is cheap next to SHA-1) and leaves each value's
// voff / vlen for the length-sorted leaf pass; a hashed value's voff becomes
// kDone.  Each workgroup leaves (0, deferred ? ~0 : 0, 0) in part, folded by
// k_locate_fold into the range whose wide Gate opens the sorted pass.
constexpr int kVerifyWaves = 4;  // whole lines in registers with the CRC state: ~105 VGPRs
__global__ __launch_bounds__(kBlock, kVerifyWaves) void k_leaf_verify(
    const uint8_t* __restrict__ stream, uint64_t stream_len, const uint64_t* __restrict__ rec_off, uint64_t n,
    int policy, uint64_t* __restrict__ voff, uint64_t* __restrict__ vlen, uint8_t* __restrict__ nodes,
    uint32_t* __restrict__ crc_out, unsigned long long* __restrict__ stats, uint32_t* __restrict__ part,
    uint32_t* __restrict__ flags, uint32_t* __restrict__ flags_next) {
    if (flags) pass_flags_reset(flags_next);
    const ClockProbe clk;
    // ONE LDS object (a second one can cost the DMA loop its waits): four
    // 4 KiB wave stages, the 4 KiB of byte-swapped word tables (CrcBE), then
    // T[0] for the bytewise steps: 21 KiB, seven workgroups per CU
    __shared__ __attribute__((aligned(16))) uint8_t smem[kBlock * 64 + 4096 + 1024];
    uint32_t* swtab = reinterpret_cast<uint32_t*>(smem + kBlock * 64);
    uint32_t* tab = swtab + 4 * 256;
    for (int i = threadIdx.x; i < 4 * 256; i += kBlock)
        swtab[i] = __builtin_bswap32(c_crc_leaf.t[3 - (i >> 8)][i & 255]);
    for (int i = threadIdx.x; i < 256; i += kBlock) tab[i] = c_crc_leaf.t[0][i];
    __syncthreads();
    const uint64_t t = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool live = t < n;
    const uint8_t* key = stream;
    const uint8_t* p = stream;
    uint64_t ks = 0, ln = 0;
    uint32_t stored = 0;
    bool hdr_bad = false;
    if (live) {
        const uint64_t r = rec_off[t];
        if (header_in(r, stream_len)) {
            uint64_t k, v;
            ld_header_sizes(stream + r, k, v);
            if (k <= stream_len && v <= stream_len && r + 30 + k + v <= stream_len) {
                key = stream + r + 30;
                ks = k;
                p = key + k;
                ln = v;
                // the stored Crc (header bytes 0..3) from the one or two aligned
                // words that hold it
                const uint8_t* c = stream + r;
                const uint32_t mis = uint32_t(reinterpret_cast<uintptr_t>(c) & 3u);
                const uint32_t* cw = reinterpret_cast<const uint32_t*>(c - mis);
                const uint32_t c0 = cw[0];
                const uint32_t c1 = mis ? cw[1] : 0u;
                stored = mis ? (c0 >> (8u * mis)) | (c1 << (32u - 8u * mis)) : c0;
            } else {
                hdr_bad = true;
            }
        } else {
            hdr_bad = true;
        }
    }
    const uint64_t bl = ln >> 6;
    const uint32_t my_nfull = bl > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(bl);
    const uint32_t wlo = wave_min_u32(live ? my_nfull : 0xFFFFFFFFu);
    const uint32_t whi = wave_max_u32(live ? my_nfull : 0u);
    const bool any = __any(live);
    const bool hash = any && (policy == 0 || (policy == 1 && whi <= wlo + max(1u, wlo / 16u)));
    uint32_t crc;
    if (hash) {
        uint32_t cs = 0xFFFFFFFFu;  // bswap(~0): the CRC starts in the swapped domain
        CrcBE hook{cs, swtab, tab};
        {  // the key, 64 bytes at a time from aligned 16-byte loads (most keys: one pass)
            const uint32_t kch = wave_max_u32(uint32_t(min<uint64_t>((ks + 63) >> 6, 0xFFFFFFFFull)));
            for (uint32_t c = 0; c < kch; ++c) {
                const uint64_t done = 64ull * c;
                const uint32_t avail = ks > done ? uint32_t(min<uint64_t>(64ull, ks - done)) : 0u;
                const uint8_t* kc = key + (avail ? done : 0ull);
                uint32_t d[20], w[16];
                load_window(kc, avail, d);
                be16_funnel(d, uint32_t(reinterpret_cast<uintptr_t>(kc) & 15u), w);
                hook.span(w, avail);
            }
        }
        uint8_t* wbuf = smem + 4096 * wave;
        const uint32_t q = (uint32_t(lane) & 3u) ^ ((uint32_t(lane) >> 4) & 3u);
        uint32_t h[5];
        sha1_init(h);
        const uint8_t* src[4];
        uint32_t nf[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = 16 * k + (lane >> 2);
            const uint64_t pj = uint64_t(__shfl(int64_t(reinterpret_cast<uintptr_t>(p)), j));
            src[k] = reinterpret_cast<const uint8_t*>(pj) + 16 * q;
            nf[k] = uint32_t(__shfl(int(my_nfull), j));
        }
        auto issue = [&](uint32_t b) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (b < nf[k]) __builtin_amdgcn_global_load_lds(src[k] + 64ull * b, wbuf + 1024 * k, 16, 0, 0);
        };
        // records of one size share their offset mod 64: each line once
        // through the segment stage (LOAD 11); else the value-relative stream
        if (!sha1_blocks_shift<decltype(hook), true>(wbuf, p, live, my_nfull, h, hook))
            sha1_blocks_lds(wbuf, whi, my_nfull, issue, h, hook);
        if (live) {
            sha1_tail<false>(p, ln, h, hook);  // the tail's checksum from the same loads
            store_digest(nodes, t, h);
            if (voff) {
                voff[t] = kDone;
                vlen[t] = 0;
            }
        }
        crc = ~__builtin_bswap32(cs);
    } else {
        // deferred: Key ++ Value is one contiguous span of the record
        crc = crc_span<1, true>(key, ks + ln, tab, swtab);
        if (live) {
            voff[t] = uint64_t(p - stream);
            vlen[t] = ln;
        }
    }
    if (live) {
        if (crc_out) crc_out[t] = crc;
        if (hdr_bad) {
            atomicOr(stats + 2, 1ull);
        } else if (crc != stored) {
            atomicAdd(stats, 1ull);
            atomicMin(stats + 1, (unsigned long long)t);
        }
    }
    if (part || flags) {  // one partial per workgroup, through the (now idle) stage LDS
        const bool wdefer = any && !hash;
        uint32_t* wf = reinterpret_cast<uint32_t*>(smem);
        __syncthreads();
        if (lane == 0) wf[threadIdx.x >> 6] = wdefer ? 1u : 0u;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t f = 0u;
#pragma unroll
            for (int k = 0; k < kBlock / 64; ++k) f |= wf[k];
            if (flags) {
                if (f) pass_flag_raise(flags + 1, 0xFFFFFFFFu);
            } else {
                part[3 * blockIdx.x] = 0u;
                part[3 * blockIdx.x + 1] = f ? 0xFFFFFFFFu : 0u;
                part[3 * blockIdx.x + 2] = 0u;
            }
        }
    }
    clk.end();
}

// K1q: ragged batches, work-queue form.  Values are length-sorted, longest
// first, and cut into 64-value groups.  A group is one wavefront's work, and a
// group's 64 chains run as long as its longest value, so the batch can finish
// no sooner than its longest group.  Static dispatch places consecutive
// (= equally long) workgroups on one CU, which stacks the longest chains on a
// few SIMDs.  Here each wave (64-thread workgroup, two per SIMD) reads its
// SIMD id: the first wave on a SIMD pulls groups from the long end at priority
// 3, the others pull from the short end and fill the issue slots the long
// chain leaves.  The two ends meet; a per-group claim flag settles the last
// group.  Every wave exits once its end meets the other one.
//
// The other waves only take groups whose longest chain is at most split
// blocks (group index >= q[2], set by the sort's queue_header): long groups all go
// longest-first to the one raised-priority wave per SIMD, so the batch ends on
// short groups instead of on a medium one pulled late from the short end.
//
// q: [0] front ticket, [1] back ticket, [2] first short group, [3] unused,
//    [4, 4 + kSimdKeys) per-SIMD arrivals, then ngroups claim flags; zeroed
//    before the launch.
constexpr uint32_t kSimdKeys = 8 * 8 * 2 * 16 * 4;  // xcc, se, sh, cu, simd
constexpr uint32_t kQueueHeader = 8;  // tickets, first short group, pad, work (u64), pad

// Values are staged through a pipelined wave-private LDS ring of
// value-relative chunks (sha1_blocks_ring_vc, kQueueRing = 3 slots of 4 KiB:
// two blocks of DMA lookahead; 3 waves per SIMD fit).  The other rings and the
// register-prefetch forms of rounds 1-2 lost their A/Bs.
constexpr int kQueueRing = 3;
__global__ __launch_bounds__(64, kQueueRing) void k_leaf_queue(const uint8_t* __restrict__ base,
                                                       const uint64_t* __restrict__ off,
                                                       const uint64_t* __restrict__ len,
                                                       const uint32_t* __restrict__ perm, uint64_t n,
                                                       uint32_t ngroups, uint32_t simds, uint32_t* __restrict__ q,
                                                       uint8_t* __restrict__ nodes, Gate gate) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[4096 * kQueueRing];
    if (!gate.open()) return;
    const ClockProbe clk;
    const int lane = threadIdx.x;
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint32_t key = ((((xcc & 7) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15)) * 4 +
                         ((hw >> 4) & 3);
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(q + kQueueHeader + key, 1u);
    slot = __builtin_amdgcn_readfirstlane(slot);
    const bool front = slot == 0;
    if (front) __builtin_amdgcn_s_setprio(3);
    // queue_header's results: the first group short enough for the
    // non-priority waves, and the batch's work; a throughput-bound batch (work
    // at least twice what the longest chain keeps every SIMD busy for) lets
    // every wave take any group
    const uint64_t work = reinterpret_cast<const unsigned long long*>(q)[2];
    const uint64_t longest = compressions(len[perm[0]]);
    const uint32_t first_short = __builtin_amdgcn_readfirstlane(
        work >= 2ull * simds * longest ? 0u : min(q[2], ngroups));
    uint32_t* claimed = q + kQueueHeader + kSimdKeys;
#ifdef NKV_DIAG
    uint64_t d_t0 = __builtin_amdgcn_s_memrealtime(), d_c0 = __builtin_amdgcn_s_memtime(), d_first = 0;
    uint64_t d_groups = 0, d_blocks = 0;
#endif
    while (true) {
        uint32_t g = 0xFFFFFFFFu;
        if (lane == 0) {
            const uint32_t t = atomicAdd(q + (front ? 0 : 1), 1u);
            if (t < ngroups) {
                const uint32_t c = front ? t : ngroups - 1 - t;
                if ((front || c >= first_short) && atomicExch(claimed + c, 1u) == 0u) g = c;
            }
        }
        g = __builtin_amdgcn_readfirstlane(g);
        if (g == 0xFFFFFFFFu) break;
        const uint64_t i = uint64_t(g) * 64 + lane;
        const uint64_t leaf = i < n ? perm[i] : 0;
        const uint64_t vo = i < n ? off[leaf] : kDone;
        const bool live = vo != kDone;  // kDone: hashed by k_leaf_records
        const uint8_t* p = live ? base + vo : base;
        const uint64_t ln = live ? len[leaf] : 0;
        uint32_t h[5];
        sha1_init(h);
        sha1_blocks_ring_vc<kQueueRing>(smem, p, uint32_t(ln >> 6), h);
        if (live) {
            sha1_tail<false>(p, ln, h);
            store_digest(nodes, leaf, h);
        }
#ifdef NKV_DIAG
        d_blocks += wave_max_u32(i < n ? uint32_t(len[perm[i]] >> 6) : 0u);
        if (d_groups++ == 0) d_first = __builtin_amdgcn_s_memrealtime();
#endif
    }
    clk.end();
#ifdef NKV_DIAG
    if (g_diag && lane == 0) {
        unsigned long long* d = g_diag + size_t(blockIdx.x) * 8;
        d[0] = d_t0;
        d[1] = __builtin_amdgcn_s_memrealtime();
        d[2] = d_c0;
        d[3] = __builtin_amdgcn_s_memtime();
        d[4] = (uint64_t(slot) << 32) | key;
        d[5] = d_groups;
        d[6] = d_blocks;
        d[7] = d_first;
    }
#endif
}

// K2: a B-node slab of level j0 (already in nodes) reduced up to
// min(j0 + log2 B, top) in LDS, one workgroup of B threads per slab: 8 levels
// per launch with B = 256, 10 with B = 1024 (the narrow levels are a chain of
// one compression per level, so fewer launches is a shorter tree).
template <int B>
__global__ __launch_bounds__(B) void k_reduce(uint8_t* __restrict__ nodes, uint64_t n, int j0, int jmax, Gate gate) {
    __shared__ uint32_t lds[5][B];
    if (!gate.open()) return;
    const uint64_t lo = uint64_t(blockIdx.x) * B;
    const uint64_t cnt = lvl_count(n, j0);
    const uint64_t idx = lo + threadIdx.x;
    uint32_t h[5] = {0u, 0u, 0u, 0u, 0u};
    if (idx < cnt) load_digest(nodes, lvl_start(n, j0) + idx, h);
#pragma unroll
    for (int k = 0; k < 5; ++k) lds[k][threadIdx.x] = h[k];
    subtree_reduce<B>(lds, n, j0, jmax, lo, nodes);
}

// K2w: the wide bottom levels at full lane use.  A wavefront takes 256 nodes
// of level j0: their 128 parents (two per lane), then those parents' 64
// parents (one per lane) when jmax >= j0 + 2.  A k_reduce slab runs 8 levels
// but keeps at most half a wave busy past its first two, while the two bottom
// levels hold three quarters of all parents: 3 wave-compressions per 256 nodes
// here against 9 there.
__global__ __launch_bounds__(kBlock) void k_reduce2(uint8_t* __restrict__ nodes, uint64_t n, int j0, int jmax,
                                                     Gate gate) {
    if (!gate.open()) return;
    const int lane = threadIdx.x & 63;
    const uint64_t w = uint64_t(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t n0 = lvl_count(n, j0), s0 = lvl_start(n, j0);
    const uint64_t n1 = ((n0 - 1) >> 1) + 1, s1 = s0 + n0;
    uint32_t hp[2][5];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int k = 0; k < 5; ++k) hp[p][k] = 0u;
        const uint64_t i1 = 128 * w + uint64_t(lane) + 64 * p;
        if (i1 < n1) {
            const bool lone = 2 * i1 + 1 >= n0;
            uint32_t l[5], r[5] = {0u, 0u, 0u, 0u, 0u};
            load_digest(nodes, s0 + 2 * i1, l);
            if (!lone) load_digest(nodes, s0 + 2 * i1 + 1, r);
            sha1_parent(l, r, lone, hp[p]);
            store_digest(nodes, s1 + i1, hp[p]);
        }
    }
    if (jmax < j0 + 2) return;
    const uint64_t n2 = ((n1 - 1) >> 1) + 1, s2 = s1 + n1;
    const uint64_t i2 = 64 * w + uint64_t(lane);
    // children 2 lane, 2 lane + 1 of this wave's 128: pass 0 for lane < 32
    const int src = (2 * lane) & 63;
    uint32_t l[5], r[5], h[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t l0 = uint32_t(__shfl(int(hp[0][k]), src)), l1 = uint32_t(__shfl(int(hp[1][k]), src));
        const uint32_t r0 = uint32_t(__shfl(int(hp[0][k]), src + 1)), r1 = uint32_t(__shfl(int(hp[1][k]), src + 1));
        l[k] = lane < 32 ? l0 : l1;
        r[k] = lane < 32 ? r0 : r1;
    }
    if (i2 < n2) {
        const bool lone = 2 * i2 + 1 >= n1;
        sha1_parent(l, r, lone, h);
        store_digest(nodes, s2 + i2, h);
    }
}

// K2x: the bottom twelve levels in one launch.  A workgroup of 1024 threads
// (16 waves) takes 4096 nodes of level j0: each wave builds the two levels
// above its 256 nodes at full lane use exactly as k_reduce2 does (128 parents,
// two per lane, then their 64 parents by shuffles), the workgroup's 1024
// level-(j0 + 2) nodes go to LDS, and subtree_reduce<1024> builds ten more
// levels: jmax = min(j0 + 12, top).  Replaces k_reduce2 + one 1024-slab launch
// (the slab part is a chain of one compression per level either way).
__global__ __launch_bounds__(1024) void k_reduce_wide(uint8_t* __restrict__ nodes, uint64_t n, int j0, int jmax,
                                                      Gate gate) {
    __shared__ uint32_t lds[5][1024];
    if (!gate.open()) return;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const uint64_t w = uint64_t(blockIdx.x) * 16 + uint64_t(wv);
    const uint64_t n0 = lvl_count(n, j0), s0 = lvl_start(n, j0);
    const uint64_t n1 = ((n0 - 1) >> 1) + 1, s1 = s0 + n0;
    uint32_t hp[2][5];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int k = 0; k < 5; ++k) hp[p][k] = 0u;
        const uint64_t i1 = 128 * w + uint64_t(lane) + 64 * p;
        if (i1 < n1) {
            const bool lone = 2 * i1 + 1 >= n0;
            uint32_t l[5], r[5] = {0u, 0u, 0u, 0u, 0u};
            load_digest(nodes, s0 + 2 * i1, l);
            if (!lone) load_digest(nodes, s0 + 2 * i1 + 1, r);
            sha1_parent(l, r, lone, hp[p]);
            store_digest(nodes, s1 + i1, hp[p]);
        }
    }
    const uint64_t n2 = ((n1 - 1) >> 1) + 1, s2 = s1 + n1;
    const uint64_t i2 = 64 * w + uint64_t(lane);
    const int src = (2 * lane) & 63;
    uint32_t l[5], r[5], h[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t l0 = uint32_t(__shfl(int(hp[0][k]), src)), l1 = uint32_t(__shfl(int(hp[1][k]), src));
        const uint32_t r0 = uint32_t(__shfl(int(hp[0][k]), src + 1)), r1 = uint32_t(__shfl(int(hp[1][k]), src + 1));
        l[k] = lane < 32 ? l0 : l1;
        r[k] = lane < 32 ? r0 : r1;
    }
    if (i2 < n2) {
        const bool lone = 2 * i2 + 1 >= n1;
        sha1_parent(l, r, lone, h);
        store_digest(nodes, s2 + i2, h);
    }
    // level j0 + 2 of this workgroup's 4096 nodes: 1024 nodes, node 64 wv + lane
#pragma unroll
    for (int k = 0; k < 5; ++k) lds[k][threadIdx.x] = h[k];
    subtree_reduce<1024>(lds, n, j0 + 2, jmax, uint64_t(blockIdx.x) * 1024, nodes);
}

// ---------------------------------------------------------------------------
// Length bucketing for ragged values: one lane per value means a wavefront
// runs for its longest value, so values are ordered by compression count,
// longest first (longest-processing-time order for the dispatcher), and the
// leaf kernel reads them through the permutation.  A counting sort over 640
// buckets (exact below 256 compressions, 16 buckets per octave above, so a
// bucket spans at most 1/16 of its length) in two gated kernels (below).
// Order inside a bucket is arbitrary (digests are written by leaf index, so
// results do not depend on it).
__device__ __forceinline__ uint32_t len_bucket_desc(uint64_t len) {
    const uint64_t c64 = compressions(len);
    const uint32_t c = c64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(c64);
    uint32_t k = c;
    if (c >= 256) {
        const uint32_t e = 31u - uint32_t(__clz(c));
        k = 256u + (e - 8u) * 16u + ((c >> (e - 4u)) & 15u);
    }
    return kLenBuckets - 1u - k;
}

// Smallest compression count of a bucket (exact below 256 compressions).
__device__ __forceinline__ uint64_t bucket_compressions(uint32_t bucket) {
    const uint32_t k = kLenBuckets - 1u - bucket;
    if (k < 256u) return k;
    const uint32_t e = 8u + (k - 256u) / 16u;
    return uint64_t(16u + (k - 256u) % 16u) << (e - 4u);
}

// The work queue's header from the sorted order's bucket starts (start[b] =
// first sorted position of bucket b, total = values sorted), by one workgroup,
// so no separate launch sets the queue up: tickets 0; q[2] = the first group
// (64 sorted values, longest first) whose first value is short, i.e. has at
// most split + 1 compressions (0xFFFFFFFF if none); q[4..5] = the batch's work,
// the sum over groups of their first value's compressions (each bucket's
// smallest count: exact below 256 compressions, within 1/16 above -- it only
// feeds k_leaf_queue's throughput-bound test).
__device__ void queue_header(const uint32_t* start, uint32_t total, const QueueInit& qi) {
    uint32_t first = 0xFFFFFFFFu, none_hi = 0u, none_fl = 0u;
    unsigned long long work = 0;
    for (uint32_t b = threadIdx.x; b < kLenBuckets; b += kBlock) {
        const uint64_t s0 = start[b], s1 = b + 1u < kLenBuckets ? start[b + 1] : total;
        const uint64_t comp = bucket_compressions(b);
        work += (((s1 + 63) >> 6) - ((s0 + 63) >> 6)) * comp;  // groups whose first value is in the bucket
        if (s1 > s0 && comp <= uint64_t(qi.split) + 1u) first = min(first, uint32_t(s0));
    }
    block_fold(first, none_hi, none_fl, work);
    if (threadIdx.x == 0) {
        uint32_t* q = qi.q;
        q[0] = 0u;
        q[1] = 0u;
        q[2] = first == 0xFFFFFFFFu ? first : uint32_t((uint64_t(first) + 63) >> 6);
        q[3] = 0u;
        reinterpret_cast<unsigned long long*>(q)[2] = work;
        q[6] = 0u;
        q[7] = 0u;
    }
}

// Two-launch form: k_len_hist_alloc reserves each (bucket, tile) run inside
// its bucket with one device atomic per nonzero bucket (bucket totals at the
// head of the scratch), and k_len_scatter_alloc scans the 640 totals itself,
// so the three column-scan launches go away.  Runs of one bucket land in the
// order the tiles' atomics arrive (order inside a bucket is free).  The last
// workgroup of the scatter (a ticket after every workgroup has read the
// totals) restores the totals to zero for the next sort.
constexpr uint32_t kSortHead = 1024;  // [0, 640) bucket totals, [640] ticket
__global__ __launch_bounds__(kBlock) void k_len_hist_alloc(const uint64_t* __restrict__ len, uint64_t n,
                                                            uint32_t* __restrict__ scratch, uint32_t tiles,
                                                            Gate gate, QueueInit qi, CopyWords cw) {
    __shared__ uint32_t h[kLenBuckets];
    if (blockIdx.x == 0 && threadIdx.x < cw.n) cw.dst[threadIdx.x] = cw.src[threadIdx.x];
    if (!gate.open()) return;
    for (uint32_t i = threadIdx.x; i < kLenBuckets; i += kBlock) h[i] = 0u;
    if (qi.q)  // the work queue's per-SIMD arrivals and claim flags (its header: k_len_scatter_alloc)
        for (uint64_t i = kQueueHeader + uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < qi.nq;
             i += uint64_t(tiles) * kBlock)
            qi.q[i] = 0u;
    __syncthreads();
    const uint64_t base = uint64_t(blockIdx.x) * kSortTile;
    uint32_t bk[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
        bk[j] = i < n ? len_bucket_desc(len[i]) : kLenBuckets;
    }
#pragma unroll
    for (int j = 0; j < kSortItems; ++j)
        if (bk[j] < kLenBuckets) atomicAdd(&h[bk[j]], 1u);
    __syncthreads();
    uint32_t* hist = scratch + kSortHead;
    for (uint32_t i = threadIdx.x; i < kLenBuckets; i += kBlock) {
        const uint32_t c = h[i];
        hist[uint64_t(i) * tiles + blockIdx.x] = c ? atomicAdd(scratch + i, c) : 0u;
    }
}

__global__ __launch_bounds__(kBlock) void k_len_scatter_alloc(const uint64_t* __restrict__ len, uint64_t n,
                                                               uint32_t* __restrict__ scratch, uint32_t tiles,
                                                               uint32_t* __restrict__ perm, Gate gate,
                                                               QueueInit qi) {
    __shared__ uint32_t cur[kLenBuckets];
    __shared__ uint32_t last, total;
    if (!gate.open()) return;
    if (threadIdx.x < 64) {  // exclusive scan of the bucket totals, 64 at a time
        const int lane = threadIdx.x;
        uint32_t carry = 0u;
        for (uint32_t c0 = 0; c0 < kLenBuckets; c0 += 64) {
            const uint32_t v = scratch[c0 + lane];
            uint32_t x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = uint32_t(__shfl_up(int(x), o));
                if (lane >= o) x += y;
            }
            cur[c0 + lane] = carry + x - v;
            carry += uint32_t(__shfl(int(x), 63));
        }
        if (lane == 0) total = carry;
    }
    __syncthreads();
    if (qi.q && blockIdx.x == 0) queue_header(cur, total, qi);
    const uint32_t* hist = scratch + kSortHead;
    for (uint32_t i = threadIdx.x; i < kLenBuckets; i += kBlock) cur[i] += hist[uint64_t(i) * tiles + blockIdx.x];
    __syncthreads();  // every read of the totals is done
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(scratch + kLenBuckets, 1u) == tiles - 1u ? 1u : 0u;
    }
    __syncthreads();
    if (last) {  // every workgroup has read the totals: restore them for the next sort
        for (uint32_t i = threadIdx.x; i < kLenBuckets; i += kBlock) scratch[i] = 0u;
        if (threadIdx.x == 0) scratch[kLenBuckets] = 0u;
    }
    const uint64_t base = uint64_t(blockIdx.x) * kSortTile;
    uint32_t bk[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        const uint64_t i = base + uint64_t(j) * kBlock + threadIdx.x;
        bk[j] = i < n ? len_bucket_desc(len[i]) : kLenBuckets;
    }
#pragma unroll
    for (int j = 0; j < kSortItems; ++j)
        if (bk[j] < kLenBuckets)
            perm[atomicAdd(&cur[bk[j]], 1u)] = uint32_t(base + uint64_t(j) * kBlock + threadIdx.x);
}

// ---------------------------------------------------------------------------
// K3: BFS image.  Levels are written top-down; level L contributes 21 bytes
// per node (0x00 flag + digest) plus one 0x01 byte for the pad of an odd
// level below the top.  One workgroup builds one 4 KiB segment of the image
// in LDS: for every level that overlaps the segment, each thread takes nodes
// of it (one 64-bit division by 21 per level, not per byte) and writes their
// 21-byte records, clipped to the segment, as byte stores into LDS; then each
// thread stores 16 aligned bytes of the segment.  A record that straddles two
// segments is written, clipped, by both workgroups.
constexpr uint32_t kBfsSeg = kBlock * 16;
__global__ __launch_bounds__(kBlock) void k_bfs_image(const uint8_t* __restrict__ nodes,
                                                       BfsLayout lay, uint8_t* __restrict__ img) {
    __shared__ __attribute__((aligned(16))) uint8_t seg[kBfsSeg];
    const uint64_t s0 = uint64_t(blockIdx.x) * kBfsSeg;
    if (s0 >= lay.total) return;
    const uint64_t s1 = min(s0 + kBfsSeg, lay.total);
    for (int L = 0; L < lay.nlev; ++L) {
        const uint64_t A = lay.img_start[L];
        const uint64_t E = A + 21 * lay.count[L];           // end of the node records
        const uint64_t Z = L + 1 < lay.nlev ? lay.img_start[L + 1] : lay.total;  // E or E + 1 (pad)
        if (Z <= s0 || A >= s1) continue;
        if (E < Z && E >= s0 && E < s1 && threadIdx.x == 0)
            seg[E - s0] = 0x01u;  // MERKLE_NODE_EMPTY pad (merklenode.go:11, merkletree.go:32-34)
        if (E <= s0) continue;
        const uint64_t k0 = s0 > A ? (s0 - A) / 21 : 0;
        const uint64_t k1 = (min(s1, E) - 1 - A) / 21;  // last node with a byte in the segment
        for (uint64_t k = k0 + threadIdx.x; k <= k1; k += kBlock) {
            const uint32_t* d = reinterpret_cast<const uint32_t*>(nodes + 20 * (lay.node_start[L] + k));
            uint32_t w[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) w[i] = d[i];
            const int64_t pos = int64_t(A + 21 * k) - int64_t(s0);  // record start in the segment
            if (pos >= 0 && pos + 21 <= int64_t(kBfsSeg)) {
                uint8_t* o = seg + pos;
                o[0] = 0u;
#pragma unroll
                for (int j = 0; j < 20; ++j) o[1 + j] = uint8_t(w[j >> 2] >> (8 * (j & 3)));
            } else {
#pragma unroll
                for (int j = 0; j < 21; ++j) {
                    const int64_t q = pos + j;
                    if (q >= 0 && q < int64_t(kBfsSeg))
                        seg[q] = j == 0 ? 0u : uint8_t(w[(j - 1) >> 2] >> (8 * ((j - 1) & 3)));
                }
            }
        }
    }
    __syncthreads();
    const uint64_t p0 = s0 + 16 * threadIdx.x;
    if (p0 + 16 <= s1) {
        *reinterpret_cast<uint4*>(img + p0) = *reinterpret_cast<const uint4*>(seg + 16 * threadIdx.x);
    } else {
        for (uint64_t p = p0; p < s1; ++p) img[p] = seg[p - s0];
    }
}

// ---------------------------------------------------------------------------
// K0: locate values inside a serialized Data-table stream.
// Record layout (record.go:191-199, little endian): Crc u32 @0, Timestamp i64
// @4, Status u8 @12, TypeInfo u8 @13, KeySize u64 @14, ValueSize u64 @22,
// Key @30, Value @30+KeySize.  rec_off[i] = start of record i.

// One record per thread; each workgroup leaves its range and error flag in
// part[3 b .. 3 b + 2] (plain stores: no same-address atomics across 4096
// blocks), and k_locate_fold combines them in a one-workgroup launch.
__global__ __launch_bounds__(kBlock) void k_locate(const uint8_t* __restrict__ stream,
                                                    uint64_t stream_len,
                                                    const uint64_t* __restrict__ rec_off, uint64_t n,
                                                    uint64_t* __restrict__ voff,
                                                    uint64_t* __restrict__ vlen, uint32_t* __restrict__ part) {
    const uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    uint32_t lo = 0xFFFFFFFFu, hi = 0u, bad = 0u;
    unsigned long long none = 0;
    if (i < n) {
        const uint64_t r = rec_off[i];
        uint64_t o = 0, l = 0;
        if (header_in(r, stream_len)) {
            uint64_t ks, vs;
            ld_header_sizes(stream + r, ks, vs);
            o = r + 30 + ks;
            l = vs;
            if (ks > stream_len || vs > stream_len || o + l > stream_len) {
                bad = 1u;
                o = 0;
                l = 0;
            }
        } else {
            bad = 1u;
        }
        voff[i] = o;
        vlen[i] = l;
        const uint64_t b = l >> 6;
        lo = hi = b > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(b);
    }
    block_fold(lo, hi, bad, none);
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x] = lo;
        part[3 * blockIdx.x + 1] = hi;
        part[3 * blockIdx.x + 2] = bad;
    }
}

__global__ __launch_bounds__(kBlock) void k_locate_fold(const uint32_t* __restrict__ part, uint32_t nb,
                                                         unsigned int* __restrict__ err,
                                                         unsigned int* __restrict__ range) {
    uint32_t lo = 0xFFFFFFFFu, hi = 0u, bad = 0u;
    unsigned long long none = 0;
    // coalesced, independent loads over the flat triples (one per workgroup)
    const uint32_t words = 3u * nb;
#pragma unroll 8
    for (uint32_t x = threadIdx.x; x < words; x += kBlock) {
        const uint32_t v = part[x];
        const uint32_t kind = x % 3u;
        if (kind == 0u) lo = min(lo, v);
        else if (kind == 1u) hi = max(hi, v);
        else bad |= v;
    }
    block_fold(lo, hi, bad, none);
    if (threadIdx.x == 0) {
        if (err) *err = bad;
        if (range) {
            range[0] = lo;
            range[1] = hi;
        }
    }
}

// K1r: the records form's leaf pass in one launch (nkv_tree_from_records*):
// k_locate's header parse (value = rec + 30 + KeySize, ValueSize bytes;
// record.go:191-199) and k_leaf's hash of the value, so the header line is
// read once and no separate locate pass runs.  policy 0 hashes every wave in
// input order; 1 (auto) hashes the waves whose full-block counts are narrow
// by the plan rule (max <= min + max(1, min / 16), Gate) and defers the others
// to the length-sorted work queue; 2 defers all.  A hashed value's voff is
// set to kDone (vlen 0): the sorted pass skips it.  A deferred value keeps its
// voff / vlen.  Each workgroup leaves (0, deferred ? ~0 : 0, bad) in part,
// which k_locate_fold turns into err and a range whose wide Gate opens the
// sorted pass only when something was deferred.  A header outside the
// stream flags bad and hashes the empty value (as k_locate).
#if NKV_EXP_REC == 1
constexpr int kRecordsWaves = 4;  // experiment: a fourth segment set
#else
constexpr int kRecordsWaves = 5;  // narrow waves of line-aligned records take whole lines: ~86 VGPRs
#endif
__global__ __launch_bounds__(kBlock, kRecordsWaves) void k_leaf_records(
    const uint8_t* __restrict__ stream, uint64_t stream_len, const uint64_t* __restrict__ rec_off, uint64_t n,
    int policy, uint64_t* __restrict__ voff, uint64_t* __restrict__ vlen, uint8_t* __restrict__ nodes,
    uint32_t* __restrict__ part, uint32_t* __restrict__ flags, uint32_t* __restrict__ flags_next) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kBlock * 80];
    if (flags) pass_flags_reset(flags_next);
    const ClockProbe clk;
    const uint64_t t = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    const bool live = t < n;
    uint64_t o = 0, l = 0;
    uint32_t bad = 0u;
    if (live) {
        const uint64_t r = rec_off[t];
        if (header_in(r, stream_len)) {
            uint64_t ks, vs;
            ld_header_sizes(stream + r, ks, vs);
            o = r + 30 + ks;
            l = vs;
            if (ks > stream_len || vs > stream_len || o + l > stream_len) {
                bad = 1u;
                o = 0;
                l = 0;
            }
        } else {
            bad = 1u;
        }
        voff[t] = o;
        vlen[t] = l;
    }
    const uint64_t bl = l >> 6;
    const uint32_t b32 = bl > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(bl);
    const uint32_t wlo = wave_min_u32(live ? b32 : 0xFFFFFFFFu);
    const uint32_t whi = wave_max_u32(live ? b32 : 0u);
    const bool any = __any(live);
    const bool hash = any && (policy == 0 || (policy == 1 && whi <= wlo + max(1u, wlo / 16u)));
    // wave-level partials, so no per-lane flag stays live through the stage
    const bool wbad = __any(bad != 0u);
    const bool wdefer = any && !hash;
    if (hash) {
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        uint32_t h[5];
        sha1_init(h);
        sha1_blocks_any<true>(smem + 5120 * wave, stream + o, live, live ? b32 : 0u, h);
        // reload the value's place (written above by this lane) rather than
        // keeping it, or its addresses, live through the stage
        asm volatile("" ::: "memory");
        uint32_t tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const uint64_t u = uint64_t(blockIdx.x) * kBlock + tid;
        if (u < n) {
            o = voff[u];
            l = vlen[u];
            sha1_tail<false>(stream + o, l, h);
            store_digest(nodes, u, h);
            voff[u] = kDone;
            vlen[u] = 0;
        }
    }
    // one partial per workgroup, folded through the (now idle) stage LDS: a
    // block_fold of its own would cost LDS, i.e. a workgroup per CU
    const int wv = threadIdx.x >> 6;
    uint32_t* wf = reinterpret_cast<uint32_t*>(smem);
    __syncthreads();  // every wave is done with its stage
    if ((threadIdx.x & 63) == 0) wf[wv] = (wdefer ? 2u : 0u) | (wbad ? 1u : 0u);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t f = 0u;
#pragma unroll
        for (int k = 0; k < kBlock / 64; ++k) f |= wf[k];
        if (flags) {  // the pass flags (no fold launch)
            if (f & 2u) pass_flag_raise(flags + 1, 0xFFFFFFFFu);
            if (f & 1u) pass_flag_raise(flags + 2, 1u);
        } else {
            part[3 * blockIdx.x] = 0u;
            part[3 * blockIdx.x + 1] = (f & 2u) ? 0xFFFFFFFFu : 0u;
            part[3 * blockIdx.x + 2] = f & 1u;
        }
    }
    clk.end();
}

// Range of full-block counts of a batch: out[0] = min, out[1] = max.  Lets
// the leaf level choose input order (narrow range: no sort) or the
// length-sorted work queue, on the device (Gate).
__global__ __launch_bounds__(kBlock) void k_len_range(const uint64_t* __restrict__ len, uint64_t n,
                                                       uint32_t* __restrict__ part, unsigned int* __restrict__ out,
                                                       unsigned int* __restrict__ ticket) {
    // eight values per thread, loads first; one (lo, hi, 0) partial per
    // workgroup, and the last workgroup to finish (a ticket) folds them into
    // out (no same-address min/max atomics: a grid fold over 256 workgroups
    // serialised them for 12.6 us at 453 K values; and no fold launch)
    uint32_t lo = 0xFFFFFFFFu, hi = 0u, none = 0u;
    unsigned long long zero = 0;
    const uint64_t base = uint64_t(blockIdx.x) * (kBlock * 8) + threadIdx.x;
    uint64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const uint64_t i = base + uint64_t(u) * kBlock;
        v[u] = i < n ? len[i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        if (base + uint64_t(u) * kBlock >= n) continue;
        const uint64_t b = v[u] >> 6;
        const uint32_t bb = b > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(b);
        lo = min(lo, bb);
        hi = max(hi, bb);
    }
    block_fold(lo, hi, none, zero);
    __shared__ uint32_t is_last;
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x] = lo;
        part[3 * blockIdx.x + 1] = hi;
        part[3 * blockIdx.x + 2] = 0u;
        __threadfence();
        is_last = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!is_last) return;
    __threadfence();
    lo = 0xFFFFFFFFu;
    hi = 0u;
    for (uint32_t b = threadIdx.x; b < gridDim.x; b += kBlock) {
        lo = min(lo, __atomic_load_n(part + 3 * b, __ATOMIC_RELAXED));
        hi = max(hi, __atomic_load_n(part + 3 * b + 1, __ATOMIC_RELAXED));
    }
    block_fold(lo, hi, none, zero);
    if (threadIdx.x == 0) {
        out[0] = lo;
        out[1] = hi;
        atomicExch(ticket, 0u);  // the next launch counts from 0
    }
}

hipError_t launch_len_range(const uint64_t* len, uint64_t n, unsigned int* out, uint32_t* part, unsigned int* ticket,
                            hipStream_t s) {
    const unsigned nb = unsigned((n + kBlock * 8 - 1) / (kBlock * 8));
    hipLaunchKernelGGL(k_len_range, dim3(nb), dim3(kBlock), 0, s, len, n, part, out, ticket);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// synthetic input: byte j = byte (j % 8) of splitmix64(seed, j / 8), LE.
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void k_fill(uint8_t* __restrict__ buf, uint64_t nbytes,
                                                  uint64_t seed) {
    const uint64_t stride = uint64_t(gridDim.x) * kBlock;
    for (uint64_t t = uint64_t(blockIdx.x) * kBlock + threadIdx.x; 16 * t < nbytes; t += stride) {
        const uint64_t a = splitmix64_at(seed, 2 * t), b = splitmix64_at(seed, 2 * t + 1);
        if (16 * t + 16 <= nbytes) {
            *reinterpret_cast<uint4*>(buf + 16 * t) =
                make_uint4(uint32_t(a), uint32_t(a >> 32), uint32_t(b), uint32_t(b >> 32));
        } else {
            for (uint64_t j = 16 * t; j < nbytes; ++j) {
                const uint64_t v = (j - 16 * t) < 8 ? a : b;
                buf[j] = uint8_t(v >> (8 * (j & 7)));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Ks: a whole small tree in ONE launch -- the sizes the reference engine runs at
// by default (coreconf.go:33-34: a flush of MEMTABLE_CAPACITY = 10 records;
// :39: a compaction of lsm_run_max = 4 such runs), where a launch per level
// and copies per buffer would cost more than the hashing.
//
// Input: n (offset, length) u64 pairs at desc and the values at vals + offset
// (16-byte aligned).  The host packs both into host-coherent pinned memory that
// the kernel reads across PCIe (no DMA), or copies them to HBM first
// (NKV_OPT_SMALL_PATH); values already in a host-coherent pinned arena block
// (the deferred-NewLeaf arena, nkv_host_alloc) are read where they lie.  One lane per leaf and one
// 256-lane workgroup per 256 leaves, so each wave runs alone on its SIMD (a
// leaf's SHA-1 is a serial chain: DESIGN.md section 4, lone-wave cadence); the
// last workgroup to finish (a ticket) takes every leaf digest, builds all levels
// (merkletree.go:31-64) and the Serialize image (merkletree.go:67-92,
// merklenode.go:37-63) in LDS, and stores nodes (level-major, 20 B each) at out
// and the image at out + img_at with 16-byte stores.  LDS: every node (at most
// 2 x 1024 - 1) plus one 16 KiB image segment, under the 64 KiB a workgroup
// gets without opting in.

constexpr uint32_t kSmallBlock = 256;

// SHA-1 of p[0, len), p 16-byte aligned, one block of register lookahead,
// with every lane of the wave issuing every compression.  A wave runs its VALU work up to 35 % slower on some CUs when fewer than ~48 of
// its lanes are active than with all of them (one clock, same instructions:
// tools/svc_shape.hip, profiles/r06_svc_shape_lanes.txt -- 10 active lanes take
// 11.2-15.1 us by CU for what 48 or 64 lanes do in 11.0 us on every CU), and a
// small tree's waves have few values.  So the full-block loop runs to the
// wave's largest block count (a lane past its own blocks compresses its stale
// block into a copy it drops) and the padding blocks run in every lane; a lane
// with no value (len 0) hashes the empty value, which its caller drops.  The
// caller calls it with every lane of the wave active.
__device__ __forceinline__ void sha1_value_all_lanes(const uint8_t* p, uint32_t len, uint32_t h[5]) {
    sha1_init(h);
    const uint32_t nfull = len >> 6;
    uint32_t most = nfull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) most = max(most, uint32_t(__shfl_xor(int(most), o)));
    most = uint32_t(__builtin_amdgcn_readfirstlane(int(most)));  // wave-uniform trip count
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        cur[k] = nfull ? q[k] : make_uint4(0u, 0u, 0u, 0u);
        nxt[k] = make_uint4(0u, 0u, 0u, 0u);
    }
    for (uint32_t b = 0; b < most; ++b) {
        if (b + 1 < nfull) {
#pragma unroll
            for (int k = 0; k < 4; ++k) nxt[k] = q[4 * (b + 1) + k];
        }
        uint32_t w[16], t[5];
        be16_from_raw(cur, w);
#pragma unroll
        for (int i = 0; i < 5; ++i) t[i] = h[i];
        sha1_compress(t, w);
        const bool mine = b < nfull;
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] = mine ? t[i] : h[i];
#pragma unroll
        for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
    }
    sha1_tail<true>(p, len, h);
}

// bytes [0, bytes) of LDS src to dst (16-byte aligned both), 16 per store;
// B = the workgroup's threads
template <uint32_t B>
__device__ __forceinline__ void small_copy_out(const uint8_t* src, uint8_t* dst, uint32_t bytes) {
    const uint32_t whole = bytes & ~15u;
    for (uint32_t b = 16 * threadIdx.x; b < whole; b += 16 * B)
        *reinterpret_cast<uint4*>(dst + b) = *reinterpret_cast<const uint4*>(src + b);
    for (uint32_t b = whole + threadIdx.x; b < bytes; b += B) dst[b] = src[b];
}

__device__ __forceinline__ uint32_t small_count(uint32_t n, int L) { return L == 0 ? n : ((n - 1) >> L) + 1; }

// bytes [0, bytes) of src (16-byte aligned, host or device memory) into LDS
// dst: every thread's loads are issued before any store, so an input of up to
// 16 KiB crosses PCIe in one round trip
template <uint32_t B>
__device__ __forceinline__ void small_stage_in(const uint8_t* src, uint8_t* dst, uint32_t bytes) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    const uint32_t nq = (bytes + 15u) >> 4;
    for (uint32_t c0 = 0; c0 < nq; c0 += 4 * B) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = c0 + threadIdx.x + k * B;
            v[k] = c < nq ? s4[c] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = c0 + threadIdx.x + k * B;
            if (c < nq) d4[c] = v[k];
        }
    }
}

// Every level above the leaf digests in sm (at least one; a lone last node is
// hashed alone, its sibling being the empty pad: merkletree.go:31-64), the
// nodes stored level-major at out, then the Serialize image at out + img_at,
// top level first: 0x00 + digest per node, one 0x01 after each odd level below
// the top (merklenode.go:37-63, MERKLE_NODE_EMPTY :11), built kSmallSeg bytes
// at a time in seg from whole node records clipped to the segment (as
// k_bfs_image does); img_at 0: no image.  Starts at a workgroup barrier.
template <uint32_t B>
__device__ __forceinline__ void small_levels_and_image(uint8_t* sm, uint8_t* seg, uint32_t n, uint8_t* out,
                                                       uint32_t img_at, uint64_t* trace = nullptr) {
    const uint32_t tid = threadIdx.x;
    // diagnostics (the service's traced requests): (s_memrealtime, s_memtime)
    // into trace[2k], trace[2k + 1] by thread 0
    auto mark = [&](int k) {
        if (trace && tid == 0) {
            __hip_atomic_store(trace + 2 * k, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(trace + 2 * k + 1, __builtin_amdgcn_s_memtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    };
    __syncthreads();
    uint32_t cnt = n, base = 0;
    int lv = 1;
    do {
        const uint32_t pc = (cnt + 1) >> 1;
        // every lane of a wave that has a parent to build takes part (a lane
        // past the level's end rebuilds the last parent and drops it): a wave
        // with few active lanes computes slower on some CUs (sha1_value_all_lanes)
        for (uint32_t j0 = 0; j0 < pc; j0 += B) {
            const uint32_t j = j0 + tid;
            if ((j & ~63u) < pc) {
                const uint32_t jj = min(j, pc - 1u);
                const bool lone = 2 * jj + 1 >= cnt;
                uint32_t l[5], r[5] = {0u, 0u, 0u, 0u, 0u}, o[5];
                load_digest(sm, base + 2 * jj, l);
                if (!lone) load_digest(sm, base + 2 * jj + 1, r);
                sha1_parent(l, r, lone, o);
                if (j < pc) store_digest(sm, base + cnt + j, o);
            }
        }
        __syncthreads();
        base += cnt;
        cnt = pc;
        ++lv;
    } while (cnt > 1);
    NKV_STAMP(3);
    mark(0);
    const uint32_t total = base + 1;
    if (img_at == 0u) {  // the caller asked for no image (the nodes start at out + 0)
        small_copy_out<B>(sm, out, 20u * total);
        return;
    }
    uint32_t img_len = 0;
    for (int L = lv - 1; L >= 0; --L) {
        const uint32_t c = small_count(n, L);
        img_len += 21u * c + ((L < lv - 1 && (c & 1u)) ? 1u : 0u);
    }
    // (seg's staged input was last read before the first level's barrier)
    // The nodes leave with the first image segment, after it is built.
    // Every node record of the image is built by its own thread at once (all
    // levels together): the thread finds its record's level from the top,
    // loads the 20-byte digest as five LDS words and stores the 21 bytes, so
    // no LDS load waits inside a byte loop (per-level, byte-by-byte copying
    // cost 6 us for a 10-leaf tree, more than its four tree levels).
    for (uint32_t s0 = 0; s0 < img_len; s0 += kSmallSeg) {
        const uint32_t s1 = min(s0 + kSmallSeg, img_len);
        for (uint32_t r = tid; r < total; r += B) {
            uint32_t A = 0, before = 0;  // image offset of level L's first record; records above it
            int L = lv - 1;
            uint32_t c = small_count(n, L);
            while (r >= before + c) {
                A += 21u * c + ((L < lv - 1 && (c & 1u)) ? 1u : 0u);
                before += c;
                --L;
                c = small_count(n, L);
            }
            const uint32_t k = r - before;
            uint32_t ns = 0;  // node index of level L's first node (levels stored bottom-up)
            for (int jl = 0; jl < L; ++jl) ns += small_count(n, jl);
            const uint32_t* d = reinterpret_cast<const uint32_t*>(sm + 20u * (ns + k));
            uint32_t w[5];
#pragma unroll
            for (int q = 0; q < 5; ++q) w[q] = d[q];
            const int32_t pos = int32_t(A + 21u * k) - int32_t(s0);
            if (pos >= 0 && pos + 21 <= int32_t(s1 - s0)) {
                seg[pos] = 0u;
#pragma unroll
                for (int b = 0; b < 20; ++b) seg[pos + 1 + b] = uint8_t(w[b >> 2] >> (8 * (b & 3)));
            } else if (pos + 21 > 0 && pos < int32_t(s1 - s0)) {  // a record across a segment edge
#pragma unroll
                for (int b = 0; b < 21; ++b) {
                    const int32_t qb = pos + b;
                    if (qb >= 0 && qb < int32_t(s1 - s0)) seg[qb] = b == 0 ? 0u : uint8_t(w[(b - 1) >> 2] >> (8 * ((b - 1) & 3)));
                }
            }
        }
        // the pads: one 0x01 after each odd level below the top, by thread L
        if (tid + 1 < uint32_t(lv)) {
            const int L = int(tid);
            uint32_t A = 0;
            for (int Lu = lv - 1; Lu > L; --Lu) {
                const uint32_t cu = small_count(n, Lu);
                A += 21u * cu + ((Lu < lv - 1 && (cu & 1u)) ? 1u : 0u);
            }
            const uint32_t c = small_count(n, L);
            const uint32_t E = A + 21u * c;
            if ((c & 1u) && E >= s0 && E < s1) seg[E - s0] = NKV_MERKLE_NODE_EMPTY;
        }
        __syncthreads();
        if (s0 == 0) {
            mark(1);
            small_copy_out<B>(sm, out, 20u * total);
        }
        small_copy_out<B>(seg, out + img_at + s0, s1 - s0);
        if (s1 < img_len) __syncthreads();  // seg is rebuilt for the next segment
    }
}

// seq into the host-coherent completion word once every output byte of the
// workgroup is written at system scope.  One release for the workgroup, not one
// per wave (the guide's producer form: every storing wave waits for its own
// stores, a barrier, then ONE lane's release fence -- a single L2 write-back --
// its wait, and the flag); a fence in every wave cost each wave an L2
// write-back (16 of them in the service's first, 1024-thread form).
__device__ __forceinline__ void small_signal_done(unsigned int* done, uint32_t seq) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's output stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-back before the flag (guide: compiler hazard)
        __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// vbytes: the extent of vals the values lie in.  A one-workgroup launch whose
// descriptors and values fit kSmallSeg bytes stages both into LDS first (one
// PCIe round trip for the whole input instead of one per block of each lane).
// done (nullable, host-coherent): receives seq once every output byte is
// written, so the host can spin on it instead of waiting for the runtime's
// completion signal.
__global__ __launch_bounds__(kSmallBlock) void k_small_tree(const uint64_t* __restrict__ desc,
                                                            const uint8_t* __restrict__ vals, uint32_t vbytes,
                                                            uint32_t n, uint8_t* __restrict__ out, uint32_t img_at,
                                                            uint8_t* __restrict__ scratch,
                                                            unsigned int* __restrict__ ticket,
                                                            unsigned int* __restrict__ done, uint32_t seq) {
    __shared__ __attribute__((aligned(16))) uint8_t sm[20 * (2 * kSmallMaxN - 1) + 12];  // every node
    __shared__ __attribute__((aligned(16))) uint8_t seg[kSmallSeg];  // the staged input, then image segments
    __shared__ uint32_t is_last;
    const uint32_t tid = threadIdx.x;
    const uint32_t i = blockIdx.x * kSmallBlock + tid;
    NKV_STAMP(0);
    // the input may lie in fine-grained device memory the host stored to
    // (NKV_OPT_SERVICE_MAILBOX 0): no stale L2 line of an earlier call's input
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (gridDim.x == 1 && 16u * n + vbytes <= kSmallSeg) {
        small_stage_in<kSmallBlock>(reinterpret_cast<const uint8_t*>(desc), seg, 16u * n);
        small_stage_in<kSmallBlock>(vals, seg + 16u * n, vbytes);
        __syncthreads();
        desc = reinterpret_cast<const uint64_t*>(seg);
        vals = seg + 16u * n;
    }
    NKV_STAMP(1);
    uint32_t h[5] = {0u, 0u, 0u, 0u, 0u};
    if ((i & ~63u) < n) {  // every lane of a wave with a value (sha1_value_all_lanes)
        const bool real = i < n;
        sha1_value_all_lanes(real ? vals + desc[2 * i] : vals, real ? uint32_t(desc[2 * i + 1]) : 0u,
                             h);  // NewLeaf, merklenode.go:27-34
    }
    NKV_STAMP(2);
    if (gridDim.x > 1) {
        if (i < n) store_digest(scratch, i, h);
        __threadfence();
        __syncthreads();
        if (tid == 0) is_last = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
        __syncthreads();
        if (!is_last) return;
        __threadfence();
        if (tid == 0) atomicExch(ticket, 0u);  // the next launch counts from 0
        for (uint32_t j = tid; j < n; j += kSmallBlock) {
            const uint32_t* s = reinterpret_cast<const uint32_t*>(scratch + 20u * j);
            uint32_t* d = reinterpret_cast<uint32_t*>(sm + 20u * j);
#pragma unroll
            for (int k = 0; k < 5; ++k) d[k] = __atomic_load_n(s + k, __ATOMIC_RELAXED);
        }
    } else if (i < n) {
        store_digest(sm, i, h);
    }
    small_levels_and_image<kSmallBlock>(sm, seg, n, out, img_at);
    if (done) small_signal_done(done, seq);
}

// The resident small-tree service (NKV_OPT_SMALL_PATH 3): ONE workgroup of
// kSvcBlock threads stays on the GPU between calls and serves one request of at
// most kSvcMaxN leaves at a time from a mailbox, so a default-size flush pays neither a
// launch nor the runtime's completion path ("The
// small-flush floor").  The request side (rb: doorbell, request line; fixed_in:
// the service's own input buffer) lies in device memory the host stores to
// directly on a large-BAR GPU, else in host-coherent memory with the rest of
// the mailbox (rb == mb; NKV_OPT_SERVICE_MAILBOX); the answer side (mb: served,
// done, refused, stamps) is always host-coherent, where the host spins on it.
// Wave 0 polls the doorbell (relaxed
// system-scope loads, s_sleep between polls); a new seq is acquired at system
// scope, the request (the same descriptors, values and output layout
// k_small_tree takes) is served exactly as k_small_tree serves a one-workgroup
// launch -- leaves one lane each, every level and the image in LDS -- and seq
// goes to mb->done behind every output byte.  Every wave leaves when the
// doorbell reads kSvcExit (nkv_ctx_destroy), after idle_ticks of the 100 MHz
// real-time counter with no request, or between requests once it has lived
// life_ticks (the host relaunches on its next call), so the grid always drains
// and work queued behind it on a shared hardware queue waits a bounded time.
// s_getreg_b32 operands: HW_REG_HW_ID (id 4: wave, SIMD, CU, SH, SE ...) and
// HW_REG_XCC_ID (id 20, bits [3:0]), whole registers
constexpr int kHwRegHwId = 4 | (0 << 6) | (31 << 11);
constexpr int kHwRegXccId = 20 | (0 << 6) | (15 << 11);

template <uint32_t B>
__global__ __launch_bounds__(B) void k_small_service(SmallMailbox* __restrict__ mb, const SmallMailbox* rb,
                                                     const uint8_t* __restrict__ fixed_in, uint64_t idle_ticks,
                                                     uint64_t life_ticks) {
    __shared__ __attribute__((aligned(16))) uint8_t sm[20 * (2 * kSvcMaxN - 1) + 12];
    __shared__ __attribute__((aligned(16))) uint8_t seg[kSmallSeg];
    __shared__ uint32_t cmd;
    __shared__ uint32_t rq[16];  // the request line
    // Control flow stays wave-uniform: the whole of wave 0 polls (every lane
    // the same word, the value made scalar), and every decision after the
    // barrier is on a scalar.  A poll loop run by one LANE with a workgroup
    // barrier after it lets the compiler park that lane while its wave's other
    // lanes go round the outer loop's barrier on their own (the first build
    // served one request and then spun on it).
    const uint32_t tid = threadIdx.x;
    const bool poller = tid < 64;
    uint32_t served =
        __builtin_amdgcn_readfirstlane(__hip_atomic_load(&mb->served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    const uint64_t born = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {  // where this launch landed (nkv_ctx_small_service_state)
        __hip_atomic_store(&mb->hw_id, uint32_t(__builtin_amdgcn_s_getreg(kHwRegHwId)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->xcc_id, uint32_t(__builtin_amdgcn_s_getreg(kHwRegXccId)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    uint64_t seen_rt = 0, seen_mt = 0;  // wave 0: when the latest doorbell was seen (traced requests)
    // (s_memrealtime, s_memtime) of a traced request's phase k into the mailbox
    auto stamp = [&](int k, uint64_t rt, uint64_t mt) {
        __hip_atomic_store(&mb->stamps[2 * k], rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->stamps[2 * k + 1], mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    };
    while (true) {
        if (poller) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t bell;
            while (true) {
                bell = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&rb->doorbell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
                seen_rt = __builtin_amdgcn_s_memrealtime();
                seen_mt = __builtin_amdgcn_s_memtime();
                if (bell != served) break;
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                if (now - t0 > idle_ticks || now - born > life_ticks) {
                    bell = kSvcExit;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the request's bytes
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (tid == 0) cmd = bell;
        }
        __syncthreads();
        const uint32_t seq = __builtin_amdgcn_readfirstlane(cmd);
        if (seq == kSvcExit) break;
        // One PCIe round trip for the request: the request line (16 lanes of
        // wave 0, one dword each) and, speculatively, the first kSvcSpec bytes
        // of the service's input buffer (16 per thread), all in flight at once;
        // a request packed there (inline_in) needs no second trip below 4 KiB.
        const uint4 spec = reinterpret_cast<const uint4*>(fixed_in)[tid];
        if (tid < 16)
            rq[tid] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(&rb->req) + tid, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        // readfirstlane returns an int: widen through uint32_t, or a low word
        // with its top bit set sign-extends into the pointer's high word (the
        // first build of this read faulted on exactly that)
        auto rq32 = [&](int k) { return uint32_t(__builtin_amdgcn_readfirstlane(rq[k])); };
        auto rq64 = [&](int k) { return uint64_t(rq32(k)) | (uint64_t(rq32(k + 1)) << 32); };
        const uint32_t n = rq32(0);
        const uint32_t vbytes = rq32(1);
        const uint32_t img_at = rq32(2);
        const bool traced = rq32(3) != 0u;
        const uint64_t* desc = reinterpret_cast<const uint64_t*>(rq64(4));
        const uint8_t* vals = reinterpret_cast<const uint8_t*>(rq64(6));
        uint8_t* out = reinterpret_cast<uint8_t*>(rq64(8));
        const bool inline_in = rq32(10) != 0u;
        if (traced && tid == 0) stamp(0, seen_rt, seen_mt);
        // the host never rings with other values; a request out of range is
        // refused (flagged, nothing read or written) rather than followed
        const bool sane = n >= 1 && n <= kSvcMaxN && desc && vals && out &&
                          ((reinterpret_cast<uintptr_t>(desc) | reinterpret_cast<uintptr_t>(vals) |
                            reinterpret_cast<uintptr_t>(out) | img_at) & 15u) == 0u;
        if (!sane && tid == 0) __hip_atomic_store(&mb->refused, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (sane) {
            const uint32_t in_bytes = 16u * n + vbytes;
            if (inline_in && in_bytes <= kSmallSeg) {  // descriptors + values at fixed_in, packed
                if (16u * tid < in_bytes) reinterpret_cast<uint4*>(seg)[tid] = spec;
                if (in_bytes > kSvcSpec)
                    small_stage_in<B>(fixed_in + kSvcSpec, seg + kSvcSpec, in_bytes - kSvcSpec);
                __syncthreads();
                desc = reinterpret_cast<const uint64_t*>(seg);
                vals = seg + 16u * n;
            } else if (in_bytes <= kSmallSeg) {
                small_stage_in<B>(reinterpret_cast<const uint8_t*>(desc), seg, 16u * n);
                small_stage_in<B>(vals, seg + 16u * n, vbytes);
                __syncthreads();
                desc = reinterpret_cast<const uint64_t*>(seg);
                vals = seg + 16u * n;
            }
            if (traced && tid == 0) stamp(1, __builtin_amdgcn_s_memrealtime(), __builtin_amdgcn_s_memtime());
            static_assert(kSvcMaxN <= B, "one leaf per thread");
            if ((tid & ~63u) < n) {  // every lane of a wave with a value (sha1_value_all_lanes)
                const bool real = tid < n;
                uint32_t h[5];
                sha1_value_all_lanes(real ? vals + desc[2 * tid] : vals, real ? uint32_t(desc[2 * tid + 1]) : 0u,
                                     h);  // NewLeaf, merklenode.go:27-34
                if (real) store_digest(sm, tid, h);
            }
            if (traced) {
                __syncthreads();
                if (tid == 0) stamp(2, __builtin_amdgcn_s_memrealtime(), __builtin_amdgcn_s_memtime());
            }
            small_levels_and_image<B>(sm, seg, n, out, img_at, traced ? mb->stamps + 10 : nullptr);
            if (traced && tid == 0) stamp(3, __builtin_amdgcn_s_memrealtime(), __builtin_amdgcn_s_memtime());
        }
        served = seq;
        if (tid == 0) __hip_atomic_store(&mb->served, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (traced && tid == 0) {  // before the completion word: the host reads the stamps after it
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp(4, __builtin_amdgcn_s_memrealtime(), __builtin_amdgcn_s_memtime());
        }
        small_signal_done(&mb->done, seq);
    }
}

// ---------------------------------------------------------------------------
// host-side launchers

hipError_t launch_small_tree(const uint64_t* desc, const uint8_t* vals, uint32_t vbytes, uint32_t n, uint8_t* out,
                             uint32_t img_at, uint8_t* scratch, unsigned int* ticket, unsigned int* done, uint32_t seq,
                             hipStream_t s) {
    if (n == 0 || n > kSmallMaxN || (img_at & 15u) || (reinterpret_cast<uintptr_t>(vals) & 15u) ||
        (reinterpret_cast<uintptr_t>(desc) & 15u))
        return hipErrorInvalidValue;
    const unsigned grid = unsigned((n + kSmallBlock - 1) / kSmallBlock);
    hipLaunchKernelGGL(k_small_tree, dim3(grid), dim3(kSmallBlock), 0, s, desc, vals, vbytes, n, out, img_at, scratch,
                       ticket, done, seq);
    return hipGetLastError();
}

hipError_t launch_small_service(SmallMailbox* mb, const SmallMailbox* rb, const uint8_t* in, uint64_t idle_ticks,
                                uint64_t life_ticks, hipStream_t s) {
    if (!mb || !rb || !in || (reinterpret_cast<uintptr_t>(in) & 15u)) return hipErrorInvalidValue;
    static_assert(kSvcSpec <= kSmallSeg, "speculative read inside the input buffer");
    hipLaunchKernelGGL(k_small_service<kSvcBlock>, dim3(1), dim3(kSvcBlock), 0, s, mb, rb, in, idle_ticks,
                       life_ticks);
    return hipGetLastError();
}

static inline unsigned grid_for(uint64_t n) { return unsigned((n + kBlock - 1) / kBlock); }

template <int MODE, int LOAD>
static void leaf_kernel(const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t stride, uint64_t L,
                        const uint32_t* perm, uint64_t n, uint8_t* nodes, hipStream_t s, Gate gate) {
    hipLaunchKernelGGL((k_leaf<MODE, LOAD>), dim3(grid_for(n)), dim3(kBlock), 0, s, base, off, len, stride, L,
                       perm, n, nodes, gate);
}

// load (NKV_OPT_LEAF_LOAD): 4 = 128-byte register runs for 16-byte aligned
// values (anything else takes 11); 11 = the staged paths for every value
template <int MODE>
static void leaf_dispatch(int load, bool aligned, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                          uint64_t stride, uint64_t L, const uint32_t* perm, uint64_t n, uint8_t* nodes,
                          hipStream_t s, Gate g) {
    if (load == 4 && aligned) leaf_kernel<MODE, 4>(base, off, len, stride, L, perm, n, nodes, s, g);
    else leaf_kernel<MODE, 11>(base, off, len, stride, L, perm, n, nodes, s, g);
}

hipError_t launch_leaf_strided(const uint8_t* base, uint64_t stride, uint64_t L, uint64_t n, int load,
                               uint8_t* nodes, hipStream_t s) {
    const bool al = ((reinterpret_cast<uintptr_t>(base) | stride) & 15) == 0;
    leaf_dispatch<0>(load, al, base, nullptr, nullptr, stride, L, nullptr, n, nodes, s, Gate{});
    return hipGetLastError();
}

hipError_t launch_leaf_offsets(const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                               bool aligned, int load, uint8_t* nodes, hipStream_t s, Gate gate) {
    leaf_dispatch<1>(load, aligned, base, off, len, 0, 0, nullptr, n, nodes, s, gate);
    return hipGetLastError();
}

hipError_t launch_leaf_verify(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                              int policy, uint64_t* voff, uint64_t* vlen, uint8_t* nodes, uint32_t* crc_out,
                              unsigned long long* stats, unsigned int* range, uint32_t* part, hipStream_t s,
                              uint32_t* flags, uint32_t* flags_next) {
    const unsigned nb = grid_for(n);
    if (policy == 0) flags = nullptr;
    hipLaunchKernelGGL(k_leaf_verify, dim3(nb), dim3(kBlock), 0, s, stream, stream_len, rec_off, n, policy, voff,
                       vlen, nodes, crc_out, flags ? reinterpret_cast<unsigned long long*>(flags + 4) : stats,
                       (policy == 0 || flags) ? nullptr : part, flags, flags_next);
    if (policy != 0 && !flags)
        hipLaunchKernelGGL(k_locate_fold, dim3(1), dim3(kBlock), 0, s, part, nb, nullptr, range);
    return hipGetLastError();
}

hipError_t launch_leaf_queue(const uint8_t* base, const uint64_t* off, const uint64_t* len, const uint32_t* perm,
                             uint64_t n, uint32_t* q, uint32_t simds, uint32_t waves_per_simd, uint8_t* nodes,
                             hipStream_t s, Gate gate) {
    const uint32_t ngroups = uint32_t((n + 63) / 64);
    const uint32_t waves = simds * std::min<uint32_t>(std::max<uint32_t>(waves_per_simd, 1u), uint32_t(kQueueRing));
    hipLaunchKernelGGL(k_leaf_queue, dim3(waves), dim3(64), 0, s, base, off, len, perm, n, ngroups, simds, q, nodes,
                       gate);
    return hipGetLastError();
}

uint64_t queue_words(uint64_t n) { return kQueueHeader + kSimdKeys + (n + 63) / 64; }

hipError_t launch_reduce(uint8_t* nodes, uint64_t n, int from_level, int top, hipStream_t s, Gate gate) {
    int j0 = from_level;
    // The widest levels two at a time at full lane use (k_reduce2, while a
    // level holds >= kReduce2Min = 512 Ki nodes: that launch is
    // compression-bound); then slabs, which are a chain of one compression per
    // level: 1024-node slabs (10 levels per launch) while a level holds more
    // than 256 nodes, then the last <= 8 levels in 256-node slabs.  At
    // n = 2^20: k_reduce2 0 -> 2, 1024-slabs 2 -> 12, 256-slab 12 -> 20: 52.5 us
    // against 60.7 us for r01's three k_reduce2 and two 256-slab launches
    // (tools/ab_reduce.sh, one box).
    // 4096-node workgroups build the bottom twelve levels in one launch
    // (k_reduce_wide) when the tree is that tall and the level between 64 Ki
    // and 2 Mi nodes: at most two 1024-thread workgroups per CU, so beyond
    // that the ten-level chains run in several rounds (at 8 Mi nodes 231 us
    // against 209 us for k_reduce2 + slabs; at 1 Mi 50.5 against 53.9 us)
    for (uint64_t cnt = j0 == 0 ? n : ((n - 1) >> j0) + 1;
         top - j0 >= 12 && cnt >= kReduceWideMin && cnt <= (uint64_t(2) << 20); cnt = ((cnt - 1) >> 12) + 1) {
        hipLaunchKernelGGL(k_reduce_wide, dim3(unsigned((cnt + 4095) / 4096)), dim3(1024), 0, s, nodes, n, j0,
                           j0 + 12, gate);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        j0 += 12;
    }
    for (uint64_t cnt = j0 == 0 ? n : ((n - 1) >> j0) + 1; top - j0 >= 2 && cnt >= kReduce2Min;
         cnt = ((cnt - 1) >> 2) + 1) {
        const uint64_t waves = (cnt + 255) / 256;
        hipLaunchKernelGGL(k_reduce2, dim3(unsigned((waves + 3) / 4)), dim3(kBlock), 0, s, nodes, n, j0, j0 + 2,
                           gate);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        j0 += 2;
    }
    while (j0 < top) {
        const uint64_t cnt = j0 == 0 ? n : ((n - 1) >> j0) + 1;
        if (cnt > 256 && top - j0 > kSlabLevels) {
            const int jmax = (j0 + 10 < top) ? j0 + 10 : top;
            hipLaunchKernelGGL(k_reduce<1024>, dim3(unsigned((cnt + 1023) / 1024)), dim3(1024), 0, s, nodes, n, j0,
                               jmax, gate);
            j0 = jmax;
        } else {
            const int jmax = (j0 + kSlabLevels < top) ? j0 + kSlabLevels : top;
            hipLaunchKernelGGL(k_reduce<kBlock>, dim3(grid_for(cnt)), dim3(kBlock), 0, s, nodes, n, j0, jmax, gate);
            j0 = jmax;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_bfs_image(const uint8_t* nodes, const BfsLayout& lay, uint8_t* img,
                            hipStream_t s) {
    const uint64_t segs = (lay.total + kBfsSeg - 1) / kBfsSeg;
    if (segs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_bfs_image, dim3(uint32_t(segs)), dim3(kBlock), 0, s, nodes, lay, img);
    return hipGetLastError();
}

// one (lo, hi, flag) triple per workgroup (k_locate, k_leaf_records)
uint64_t locate_part_words(uint64_t n) { return 3 * uint64_t(grid_for(n)); }

hipError_t launch_locate(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off,
                         uint64_t n, uint64_t* voff, uint64_t* vlen, unsigned int* err, unsigned int* range,
                         uint32_t* part, hipStream_t s) {
    const unsigned nb = grid_for(n);
    hipLaunchKernelGGL(k_locate, dim3(nb), dim3(kBlock), 0, s, stream, stream_len, rec_off, n, voff, vlen, part);
    hipLaunchKernelGGL(k_locate_fold, dim3(1), dim3(kBlock), 0, s, part, nb, err, range);
    return hipGetLastError();
}

hipError_t launch_leaf_records(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                               int policy, uint64_t* voff, uint64_t* vlen, uint8_t* nodes, unsigned int* err,
                               unsigned int* range, uint32_t* part, hipStream_t s, uint32_t* flags,
                               uint32_t* flags_next) {
    const unsigned nb = grid_for(n);
    if (policy == 0) flags = nullptr;
    hipLaunchKernelGGL(k_leaf_records, dim3(nb), dim3(kBlock), 0, s, stream, stream_len, rec_off, n, policy, voff,
                       vlen, nodes, part, flags, flags_next);
    if (!flags) hipLaunchKernelGGL(k_locate_fold, dim3(1), dim3(kBlock), 0, s, part, nb, err, range);
    return hipGetLastError();
}

hipError_t scan_exclusive_u64(const uint64_t* in, uint64_t* out, uint64_t n, void* tmp,
                              size_t* tmp_bytes, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, in, out, int(n), s);
}

#ifdef NKV_DIAG
extern "C" int nkv_diag_set_buffer(void* d) {
    unsigned long long* p = static_cast<unsigned long long*>(d);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_diag), &p, sizeof(p)) == hipSuccess ? 0 : 3;
}
#endif

// ---------------------------------------------------------------------------
// In-place exclusive scan of u32 (gated): per-tile sums, one block scans the
// sums, each tile scans itself plus its offset.  a holds n + 1 words when the
// total is wanted (a zero appended).
constexpr int kScanItems = 8;
constexpr uint64_t kScanTile = uint64_t(kBlock) * kScanItems;

// exclusive scan of v over the workgroup (thread order); returns the total
__device__ __forceinline__ uint32_t block_exclusive(uint32_t& v) {
    __shared__ uint32_t wsum[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = uint32_t(__shfl_up(int(x), o));
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        if (w < wave) before += wsum[w];
        total += wsum[w];
    }
    __syncthreads();
    v = before + x - v;
    return total;
}

__global__ __launch_bounds__(kBlock) void k_scan_sums(const uint32_t* __restrict__ a, uint64_t n,
                                                       uint32_t* __restrict__ sums, Gate gate) {
    if (!gate.open()) return;
    const uint64_t base = uint64_t(blockIdx.x) * kScanTile + uint64_t(threadIdx.x) * kScanItems;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j)
        if (base + j < n) s += a[base + j];
    uint32_t v = s;
    const uint32_t tot = block_exclusive(v);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_scan_top(uint32_t* __restrict__ sums, uint32_t nt, Gate gate) {
    if (!gate.open()) return;
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nt; b += kBlock) {  // one workgroup, kBlock sums per round
        uint32_t v = b + threadIdx.x < nt ? sums[b + threadIdx.x] : 0u;
        const uint32_t tot = block_exclusive(v);
        if (b + threadIdx.x < nt) sums[b + threadIdx.x] = carry + v;
        carry += tot;
    }
}

__global__ __launch_bounds__(kBlock) void k_scan_down(uint32_t* __restrict__ a, uint64_t n,
                                                       const uint32_t* __restrict__ sums, Gate gate) {
    if (!gate.open()) return;
    const uint64_t base = uint64_t(blockIdx.x) * kScanTile + uint64_t(threadIdx.x) * kScanItems;
    uint32_t x[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        x[j] = base + j < n ? a[base + j] : 0u;
        s += x[j];
    }
    uint32_t v = s;
    (void)block_exclusive(v);
    uint32_t run = sums[blockIdx.x] + v;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        if (base + j < n) a[base + j] = run;
        run += x[j];
    }
}

uint64_t scan_sums_words(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

hipError_t scan_exclusive_u32(uint32_t* a, uint64_t n, uint32_t* sums, hipStream_t s, Gate gate) {
    const uint64_t nt = scan_sums_words(n);
    if (nt == 0) return hipSuccess;
    if (nt > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_scan_sums, dim3(uint32_t(nt)), dim3(kBlock), 0, s, a, n, sums, gate);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, s, sums, uint32_t(nt), gate);
    hipLaunchKernelGGL(k_scan_down, dim3(uint32_t(nt)), dim3(kBlock), 0, s, a, n, sums, gate);
    return hipGetLastError();
}

uint64_t sort_hist_words(uint64_t n) { return kSortHead + ((n + kSortTile - 1) / kSortTile) * kLenBuckets; }
uint64_t sort_head_words() { return kSortHead; }

// scratch: sort_hist_words(n) u32 whose first sort_head_words() are zero
// (the two-launch form keeps them zero between calls)
hipError_t sort_by_length_desc(const uint64_t* len, uint64_t n, uint32_t* perm, uint32_t* scratch, hipStream_t s,
                               Gate gate, QueueInit qi, CopyWords cw) {
    const uint64_t tiles = (n + kSortTile - 1) / kSortTile;
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(k_len_hist_alloc, dim3(uint32_t(tiles)), dim3(kBlock), 0, s, len, n, scratch,
                       uint32_t(tiles), gate, qi, cw);
    hipLaunchKernelGGL(k_len_scatter_alloc, dim3(uint32_t(tiles)), dim3(kBlock), 0, s, len, n, scratch,
                       uint32_t(tiles), perm, gate, qi);
    return hipGetLastError();
}

hipError_t launch_fill(uint8_t* buf, uint64_t nbytes, uint64_t seed, hipStream_t s) {
    uint64_t threads = (nbytes + 15) / 16;
    uint64_t blocks = (threads + kBlock - 1) / kBlock;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill, dim3(unsigned(blocks)), dim3(kBlock), 0, s, buf, nbytes, seed);
    return hipGetLastError();
}

}  // namespace nkv
