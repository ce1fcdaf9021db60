// crc.hip -- record checksums on gfx950.
//
// Reference: core/record/record.go:51 (New: Crc = crc32.ChecksumIEEE(key ++
// value)) and :163-169 (Deserialize: recompute, panic on mismatch); the
// arithmetic is Go's hash/crc32 IEEE (reflected, poly 0xEDB88320, init and
// final XOR 0xFFFFFFFF).  Key and value are contiguous in a serialized record
// (record.go:191-204), so the checksum covers one byte span per record:
// [rec + 30, rec + 30 + KeySize + ValueSize).
//
// One lane per span.  Slicing-by-4: one 32-bit word per step, four table
// lookups from LDS.  The four 256-entry tables are replicated kCrcCopies times
// and interleaved so lane l reads copy l % kCrcCopies: a ds_read_b32 is served
// in two 32-lane groups over 32 banks, entry e of table k of copy c sits in
// bank (8 e + c) % 32, so the 4 lanes sharing a copy inside a group collide only
// when their entries agree mod 4 (about 2-way on random data instead of ~4-way
// with one copy).
//
// Per span: 0-3 head bytes (byte steps) up to the first 4-aligned address,
// then whole aligned words in aligned 64-byte chunks (4 x global_load_dwordx4
// per lane per chunk; every loaded chunk holds a span byte, so no load leaves
// the span's pages), then 0-3 tail bytes.  Chunks a lane does not own are
// masked; only a span's first and last chunk mask single words.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "crc_dev.hpp"
#include "internal.hpp"

namespace nkv {

__constant__ CrcTables c_crc = make_crc_tables();

__device__ __forceinline__ uint64_t crc_ld_le64(const uint8_t* p) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v |= uint64_t(p[i]) << (8 * i);
    return v;
}

// Same checksum, span bytes staged through a wave-private LDS ring of aligned
// 64-B chunks (two 4 KiB slots, chunk c in slot c & 1) by wave-cooperative
// DMA: instruction k moves one chunk of spans 16k .. 16k+15, 64 contiguous
// bytes each (16 segments per wave-instruction instead of 64 scattered 16-B
// pieces when every lane reads its own span).  Each lane then reads its own
// chunk's four quads.  Chunk c+2 goes into chunk c's slot once c is read.
// Only chunks holding span bytes are fetched (an aligned chunk with one valid
// byte lies in that byte's page).
template <int C>
__device__ __forceinline__ uint32_t crc_span_ring(const uint8_t* s, uint64_t len, const uint32_t* tab,
                                                  uint8_t* wbuf) {
    const int lane = threadIdx.x & 63;
    uint32_t crc = 0xFFFFFFFFu;
    const uint32_t o = uint32_t(reinterpret_cast<uintptr_t>(s)) & 63u;
    const uint32_t nch = len ? uint32_t((o + len + 63) >> 6) : 0u;
    const uint32_t dq = (uint32_t(lane) & 3u) ^ ((uint32_t(lane) >> 4) & 3u);
    const uint8_t* src[4];
    uint32_t nc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = 16 * k + (lane >> 2);
        const uint64_t aj = uint64_t(__shfl(int64_t(reinterpret_cast<uintptr_t>(s - o)), j));
        src[k] = reinterpret_cast<const uint8_t*>(aj) + 16 * dq;
        nc[k] = uint32_t(__shfl(int(nch), j));
    }
    const uint32_t nmax = crc_wave_max(nch);
    if (nmax == 0) return 0u;
    auto issue = [&](uint32_t c) {
        uint8_t* dst = wbuf + 4096 * (c & 1u);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (c < nc[k]) __builtin_amdgcn_global_load_lds(src[k] + 64ull * c, dst + 1024 * k, 16, 0, 0);
    };
    const uint32_t swz = (uint32_t(lane) >> 2) & 3u;
    const uint64_t e = uint64_t(o) + len;  // span end, relative to the first chunk
    issue(0u);
    issue(1u);
    for (uint32_t c = 0; c < nmax; ++c) {
        const uint8_t* rd = wbuf + 4096 * (c & 1u) + 64 * lane;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk c landed (explicit LDS-DMA wait)
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const uint4*>(rd + 16 * (uint32_t(i) ^ swz));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot reads done before refill
        if (c + 2 < nmax) issue(c + 2);
        if (c < nch) {
            const uint32_t w[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                                    v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
            const uint64_t b0 = 64ull * c;  // chunk start, relative
            if (b0 >= o && b0 + 64 <= e) {
                crc = crc_block16<C>(crc, w, tab);
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint64_t a = b0 + 4 * j;
                    const uint32_t lo = a >= o ? 0u : (o - a >= 4 ? 4u : uint32_t(o - a));
                    const uint32_t hi = a >= e ? 0u : (e - a >= 4 ? 4u : uint32_t(e - a));
                    if (lo == 0u && hi == 4u) {
                        crc = crc_word<C>(crc, w[j], tab);
                    } else {
                        for (uint32_t b = lo; b < hi; ++b) crc = crc_byte<C>(crc, (w[j] >> (8 * b)) & 0xFFu, tab);
                    }
                }
            }
        }
    }
    return ~crc;
}

// RECORDS: span of record i from its header at base + off[i] (len unused),
// checked against stream_len; stats[0] += records whose stored Crc differs,
// stats[1] = min such index, stats[2] |= 1 on a header outside the stream.
// Otherwise span i = [base + off[i], + len[i]).
template <bool RECORDS, bool RING, int C, int B>
__global__ __launch_bounds__(B) void k_crc(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                           const uint64_t* __restrict__ len, uint64_t stream_len, uint64_t n,
                                           uint32_t* __restrict__ out, unsigned long long* __restrict__ stats,
                                           Gate gate) {
    __shared__ uint32_t tab[4 * 256 * C];
    if (!gate.open()) return;
    __shared__ __attribute__((aligned(16))) uint8_t ring[RING ? B / 64 : 1][RING ? 8192 : 16];
    for (int i = threadIdx.x; i < 4 * 256 * C; i += B) tab[i] = (&c_crc.t[0][0])[i / C];
    __syncthreads();
    const uint32_t* mytab = tab + (threadIdx.x % C);
    const uint64_t i = uint64_t(blockIdx.x) * B + threadIdx.x;
    const uint8_t* s = base;
    uint64_t L = 0;
    uint32_t stored = 0;
    bool live = i < n, hdr_bad = false;
    if (live) {
        if (RECORDS) {
            const uint64_t r = off[i];
            if (header_in(r, stream_len)) {
                const uint64_t ks = crc_ld_le64(base + r + 14);
                const uint64_t vs = crc_ld_le64(base + r + 22);
                if (ks <= stream_len && vs <= stream_len && r + 30 + ks + vs <= stream_len) {
                    s = base + r + 30;
                    L = ks + vs;
                    stored = uint32_t(base[r]) | uint32_t(base[r + 1]) << 8 | uint32_t(base[r + 2]) << 16 |
                             uint32_t(base[r + 3]) << 24;
                } else {
                    hdr_bad = true;
                }
            } else {
                hdr_bad = true;
            }
        } else {
            s = base + off[i];
            L = len[i];
        }
    }
    const uint32_t crc = RING ? crc_span_ring<C>(s, L, mytab, ring[threadIdx.x >> 6]) : crc_span<C>(s, L, mytab);
    if (!live) return;
    if (out) out[i] = crc;
    if (RECORDS && stats) {
        if (hdr_bad) atomicOr(stats + 2, 1ull);
        else if (crc != stored) {
            atomicAdd(stats, 1ull);
            atomicMin(stats + 1, (unsigned long long)i);
        }
    }
}

// ---------------------------------------------------------------------------
// Span-group form: 16 lanes per span, one 64-byte chunk per lane.
//
// CRC is affine over GF(2): the state after a span is the XOR, over its
// chunks, of each chunk's own state (chunk processed from state 0; the first
// chunk starts from 0xFFFFFFFF at the span's first byte) advanced over the
// bytes that follow the chunk, i.e. multiplied by x^(8d) mod P.  Chunks are
// aligned to the span END (chunk c = [e - 64 (n - c), + 64)), so every chunk
// but the first is a full 64 bytes and every advance is a multiple of 64 bytes:
// a window of 16 chunks is combined in 4 butterfly levels (advance by 64, 128,
// 256, 512 bytes, all lanes of a level by the same distance, one LDS table
// each), and the running state advances by 1 KiB per window.  The first
// window is padded on the left (empty chunks contribute 0), so lengths need no
// tail case; the first chunk's bytes before the span are skipped (dword loads
// from the span only).  Each lane reads its chunk as four 16-byte loads at the
// chunk address (any alignment), so a group's loads cover 1 KiB contiguous.
constexpr int kCrcGroup = 16;

struct CrcShifts {
    uint32_t t[6][4][256];  // advance by 64 << i zero bytes, i = 0..4; [5]: by 16 bytes
};

constexpr uint32_t crc_advance(const uint32_t (&t)[4][256], uint32_t v) {
    return t[0][v & 0xFFu] ^ t[1][(v >> 8) & 0xFFu] ^ t[2][(v >> 16) & 0xFFu] ^ t[3][v >> 24];
}

constexpr CrcShifts make_crc_shifts() {
    const CrcTables T = make_crc_tables();
    CrcShifts r{};
    for (int k = 0; k < 4; ++k)
        for (uint32_t b = 0; b < 256; ++b) {
            uint32_t v = b << (8 * k);
            for (int w = 0; w < 16; ++w) {  // 16 zero words = 64 zero bytes (slicing-by-4 step)
                v = T.t[3][v & 0xFFu] ^ T.t[2][(v >> 8) & 0xFFu] ^ T.t[1][(v >> 16) & 0xFFu] ^ T.t[0][v >> 24];
                if (w == 3) r.t[5][k][b] = v;
            }
            r.t[0][k][b] = v;
        }
    for (int i = 1; i < 5; ++i)  // twice the distance = the advance applied twice
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b)
                r.t[i][k][b] = crc_advance(r.t[i - 1], crc_advance(r.t[i - 1], b << (8 * k)));
    return r;
}

__constant__ CrcShifts c_crc_shift = make_crc_shifts();

__device__ __forceinline__ uint32_t lds_advance(const uint32_t* t, uint32_t v) {
    return t[v & 0xFFu] ^ t[256 + ((v >> 8) & 0xFFu)] ^ t[512 + ((v >> 16) & 0xFFu)] ^ t[768 + (v >> 24)];
}

__device__ __forceinline__ uint32_t ld_u32_any(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

// CRC-32 of [s, s + L) by the 16 lanes of a group (j = lane in the group).
// Every lane of the wave calls it (wave-uniform window loop).
template <int C>
__device__ __forceinline__ uint32_t crc_group_span(const uint8_t* s, uint64_t L, uint32_t j, const uint32_t* tab,
                                                   const uint32_t* sh) {
    const uint64_t nch = (L + 63) >> 6;
    const uint64_t W = (nch + kCrcGroup - 1) / kCrcGroup;
    uint64_t wmax = W;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, uint64_t(__shfl_xor((long long)wmax, o)));
    const uint8_t* e = s + L;
    uint32_t R = 0;
    for (uint64_t w = 0; w < wmax; ++w) {
        const int64_t c = int64_t(nch) - int64_t(kCrcGroup) * (int64_t(W) - int64_t(w)) + int64_t(j);
        uint32_t st = 0;
        if (w < W && c >= 0) {
            const uint8_t* cs = e - 64 * (nch - uint64_t(c));
            const uint32_t h = c == 0 ? uint32_t(64 * nch - L) : 0u;  // chunk bytes before the span
            if (h == 0) {
                // four independent 16-byte sub-chunks (four dependent lookup
                // chains of 4 instead of one of 16), joined by Horner steps of
                // a 16-byte advance
                const uint4* q = reinterpret_cast<const uint4*>(cs);
                uint4 v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = q[i];
                uint32_t a = c == 0 ? 0xFFFFFFFFu : 0u, b = 0u, g = 0u, d = 0u;
                a = crc_quad<C>(a, v[0], tab);
                b = crc_quad<C>(b, v[1], tab);
                g = crc_quad<C>(g, v[2], tab);
                d = crc_quad<C>(d, v[3], tab);
                const uint32_t* s16 = sh + 5 * 1024;
                st = lds_advance(s16, lds_advance(s16, lds_advance(s16, a) ^ b) ^ g) ^ d;
            } else {
                // first chunk, span starts h bytes in: 0-3 bytes up to the chunk's
                // word grid, then whole words, all read from inside the span
                st = 0xFFFFFFFFu;
                const uint32_t jw = (h + 3) >> 2;
                for (uint32_t b = 0; b < 4 * jw - h; ++b) st = crc_byte<C>(st, s[b], tab);
                for (uint32_t i = jw; i < 16; ++i) st = crc_word<C>(st, ld_u32_any(cs + 4 * i), tab);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t other = uint32_t(__shfl_xor(int(st), 1 << k));
            const bool right = (j >> k) & 1u;
            st = lds_advance(sh + 1024 * k, right ? other : st) ^ (right ? st : other);
        }
        if (w < W) R = lds_advance(sh + 4096, R) ^ st;
    }
    return L ? ~R : 0u;
}

// C slicing-table copies, WG threads: 8 x 512 (56 KiB LDS, 2 workgroups per
// CU), 4 x 512 (40 KiB, 4 per CU) or 32 x 1024 (152 KiB, one per CU; lane l
// reads copy l % 32, so every table lookup is bank-conflict free).
template <bool RECORDS, int C, int WG>
__global__ __launch_bounds__(WG) void k_crc_group(const uint8_t* __restrict__ base,
                                                      const uint64_t* __restrict__ off,
                                                      const uint64_t* __restrict__ len, uint64_t stream_len,
                                                      uint64_t n, uint32_t* __restrict__ out,
                                                      unsigned long long* __restrict__ stats, Gate gate) {
    __shared__ uint32_t tab[4 * 256 * C];
    __shared__ uint32_t sh[6 * 4 * 256];
    if (!gate.open()) return;
    for (int i = threadIdx.x; i < 4 * 256 * C; i += WG) tab[i] = (&c_crc.t[0][0])[i / C];
    for (int i = threadIdx.x; i < 6 * 4 * 256; i += WG) sh[i] = (&c_crc_shift.t[0][0][0])[i];
    __syncthreads();
    const uint32_t* mytab = tab + (threadIdx.x % C);
    const uint32_t j = threadIdx.x & (kCrcGroup - 1);
    const uint32_t gw = (threadIdx.x & 63) / kCrcGroup;  // group within the wave
    const uint64_t stride = uint64_t(gridDim.x) * (WG / kCrcGroup);
    // persistent: the tables are loaded once per workgroup; a wave's four groups
    // advance together so the loop bound is wave-uniform
    for (uint64_t i = uint64_t(blockIdx.x) * (WG / kCrcGroup) + threadIdx.x / kCrcGroup; i - gw < n;
         i += stride) {
        const bool live = i < n;
        const uint8_t* s = base;
        uint64_t L = 0;
        uint32_t stored = 0;
        bool hdr_bad = false;
        if (live) {
            if (RECORDS) {
                const uint64_t r = off[i];
                if (header_in(r, stream_len)) {
                    const uint64_t ks = crc_ld_le64(base + r + 14);
                    const uint64_t vs = crc_ld_le64(base + r + 22);
                    if (ks <= stream_len && vs <= stream_len && r + 30 + ks + vs <= stream_len) {
                        s = base + r + 30;
                        L = ks + vs;
                        stored = uint32_t(base[r]) | uint32_t(base[r + 1]) << 8 | uint32_t(base[r + 2]) << 16 |
                                 uint32_t(base[r + 3]) << 24;
                    } else {
                        hdr_bad = true;
                    }
                } else {
                    hdr_bad = true;
                }
            } else {
                s = base + off[i];
                L = len[i];
            }
        }
        const uint32_t crc = crc_group_span<C>(s, L, j, mytab, sh);
        if (live && j == 0) {
            if (out) out[i] = crc;
            if (RECORDS && stats) {
                if (hdr_bad) atomicOr(stats + 2, 1ull);
                else if (crc != stored) {
                    atomicAdd(stats, 1ull);
                    atomicMin(stats + 1, (unsigned long long)i);
                }
            }
        }
    }
}

template <bool RECORDS, int C, int WG>
static void launch_crc_group(int per_cu, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                             uint64_t stream_len, uint64_t n, uint32_t* out, unsigned long long* stats,
                             hipStream_t s, Gate gate) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t groups_per_wg = WG / kCrcGroup;
    const uint64_t want = (n + groups_per_wg - 1) / groups_per_wg;
    const uint32_t grid = uint32_t(std::min<uint64_t>(want, uint64_t(cus) * per_cu));
    hipLaunchKernelGGL((k_crc_group<RECORDS, C, WG>), dim3(grid), dim3(WG), 0, s, base, off, len, stream_len, n,
                       out, stats, gate);
}

// variant 8 / 9: span-group kernel with 8 x 512 / 32 x 1024 table copies x
// workgroup.  Else bit 0 = LDS chunk ring; bits 1-2 = table copies x workgroup
// size: 0 = 8 x 256, 1 = 16 x 512, 2 = 32 x 1024.
template <bool RECORDS>
static void launch_crc(int variant, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                       uint64_t stream_len, uint64_t n, uint32_t* out, unsigned long long* stats, hipStream_t s,
                       Gate gate) {
    if (variant == 8) return launch_crc_group<RECORDS, 8, 512>(2, base, off, len, stream_len, n, out, stats, s, gate);
    if (variant == 9) return launch_crc_group<RECORDS, 32, 1024>(1, base, off, len, stream_len, n, out, stats, s, gate);
    if (variant == 10) return launch_crc_group<RECORDS, 4, 512>(4, base, off, len, stream_len, n, out, stats, s, gate);
    const bool ring = variant & 1;
    const int cfg = (variant >> 1) & 3;
    const int B = cfg == 0 ? 256 : (cfg == 1 ? 512 : 1024);
    const dim3 grid(uint32_t((n + B - 1) / B)), block(B);
#define NKV_CRC_LAUNCH(R, C, BB) \
    hipLaunchKernelGGL((k_crc<RECORDS, R, C, BB>), grid, block, 0, s, base, off, len, stream_len, n, out, stats, gate)
    if (cfg == 0) {
        if (ring) NKV_CRC_LAUNCH(true, 8, 256);
        else NKV_CRC_LAUNCH(false, 8, 256);
    } else if (cfg == 1) {
        if (ring) NKV_CRC_LAUNCH(true, 16, 512);
        else NKV_CRC_LAUNCH(false, 16, 512);
    } else {
        NKV_CRC_LAUNCH(false, 32, 1024);  // 128 KiB of tables: no room for a ring
    }
#undef NKV_CRC_LAUNCH
}

hipError_t launch_crc_spans(const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                            uint32_t* out, int variant, hipStream_t s) {
    launch_crc<false>(variant, base, off, len, 0, n, out, nullptr, s, Gate{});
    return hipGetLastError();
}

hipError_t launch_record_crc(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                             uint32_t* out, unsigned long long* stats, int variant, hipStream_t s, Gate gate,
                             bool init_stats) {
    if (init_stats) {
        hipError_t e = hipMemsetAsync(stats, 0, 3 * sizeof(unsigned long long), s);
        if (e == hipSuccess) e = hipMemsetAsync(stats + 1, 0xFF, sizeof(unsigned long long), s);
        if (e != hipSuccess) return e;
    }
    launch_crc<true>(variant, stream, rec_off, nullptr, stream_len, n, out, stats, s, gate);
    return hipGetLastError();
}

}  // namespace nkv
