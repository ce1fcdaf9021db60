// crc.hip -- record checksums on gfx950.
//
// Reference: core/record/record.go:51 (New: Crc = crc32.ChecksumIEEE(key ++
// value)) and :163-169 (Deserialize: recompute, panic on mismatch); the
// arithmetic is Go's hash/crc32 IEEE (reflected, poly 0xEDB88320, init and
// final XOR 0xFFFFFFFF).  Key and value are contiguous in a serialized record
// (record.go:191-204), so the checksum covers one byte span per record:
// [rec + 30, rec + 30 + KeySize + ValueSize).
//
// One lane per span (k_crc_lanes).  Slicing-by-4: one 32-bit word per step,
// four table lookups from LDS.  The 4 x 256 tables are stored once per bank:
// 32 copies, copy c read only by the lanes l with l % 32 = c, entry e of copy
// c at byte e * 256 + c * 4 (+ 128 for tables 1 and 3, + 64 KiB for tables 2
// and 3), so a ds_read_b32 -- served 32 lanes per cycle over 32 banks -- has
// lane l alone in bank l % 32: no bank conflict, whatever the data (the 8-copy
// interleave of rounds 1-2 spent 63 % of its LDS cycles in conflicts,
// profiles/r01_crc_pmc_lds.json).  The row stride of 256 bytes makes each
// lookup's LDS address ONE v_perm_b32: byte j of x lands in address byte 1,
// the lane's copy offset (c * 4) in byte 0 and the 64 KiB table half in byte
// 2, both from a per-lane constant; the 128-byte half comes from the
// ds_read's immediate offset.  128 KiB of tables: one 1024-thread workgroup
// per CU (4 waves per SIMD), persistent over the spans.
//
// Per span: 0-3 head bytes (byte steps from the aligned word that holds them)
// up to the first 4-aligned address, then whole aligned words from whole
// aligned 128-byte lines (eight global_load_dwordx4 per lane per line, the
// next line loaded while this one is checksummed; a line holding a span byte
// lies in that byte's page), then 0-3 tail bytes (from one aligned word).
// Only a span's first and last line mask words.  The records form loads a
// record's header, head word and first line together (crc_span_lines).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "crc_dev.hpp"
#include "internal.hpp"

namespace nkv {

__constant__ CrcTables c_crc = make_crc_tables();

// Lane-private table layout: two 64 KiB halves (tables 0, 1 and 2, 3) of 256
// rows (entry e) of 64 words: words 0-31 = table 2h, copies 0-31; words 32-63 =
// table 2h + 1.  k_crc_lanes's only LDS object, so it starts at LDS address 0
// (checked in the kernel).
constexpr uint32_t kLaneTabWords = 2 * 256 * 64;  // 128 KiB

// one lookup: table k (compile-time), byte j (0..3) of x; la = lane constant of
// table half k >> 1 (c * 4 in byte 0, the half in byte 2)
template <int K, int J>
__device__ __forceinline__ uint32_t lane_lut(uint32_t x, uint32_t la) {
    // address = {0, la.byte2, x.byte J, la.byte0}: v_perm over (hi = x, lo = la)
    constexpr uint32_t sel = (12u << 24) | (2u << 16) | (uint32_t(4 + J) << 8) | 0u;
    const uint32_t addr = __builtin_amdgcn_perm(x, la, sel);
    uint32_t v;
    // "memory": the read depends on the table fill (its address comes from the
    // table's own LDS address through la, so the fill cannot be dropped either)
    if constexpr (K & 1) asm volatile("ds_read_b32 %0, %1 offset:128" : "=v"(v) : "v"(addr) : "memory");
    else asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

// x = crc ^ w form (crc_dev.hpp): the state after word w given x, without the
// next word (last) or with it folded in (next)
// (the lookups are inline asm, so the waits are explicit; the wait names the
// loaded registers as in/out operands, so no use of them is scheduled before it)
__device__ __forceinline__ uint32_t lane_x_next(uint32_t x, uint32_t w, uint32_t la0, uint32_t la1) {
    uint32_t a = lane_lut<3, 0>(x, la1), b = lane_lut<2, 1>(x, la1);
    uint32_t c = lane_lut<1, 2>(x, la0), d = lane_lut<0, 3>(x, la0);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    return crc_xor3(crc_xor3(a, b, c), d, w);
}
__device__ __forceinline__ uint32_t lane_x_last(uint32_t x, uint32_t la0, uint32_t la1) {
    return lane_x_next(x, 0u, la0, la1);
}
__device__ __forceinline__ uint32_t lane_byte(uint32_t crc, uint32_t b, uint32_t la0) {
    uint32_t t = lane_lut<0, 0>((crc ^ b) & 0xFFu, la0);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t));
    return t ^ (crc >> 8);
}

__device__ __forceinline__ uint64_t crc_ld_le64(const uint8_t* p) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v |= uint64_t(p[i]) << (8 * i);
    return v;
}

// Crc, KeySize, ValueSize of the record header at p (record.go:191-199: Crc at
// +0, KeySize at +14, ValueSize at +22) from aligned 8-byte loads, each inside
// the aligned word that holds a header byte (no page past the header).
__device__ __forceinline__ void crc_header(const uint8_t* p, uint32_t& stored, uint64_t& ks, uint64_t& vs) {
    const uint32_t m = uint32_t(reinterpret_cast<uintptr_t>(p) & 7u);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p - m);
    uint64_t w[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = (i < 4 || m + 29 >= 32) ? q[i] : 0ull;
    auto at = [&](uint32_t off) {  // 8 bytes from header offset off
        const uint32_t o = m + off, k = o >> 3, sh = (o & 7u) * 8u;
        uint64_t lo = 0, hi = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            lo = uint32_t(i) == k ? w[i] : lo;
            hi = uint32_t(i) == k ? w[i + 1] : hi;
        }
        return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
    };
    stored = uint32_t(at(0));
    ks = at(14);
    vs = at(22);
}

// A readable 128-byte line (zeros) for lanes that have no line of their own to
// load: every line load of the span loop below is issued by every lane.
__device__ __align__(128) uint4 g_crc_line[8];

// A line is eight 16-byte vector loads into vector registers: as vectors (not
// uint4 structs, whose fields the compiler splits into dword loads and
// re-merges) the loads stay aligned dwordx4 at offsets 0, 16, ... 112.
typedef uint32_t crc_v4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void crc_line_load(const uint4* q, crc_v4 v[8]) {
    const crc_v4* p = reinterpret_cast<const crc_v4*>(q);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = p[i];
}

// The aligned 128-byte line v at address b0 stepped into crc: every word of a
// line inside [s4, e4), else (a span's first or last line) every word steps and
// the ones outside are discarded (static indices keep the line in VGPRs).
__device__ __forceinline__ uint32_t crc_line(uint32_t crc, const crc_v4 v[8], uint64_t b0, uint64_t s4, uint64_t e4,
                                             uint32_t la0, uint32_t la1) {
    uint32_t w[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) w[j] = v[j >> 2][j & 3];
    if (b0 >= s4 && b0 + 128 <= e4) {
        uint32_t x = crc ^ w[0];
#pragma unroll
        for (int j = 1; j < 32; ++j) x = lane_x_next(x, w[j], la0, la1);
        return lane_x_last(x, la0, la1);
    }
    const uint32_t lo = s4 > b0 ? uint32_t((s4 - b0) >> 2) : 0u;
    const uint32_t hi = e4 - b0 >= 128 ? 32u : uint32_t((e4 - b0) >> 2);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const uint32_t u = lane_x_last(crc ^ w[j], la0, la1);
        crc = (uint32_t(j) >= lo && uint32_t(j) < hi) ? u : crc;
    }
    return crc;
}

// Bytes j0 .. j0 + nb - 1 (nb 0..3) of the little-endian word hw stepped into crc.
__device__ __forceinline__ uint32_t crc_word_bytes(uint32_t crc, uint32_t hw, uint32_t j0, uint32_t nb,
                                                   uint32_t la0) {
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j)
        if (j < nb) crc = lane_byte(crc, (hw >> (8u * (j0 + j))) & 0xFFu, la0);
    return crc;
}

// The first line of the record at rec that the span loop can use: the line of
// its Key || Value's first aligned word (rec + 30 rounded up to 4) when that
// line also holds header byte 29 (so it is mapped whatever the record's
// length), else the header's last line.
__device__ __forceinline__ const uint4* crc_record_line(const uint8_t* rec) {
    const uint64_t ra = uint64_t(reinterpret_cast<uintptr_t>(rec));
    const uint64_t b29 = ra + 29, A = ((ra + 33) & ~uint64_t(3)) & ~uint64_t(127);
    return reinterpret_cast<const uint4*>(rec + ((A <= b29 ? A : b29 & ~uint64_t(127)) - ra));
}

// CRC-32/IEEE of [s, s + len) for every lane of the wave (dead lanes: len 0),
// from whole aligned 128-byte lines, with the lane-private tables.
//
// The caller has loaded hw, the aligned word holding the span's first byte
// (used when the span starts inside it); va holds the line at va_from, and
// when that is the span's first line the loop starts from it.  The records
// kernel loads that line together with the record header, so the header's
// line is read from memory once (loaded after the header, as in the first
// version, the line had left the L2 under the stream and was read again:
// 1.086 x the payload read, now 1.055).  The 0-3 tail bytes come from one
// aligned word loaded before the loop.
//
// Two line buffers in turn: line c + 1 loads while line c is checksummed.  The
// loop's loads are unconditional -- a line past the span (or a lane with none)
// loads g_crc_line, which stays in the caches -- so every path issues the same
// loads and the compiler's wait before a line's first word is vmcnt(8) (only
// the line in flight may still be outstanding).  With the loads under per-lane
// conditions, or a buffer copy at the loop end, its merged counts forced
// vmcnt(0) in mid-line, which waited for the prefetch as well (4.67 TB/s).
__device__ __forceinline__ uint32_t crc_span_lines(const uint8_t* s, uint64_t len, uint32_t hw, crc_v4 va[8],
                                                   const uint4* va_from, uint32_t la0, uint32_t la1) {
    const uint64_t sa = uint64_t(reinterpret_cast<uintptr_t>(s));
    const uint64_t ea = sa + len;
    const uint64_t s4 = (sa + 3) & ~uint64_t(3);
    const uint64_t e4 = ea & ~uint64_t(3);
    const uint64_t hb = s4 < ea ? s4 : ea;
    const uint64_t tb = e4 > hb ? e4 : hb;
    const uint64_t A = s4 & ~uint64_t(127);
    const uint32_t nl = e4 > s4 ? uint32_t((e4 - A + 127) >> 7) : 0u;
    const uint32_t nmax = crc_wave_max(nl);
    // s + (A - sa): stays a global pointer (no integer-to-pointer cast)
    const uint4* q = reinterpret_cast<const uint4*>(s + (A - sa));
    auto line = [&](uint32_t c) { return c < nl ? q + 8 * c : g_crc_line; };
    // the tail word holds bytes of the span when there is a tail
    const uint32_t* tp = ea > tb ? reinterpret_cast<const uint32_t*>(s + (tb - sa)) : reinterpret_cast<const uint32_t*>(g_crc_line);
    const uint32_t tw = *tp;
    if (line(0) != va_from) crc_line_load(line(0), va);
    uint32_t crc = crc_word_bytes(0xFFFFFFFFu, hw, uint32_t(sa & 3u), uint32_t(hb - sa), la0);
    crc_v4 vb[8];
    for (uint32_t c = 0; c < nmax; c += 2) {
        crc_line_load(line(c + 1), vb);
        if (c < nl) crc = crc_line(crc, va, A + 128ull * c, s4, e4, la0, la1);
        crc_line_load(line(c + 2), va);
        if (c + 1 < nl) crc = crc_line(crc, vb, A + 128ull * (c + 1), s4, e4, la0, la1);
    }
    crc = crc_word_bytes(crc, tw, 0u, uint32_t(ea - tb), la0);
    return ~crc;
}

// RECORDS: span of record i from its header at base + off[i] (len unused),
// checked against stream_len; stats[0] += records whose stored Crc differs,
// stats[1] = min such index, stats[2] |= 1 on a header outside the stream.
// Otherwise span i = [base + off[i], + len[i]).  Persistent: the grid is one
// workgroup per CU, each loading the tables once.
constexpr int kCrcLanesWG = 1024;
template <bool RECORDS>
__global__ __launch_bounds__(kCrcLanesWG) void k_crc_lanes(const uint8_t* __restrict__ base,
                                                            const uint64_t* __restrict__ off,
                                                            const uint64_t* __restrict__ len, uint64_t stream_len,
                                                            uint64_t n, uint32_t* __restrict__ out,
                                                            unsigned long long* __restrict__ stats, Gate gate) {
    constexpr int WG = kCrcLanesWG;
    __shared__ uint32_t tab[kLaneTabWords];
    if (!gate.open()) return;
    for (uint32_t i = threadIdx.x; i < kLaneTabWords; i += WG) {
        const uint32_t half = i >> 14, e = (i >> 6) & 255u, k = 2u * half + ((i >> 5) & 1u);
        tab[i] = c_crc.t[k][e];  // every copy c = i & 31 holds the same entry
    }
    __syncthreads();
    // lane constants of the two halves: the copy offset (byte 0), the half (byte
    // 2), built on the table's real LDS address.  The v_perm address
    // form has no room for a base, so the table must be the kernel's only LDS
    // object, at address 0: the launcher checks the kernel's LDS size once
    // (lanes_layout_ok) and refuses to launch otherwise (a trap here
    // would take the whole process down); the diagnostic build also asserts it.
    const uint32_t lds_tab = uint32_t(reinterpret_cast<uintptr_t>(tab));
#ifdef NKV_DIAG
    if (lds_tab != 0u) __builtin_trap();
#endif
    const uint32_t la0 = lds_tab + (threadIdx.x & 31u) * 4u, la1 = la0 | 0x10000u;
    const uint64_t stride = uint64_t(gridDim.x) * WG;
    const uint64_t w0 = uint64_t(blockIdx.x) * WG + (threadIdx.x & ~63u);  // this wave's first span
    for (uint64_t wb = w0; wb < n; wb += stride) {  // wave-uniform loop
        const uint64_t i = wb + (threadIdx.x & 63u);
        const bool live = i < n;
        // (loading the next span's offset a span ahead measured the same)
        const uint64_t off_i = live ? off[i] : 0;
        const uint64_t len_i = live && !RECORDS ? len[i] : 0;
        const uint8_t* s = base;
        uint64_t L = 0;
        uint32_t stored = 0;
        bool hdr_bad = false;
        crc_v4 va[8];
        const uint4* first = g_crc_line;
        uint32_t hw = 0;
        if (RECORDS) {
            // The header, the aligned word holding byte 29 (the span Key || Value
            // starts at +30, so its 0-3 head bytes share that word) and the
            // span's first line, issued together: one memory read of the
            // header's line.  Lanes without a header in the stream read
            // g_crc_line instead.
            const uint64_t r = live ? off_i : 0;
            const bool hin = live && header_in(r, stream_len);
            const uint8_t* rec = hin ? base + r : reinterpret_cast<const uint8_t*>(g_crc_line);
            first = crc_record_line(rec);
            crc_line_load(first, va);
            const uint64_t ra = uint64_t(reinterpret_cast<uintptr_t>(rec));
            hw = *reinterpret_cast<const uint32_t*>(rec + (((ra + 29) & ~uint64_t(3)) - ra));
            uint64_t ks, vs;
            crc_header(rec, stored, ks, vs);
            if (!hin) {
                hdr_bad = live;
            } else if (ks <= stream_len && vs <= stream_len && r + 30 + ks + vs <= stream_len) {
                s = base + r + 30;
                L = ks + vs;
            } else {
                hdr_bad = true;
            }
        } else if (live) {
            s = base + off_i;
            L = len_i;
            const uint32_t m = uint32_t(reinterpret_cast<uintptr_t>(s) & 3u);
            hw = *(m && L ? reinterpret_cast<const uint32_t*>(s - m) : reinterpret_cast<const uint32_t*>(g_crc_line));
        }
        const uint32_t crc = crc_span_lines(s, L, hw, va, RECORDS ? first : nullptr, la0, la1);
        if (live) {
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

// variant (NKV_OPT_CRC_LOAD) 0: one lane per span, lane-private tables
// (k_crc_lanes, one 1024-thread workgroup per CU); 8: 16 lanes per span
// (k_crc_group, 8 x 512 interleaved table copies: for a few long spans)
template <bool RECORDS>
static void launch_crc(int variant, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                       uint64_t stream_len, uint64_t n, uint32_t* out, unsigned long long* stats, hipStream_t s,
                       Gate gate) {
    if (variant == 8) return launch_crc_group<RECORDS, 8, 512>(2, base, off, len, stream_len, n, out, stats, s, gate);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    auto go = [&](auto kernel, int wg) {
        const uint64_t want = (n + wg - 1) / wg;
        const uint32_t grid = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>(want, uint64_t(cus))));
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(wg), 0, s, base, off, len, stream_len, n, out, stats, gate);
    };
    go(k_crc_lanes<RECORDS>, kCrcLanesWG);
}

// k_crc_lanes addresses its table by v_perm with no base, so the table must
// be the kernel's only LDS object (at address 0): its static LDS size is
// exactly the table's.  Checked once per process and kernel on the host.
template <bool RECORDS>
static hipError_t lanes_layout_ok() {
    static const hipError_t ok = [] {
        hipFuncAttributes a;
        hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_crc_lanes<RECORDS>));
        if (e != hipSuccess) return e;
        return a.sharedSizeBytes == size_t(kLaneTabWords) * 4 ? hipSuccess : hipErrorInvalidDeviceFunction;
    }();
    return ok;
}

hipError_t launch_crc_spans(const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                            uint32_t* out, int variant, hipStream_t s) {
    if (variant != 8) {
        const hipError_t e = lanes_layout_ok<false>();
        if (e != hipSuccess) return e;
    }
    launch_crc<false>(variant, base, off, len, 0, n, out, nullptr, s, Gate{});
    return hipGetLastError();
}

hipError_t launch_record_crc(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                             uint32_t* out, unsigned long long* stats, int variant, hipStream_t s, Gate gate,
                             bool init_stats) {
    if (variant != 8) {
        const hipError_t e = lanes_layout_ok<true>();
        if (e != hipSuccess) return e;
    }
    if (init_stats) {
        hipError_t e = hipMemsetAsync(stats, 0, 3 * sizeof(unsigned long long), s);
        if (e == hipSuccess) e = hipMemsetAsync(stats + 1, 0xFF, sizeof(unsigned long long), s);
        if (e != hipSuccess) return e;
    }
    launch_crc<true>(variant, stream, rec_off, nullptr, stream_len, n, out, stats, s, gate);
    return hipGetLastError();
}

}  // namespace nkv
