// internal.hpp -- launcher declarations shared by kernels.hip and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nkv {

constexpr int kBlock = 256;       // threads per workgroup = leaves per K1 block
constexpr int kSlabLevels = 8;    // log2(kBlock): levels one k_reduce workgroup builds
// levels of at least this many nodes are reduced two at a time at full lane
// use (k_reduce2) before the slabs take over (launch_reduce)
constexpr uint64_t kReduce2Min = 524288;
// levels of at least this many nodes (and at least 12 below the top) take the
// bottom-twelve-levels launch (k_reduce_wide) first
constexpr uint64_t kReduceWideMin = 65536;
constexpr int kMaxLevels = 64;
constexpr int kLeafWavesPerSimd = 8;  // 8 waves/SIMD <=> <= 64 VGPRs

// Device-side choice between two leaf kernels launched back to back (no host
// read-back): range = the batch's (min, max) full-block counts from
// launch_len_range; pol 1 runs the kernel only for a narrow range (input
// order), pol 2 only for a wide one (length-sorted work queue), 0 always.
// A record header [r, r + 30) (record.go:191-199) lies inside a stream of len
// bytes; written so that a wild offset near 2^64 cannot wrap past the check.
__host__ __device__ inline bool header_in(uint64_t r, uint64_t len) { return r <= len && len - r >= 30; }

struct Gate {
    const unsigned int* range = nullptr;
    int pol = 0;
    __device__ __forceinline__ bool open() const {
        if (pol == 0) return true;
        const unsigned int lo = range[0], hi = range[1];
        const bool narrow = hi <= lo + (lo / 16 > 1u ? lo / 16 : 1u);
        return narrow == (pol == 1);
    }
};

// Pass flags of the records entries' deferred plan (k_leaf_records,
// k_leaf_verify), instead of per-workgroup partials and a fold launch: two
// sets per context, used by alternate calls, and each call's leaf kernel
// resets the other set, so no fill launch precedes it either.  Words: [0] 0
// (the wide Gate's lo), [1] ~0 once a wave was deferred (its hi), [2] 1 if a
// header lies outside the stream, [3] pad, [4..9] the verify pass's stats
// (3 u64: mismatches, first mismatch, bad header), [10..16) pad.  The first
// length-sort launch copies [2] (or the stats) to the caller (CopyWords).
constexpr uint32_t kPassFlagWords = 16;
struct CopyWords {
    const uint32_t* src = nullptr;
    uint32_t* dst = nullptr;
    uint32_t n = 0;  // words, at most 256
};

// BFS image layout in image order (index 0 = top level).
struct BfsLayout {
    int nlev;
    uint64_t total;
    uint64_t img_start[kMaxLevels];   // first image byte of the level
    uint64_t node_start[kMaxLevels];  // first node of the level in the nodes buffer
    uint64_t count[kMaxLevels];       // real nodes in the level
};

// load: leaf-kernel load path (NKV_OPT_LEAF_LOAD): 4 = 128-byte register runs
// for 16-byte aligned values (unaligned ones take 11), 11 = the staged paths
// (segment stage, 80-byte window stage, value-relative LDS-DMA stream) for any.
// Level 0 (the leaf digests) only; launch_reduce builds the levels above.
hipError_t launch_leaf_strided(const uint8_t* base, uint64_t stride, uint64_t L, uint64_t n, int load,
                               uint8_t* nodes, hipStream_t s);
// In input order (the length-sorted order goes through launch_leaf_queue).
hipError_t launch_leaf_offsets(const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                               bool aligned, int load, uint8_t* nodes, hipStream_t s, Gate gate = Gate{});
// The work queue's state (queue_words(n) u32 at q), set up by the length sort
// that precedes the queue kernel (sort_by_length_desc with a QueueInit): split
// = longest chain (compressions - 1) of a group the non-priority waves take
// when the longest chain bounds the batch.
uint64_t queue_words(uint64_t n);
struct QueueInit {
    uint32_t* q = nullptr;  // nullptr: no queue follows the sort
    uint64_t nq = 0;
    uint32_t split = 0;
};
// Ragged batch through the work-queue leaf kernel (perm = length-sorted order,
// longest first; q set up by the sort), values staged through a pipelined LDS
// ring of value-relative chunks; waves_per_simd: 1..3.
hipError_t launch_leaf_queue(const uint8_t* base, const uint64_t* off, const uint64_t* len, const uint32_t* perm,
                             uint64_t n, uint32_t* q, uint32_t simds, uint32_t waves_per_simd, uint8_t* nodes,
                             hipStream_t s, Gate gate = Gate{});
hipError_t launch_reduce(uint8_t* nodes, uint64_t n, int from_level, int top, hipStream_t s, Gate gate = Gate{});
hipError_t launch_bfs_image(const uint8_t* nodes, const BfsLayout& lay, uint8_t* img,
                            hipStream_t s);
// err (u32): 1 if any header points outside the stream, else 0; range
// (nullable, 2 u32): min / max full-block count of the values, as
// launch_len_range writes it.  Neither needs initialising; part: scratch of
// locate_part_words(n) u32.
uint64_t locate_part_words(uint64_t n);
hipError_t launch_locate(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off,
                         uint64_t n, uint64_t* voff, uint64_t* vlen, unsigned int* err, unsigned int* range,
                         uint32_t* part, hipStream_t s);
// The records form's leaf pass (k_leaf_records): locate each record's value and
// hash it in input order (policy 0), only in waves of narrow block counts (1,
// the rest deferred to the length-sorted pass), or never (2); voff / vlen
// receive the deferred values' places (kDone for hashed ones); err / range /
// part as launch_locate, range opening the wide Gate iff something was deferred.
// flags (policy != 0, nullable): this call's pass flags (kPassFlagWords u32)
// instead of err / range / part, and flags_next the set the kernel resets.
hipError_t launch_leaf_records(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                               int policy, uint64_t* voff, uint64_t* vlen, uint8_t* nodes, unsigned int* err,
                               unsigned int* range, uint32_t* part, hipStream_t s, uint32_t* flags = nullptr,
                               uint32_t* flags_next = nullptr);
hipError_t scan_exclusive_u64(const uint64_t* in, uint64_t* out, uint64_t n, void* tmp,
                              size_t* tmp_bytes, hipStream_t s);
// In-place exclusive scan of n u32 (gated); sums: scan_sums_words(n) u32.
uint64_t scan_sums_words(uint64_t n);
hipError_t scan_exclusive_u32(uint32_t* a, uint64_t n, uint32_t* sums, hipStream_t s, Gate gate = Gate{});
// Length-sorted order (compression count, longest first) into perm[0..n);
// scratch: sort_hist_words(n) u32 whose first sort_head_words() must be zero
// when the scratch is first used (the sort leaves them zero again).
uint64_t sort_hist_words(uint64_t n);
uint64_t sort_head_words();
// cw: words block 0 of the first launch copies before it reads the gate.
hipError_t sort_by_length_desc(const uint64_t* len, uint64_t n, uint32_t* perm, uint32_t* hist, hipStream_t s,
                               Gate gate = Gate{}, QueueInit qi = QueueInit{}, CopyWords cw = CopyWords{});
// crc.hip: CRC-32/IEEE of byte spans / of records' Key ++ Value (stats: 3 x u64,
// initialised by the launcher).
// variant: NKV_OPT_CRC_LOAD (0 = one lane per span, lane-private tables; 8 =
// 16 lanes per span).
hipError_t launch_crc_spans(const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                            uint32_t* out, int variant, hipStream_t s);
// init_stats: reset stats to {0, UINT64_MAX, 0} first (false: the caller did)
hipError_t launch_record_crc(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                             uint32_t* out, unsigned long long* stats, int variant, hipStream_t s,
                             Gate gate = Gate{}, bool init_stats = true);
// The compaction read in one pass (kernels.hip k_leaf_verify): for the record at
// stream + rec_off[i], its CRC of Key ++ Value into crc_out[i] (nullable),
// checked against the stored Crc into stats as launch_record_crc does (stats
// initialised by the caller), and the leaf digest of its Value into nodes
// (level 0) -- for every wave (policy 0), for the narrow waves (1: the others
// leave voff / vlen for the sorted pass, hashed ones kDone, and range opens
// its wide Gate only if a wave was deferred), or for none (2).  part: scratch
// of locate_part_words(n) u32; voff / vlen / range / part unused for policy 0.
// flags (policy != 0): the pass flags replace range / part, and the stats go to
// flags + 4 (copied out by the sort's first launch); flags_next as above.
hipError_t launch_leaf_verify(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                              int policy, uint64_t* voff, uint64_t* vlen, uint8_t* nodes, uint32_t* crc_out,
                              unsigned long long* stats, unsigned int* range, uint32_t* part, hipStream_t s,
                              uint32_t* flags = nullptr, uint32_t* flags_next = nullptr);
// bloom.hip: mode 0 = keys at base + off[i], len[i]; 1 = keys of the records at
// base + off[i].  query: out[i] = all k bits set; else OR the bits in.
hipError_t launch_bloom(int mode, bool query, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                        uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0, uint32_t* bits,
                        uint8_t* out, unsigned int* err, hipStream_t s);
// Range-privatised insert (mode as launch_bloom); scratch: bloom_ranges_scratch_words
// u32 (0 = not applicable: more than 4096 ranges of 32768 bits, or n * k >= 2^32).
uint64_t bloom_ranges_scratch_words(uint64_t n, uint32_t m, uint32_t k);
hipError_t launch_bloom_ranges(int mode, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                               uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0,
                               uint32_t* bits, unsigned int* err, uint32_t* scratch, hipStream_t s);
// Staged insert (one hash pass; mode as launch_bloom); scratch:
// bloom_staged_scratch_words u32 (0 = not applicable: k > 32 or more than
// 4096 ranges).
uint64_t bloom_staged_scratch_words(uint64_t n, uint32_t m, uint32_t k);
hipError_t launch_bloom_staged(int mode, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                               uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0,
                               uint32_t* bits, unsigned int* err, uint32_t* scratch, hipStream_t s);
hipError_t launch_fill(uint8_t* buf, uint64_t nbytes, uint64_t seed, hipStream_t s);
// One-launch small tree (kernels.hip k_small_tree): desc = n (offset, length)
// u64 pairs, value i at vals + offset (16-byte aligned); out receives
// the nodes (level-major) and, at out + img_at (16-byte aligned; 0 = none), the Serialize
// image.  scratch: 20 n device bytes; ticket: one device u32, zero before the
// first launch (each launch leaves it zero).
constexpr uint32_t kSmallMaxN = 1024;
constexpr uint32_t kSmallSeg = 16384;  // LDS stage: the staged input, then image segments
// vbytes: the values lie in vals[0, vbytes).  done (nullable, host-coherent
// memory): receives seq once every output byte is written.
hipError_t launch_small_tree(const uint64_t* desc, const uint8_t* vals, uint32_t vbytes, uint32_t n, uint8_t* out,
                             uint32_t img_at, uint8_t* scratch, unsigned int* ticket, unsigned int* done, uint32_t seq,
                             hipStream_t s);
// The resident small-tree service (kernels.hip k_small_service,
// NKV_OPT_SMALL_PATH 3).  The host writes a request (the fields after `done`,
// as launch_small_tree's arguments) and then its seq into `doorbell`; the
// service answers with seq in `done` behind every output byte.  Two copies of
// the struct may be in play: the request side (doorbell, req) in device memory
// the host stores to through a large BAR, the answer side (served, done,
// refused, stamps) in host-coherent memory; or one host-coherent copy for both.
struct alignas(64) SmallRequest {  // one 64-byte line: the service reads it with ONE load
    uint32_t n, vbytes, img_at, trace;  // trace: nonzero = stamp this request's phases
    uint64_t desc, vals, out;           // device addresses of host-coherent memory
    uint32_t inline_in;                 // 1: descriptors + values packed at the service's own
                                        // input buffer (its first kSvcSpec bytes come with the request)
    uint32_t pad0;
    uint64_t pad1;
};
struct alignas(64) SmallMailbox {
    uint32_t doorbell;  // host: seq of the latest request; kSvcExit: leave
    uint32_t served;    // service: the latest seq it served (a relaunch resumes from it)
    uint32_t done;      // service: seq whose outputs are all written
    uint32_t refused;   // service: seq of a request it refused (a field out of range): nothing written
    uint32_t hw_id;     // service: HW_REG_HW_ID of its wave 0 at launch (diagnostics: CU, SIMD, SE)
    uint32_t xcc_id;    // service: HW_REG_XCC_ID at launch (which XCD)
    uint32_t pad[10];
    SmallRequest req;   // host: written before the doorbell
    // service, when traced: (s_memrealtime, s_memtime) after the doorbell was
    // seen, the input staged, the leaves hashed, the levels + image written,
    // the completion word stored; then after the levels, after the first image
    // segment was built
    uint64_t stamps[14];
};
constexpr int kSvcStamps = 14;
// the service reads the request line as 16 dwords: [0] n, [1] vbytes, [2]
// img_at, [3] trace, [4..5] desc, [6..7] vals, [8..9] out, [10] inline_in
static_assert(offsetof(SmallMailbox, req) == 64 && sizeof(SmallRequest) == 64, "request line");
static_assert(offsetof(SmallRequest, desc) == 16 && offsetof(SmallRequest, vals) == 24 &&
                  offsetof(SmallRequest, out) == 32 && offsetof(SmallRequest, inline_in) == 40,
              "request dwords");
constexpr uint32_t kSvcExit = 0xFFFFFFFFu;
constexpr uint32_t kSvcBlock = 256;  // one workgroup, one lane per leaf
constexpr uint32_t kSvcMaxN = 256;   // larger batches take the one-launch kernel
constexpr uint32_t kSvcSpec = 16 * kSvcBlock;  // input bytes read together with the request line
// mb: the answer side (served, done, refused, stamps; host-coherent); rb: the
// request side (doorbell, req): device memory the host maps (a large BAR) or
// mb itself; in: the service's own input buffer (kSmallSeg bytes, beside rb)
hipError_t launch_small_service(SmallMailbox* mb, const SmallMailbox* rb, const uint8_t* in, uint64_t idle_ticks,
                                uint64_t life_ticks, hipStream_t s);
// Clock probe of the leaf kernels on the current device (NKV_TIMING_CLOCK):
// p = kClockWords u64 (8 slots of 32: shader-clock cycles, 100 MHz ticks, waves;
// zeroed by the caller) or nullptr to switch it off.
constexpr uint32_t kClockWords = 8 * 32;
hipError_t set_clock_probe(unsigned long long* p, hipStream_t s);
// out[0] / out[1] = min / max of len[i] / 64 over the batch (2 u32 on the
// device); part: scratch of locate_part_words(n) u32
// ticket: one device u32, zero before the first launch (each launch leaves it zero)
hipError_t launch_len_range(const uint64_t* len, uint64_t n, unsigned int* out, uint32_t* part, unsigned int* ticket,
                            hipStream_t s);

}  // namespace nkv
