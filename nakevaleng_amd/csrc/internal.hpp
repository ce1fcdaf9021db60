// internal.hpp -- launcher declarations shared by kernels.hip and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nkv {

constexpr int kBlock = 256;       // threads per workgroup = leaves per K1 block
constexpr int kFuseLevels = 8;    // log2(kBlock): levels one workgroup reduces in LDS
constexpr int kWaveLevels = 6;    // log2(64): levels the leaf kernel's waves reduce by shuffles
constexpr int kMaxLevels = 64;
#ifndef NKV_LEAF_WAVES
#define NKV_LEAF_WAVES 8
#endif
constexpr int kLeafWavesPerSimd = NKV_LEAF_WAVES;  // 8 waves/SIMD <=> <= 64 VGPRs

// BFS image layout in image order (index 0 = top level).
struct BfsLayout {
    int nlev;
    uint64_t total;
    uint64_t img_start[kMaxLevels];   // first image byte of the level
    uint64_t node_start[kMaxLevels];  // first node of the level in the nodes buffer
    uint64_t count[kMaxLevels];       // real nodes in the level
};

// load: leaf-kernel load path for aligned values (1 LDS-DMA, 2 direct, 3 direct
// non-temporal); unaligned values always take the register funnel (0).
hipError_t launch_leaf_strided(const uint8_t* base, uint64_t stride, uint64_t L, uint64_t n,
                               int top, bool fuse, int load, uint8_t* nodes, hipStream_t s);
hipError_t launch_leaf_offsets(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                               const uint32_t* perm, uint64_t n, int top, bool fuse, bool aligned,
                               int load, uint8_t* nodes, hipStream_t s, bool deep = true);
// Ragged batch through the work-queue leaf kernel (perm = length-sorted order,
// longest first); q must hold queue_words(n) u32; split = longest chain (full
// blocks) of a group the non-priority waves take when the longest chain bounds
// the batch.
uint64_t queue_words(uint64_t n);
hipError_t launch_leaf_queue(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                             const uint32_t* perm, uint64_t n, bool aligned, bool ring, uint32_t* q,
                             uint32_t simds, uint32_t waves_per_simd, uint32_t split, uint8_t* nodes,
                             hipStream_t s);
hipError_t launch_reduce(uint8_t* nodes, uint64_t n, int from_level, int top, hipStream_t s);
hipError_t launch_bfs_image(const uint8_t* nodes, const BfsLayout& lay, uint8_t* img,
                            hipStream_t s);
hipError_t launch_locate(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off,
                         uint64_t n, uint64_t* voff, uint64_t* vlen, unsigned int* err,
                         hipStream_t s);
hipError_t scan_exclusive_u64(const uint64_t* in, uint64_t* out, uint64_t n, void* tmp,
                              size_t* tmp_bytes, hipStream_t s);
// Two-phase (tmp == nullptr: size query).  The permutation lands in perm + n.
hipError_t sort_by_length_desc(const uint64_t* len, uint64_t n, uint32_t* keys, uint32_t* perm,
                               void* tmp, size_t* tmp_bytes, hipStream_t s);
// crc.hip: CRC-32/IEEE of byte spans / of records' Key ++ Value (stats: 3 x u64,
// initialised by the launcher).
// variant: NKV_OPT_CRC_LOAD (bit 0 LDS chunk ring; bits 1-2 table copies x
// workgroup size).
hipError_t launch_crc_spans(const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                            uint32_t* out, int variant, hipStream_t s);
hipError_t launch_record_crc(const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                             uint32_t* out, unsigned long long* stats, int variant, hipStream_t s);
// bloom.hip: mode 0 = keys at base + off[i], len[i]; 1 = keys of the records at
// base + off[i].  query: out[i] = all k bits set; else OR the bits in.
hipError_t launch_bloom(int mode, bool query, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                        uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0, uint32_t* bits,
                        uint8_t* out, unsigned int* err, hipStream_t s);
hipError_t launch_fill(uint8_t* buf, uint64_t nbytes, uint64_t seed, hipStream_t s);

}  // namespace nkv
