// context.hpp -- the nkv_ctx definition and the host helpers shared by the
// C-ABI translation units (capi.cpp: single-device entries; group.cpp: the
// multi-GPU group and the multi-table entries).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <new>
#include <vector>

#include "host_stage.hpp"
#include "internal.hpp"
#include "nkv_merkle.h"

namespace nkv {

// ---------------------------------------------------------------------------
// tree shape (merkletree.go:31-64): n_0 = n, n_{L+1} = ceil(n_L / 2), until a
// level of one node that is not the leaf level.

inline int levels_of(uint64_t n) {
    if (n == 0) return 0;
    int lv = 1;
    uint64_t c = n;
    do {
        c = (c + 1) / 2;
        ++lv;
    } while (c > 1);
    return lv;
}

inline uint64_t count_of(uint64_t n, int L) { return L == 0 ? n : ((n - 1) >> L) + 1; }

inline uint64_t start_of(uint64_t n, int L) {
    uint64_t s = 0;
    for (int j = 0; j < L; ++j) s += count_of(n, j);
    return s;
}

inline uint64_t total_of(uint64_t n) { return start_of(n, levels_of(n)); }

// Image layout (merkletree.go:67-92) of levels given bottom-up counts[0..nlev)
// of 20-byte nodes stored level-major from node index 0: top level first, 21
// bytes per node, one 0x01 pad byte after every odd level below the top.
inline BfsLayout layout_of(const std::vector<uint64_t>& counts) {
    BfsLayout lay{};
    const int nlev = int(counts.size());
    lay.nlev = nlev;
    std::vector<uint64_t> start(nlev);
    uint64_t s = 0;
    for (int L = 0; L < nlev; ++L) {
        start[L] = s;
        s += counts[L];
    }
    uint64_t p = 0;
    for (int i = 0; i < nlev; ++i) {  // image order: top first
        const int L = nlev - 1 - i;
        lay.img_start[i] = p;
        lay.node_start[i] = start[L];
        lay.count[i] = counts[L];
        p += 21 * counts[L];
        if (L < nlev - 1 && (counts[L] & 1)) p += 1;
    }
    lay.total = p;
    return lay;
}

inline std::vector<uint64_t> counts_of(uint64_t n) {
    std::vector<uint64_t> c(levels_of(n));
    for (size_t L = 0; L < c.size(); ++L) c[L] = count_of(n, int(L));
    return c;
}

// ---------------------------------------------------------------------------
// status helpers

inline int st(hipError_t e) {
    if (e == hipSuccess) return NKV_OK;
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return NKV_ERR_NOMEM;
    return NKV_ERR_DEVICE;
}

// NKV_DEBUG=1 in the environment: every failing HIP call behind HIPTRY is
// named on stderr (the status code alone does not say which call failed)
inline bool debug_on() {
    static const bool on = [] {
        const char* e = getenv("NKV_DEBUG");
        return e && *e && *e != '0';
    }();
    return on;
}
inline int st_at(hipError_t e, const char* what, const char* file, int line) {
    if (e != hipSuccess && debug_on())
        fprintf(stderr, "nkv: %s:%d: %s -> %s\n", file, line, what, hipGetErrorString(e));
    return st(e);
}

#define TRY(x)                         \
    do {                               \
        int _rc = (x);                 \
        if (_rc != NKV_OK) return _rc; \
    } while (0)
#define HIPTRY(x) TRY(::nkv::st_at((x), #x, __FILE__, __LINE__))
// Every C-ABI entry is a function-try-block: a host allocation or thread start
// that throws inside the library becomes a status code, never an exception
// crossing the C boundary (cgo / ctypes callers cannot catch it).
#define NKV_CATCH                      \
    catch (const std::bad_alloc&) {    \
        return NKV_ERR_NOMEM;          \
    }                                  \
    catch (...) {                      \
        return NKV_ERR_DEVICE;         \
    }

// Largest batch: leaf indices are 32-bit in the sort and queue kernels
// (2^31 - 1 values of 4 KiB would be 8 TiB, far beyond one GPU's HBM).
constexpr uint64_t kMaxN = 0x7fffffffull;

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

// Grow a device scratch buffer (contents are not kept).
int grow(DevBuf& b, size_t bytes);

}  // namespace nkv

// ---------------------------------------------------------------------------
// context

struct nkv_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    int leaf_load = 4;  // NKV_OPT_LEAF_LOAD
    int bucket = 2;     // NKV_OPT_BUCKET
    uint32_t simds = 1024;  // SIMDs on the device (CUs x 4)
    int queue_split = 32;   // NKV_OPT_QUEUE_SPLIT
    int queue_waves = 3;    // NKV_OPT_QUEUE_WAVES
    int bloom_path = 2;     // NKV_OPT_BLOOM_PATH
    int crc_load = 0;       // NKV_OPT_CRC_LOAD
    int records_fused = 1;  // NKV_OPT_RECORDS_FUSED
    int table_lanes = 2;    // NKV_OPT_TABLE_LANES
    bool timing = false;
    bool timed = false;
    // NKV_OPT_TIMING_EVERY: the tree calls record their events on every k-th
    // call only (counted from nkv_ctx_set_timing); sampled: the current call
    int timing_every = 1;
    uint64_t timing_calls = 0;
    bool sampled = true;
    // per-call event triples (leaf start, leaf end / reduce start, reduce end),
    // the latest kTimingRing / 3 calls
    static constexpr size_t kTimingRing = 3 * 65536;
    std::vector<hipEvent_t> ring;
    size_t ring_used = 0;
    hipEvent_t host_ev[2] = {nullptr, nullptr};  // host-buffer call: before the upload, after the download
    bool host_timed = false;
    nkv::DevBuf d_data, d_off, d_len, d_nodes, d_img, d_tmp, d_err, d_aux, d_keys, d_perm, d_stmp, d_queue,
        d_stats, d_range, d_part, d_tmp2, d_flags, d_clk,
        d_ticket;  // k_len_range's ticket (zeroed when allocated; each launch leaves it zero)
    int flag_set = 0;  // which of the two pass-flag sets in d_flags the next records call uses
    // the length sort's bucket totals may be non-zero (a sort was cut short):
    // the next sort clears them first (internal.hpp sort_head_words)
    bool sort_dirty = false;
    void* h_stage = nullptr;  // small pinned staging (offsets, lengths, stats)
    unsigned int* h_small = nullptr;  // 64 pinned bytes for device-to-host decisions
    size_t h_cap = 0;
    nkv::Stager stage;  // pipelined pinned staging of bulk bytes (host_stage.hpp)
    // stream hand-over (nkv_ctx_set_stream): the new stream waits for the old
    hipEvent_t switch_ev = nullptr;
    // multi-table entries (nkv_trees_dev): sub-contexts of the same device with
    // their own streams, forked from and joined to this context's stream
    std::vector<nkv_ctx*> lanes;
    hipEvent_t fork_ev = nullptr;
    std::vector<hipEvent_t> join_ev;
    bool clock_probe = false;  // NKV_TIMING_CLOCK: leaf kernels add their waves' clocks into d_clk
    // pinned blocks from nkv_host_alloc (the deferred-NewLeaf arena): calls whose
    // values lie inside one are copied straight from it (no staging gather), and
    // nkv_host_stream copies a block's settled prefix ahead of the call
    struct Pinned {
        uint8_t* p;
        uint64_t bytes;
        uint64_t streamed;  // bytes [0, streamed) already queued to d_arena
        nkv::DevBuf d_arena;  // device mirror of the block
        bool coherent;        // host-coherent (the small-tree kernel may read it in place)
    };
    std::vector<Pinned*> pinned;
    // the one-launch small-tree path of the host-buffer calls (NKV_OPT_SMALL_*):
    // host-coherent pinned in / out buffers the kernel reads and writes across
    // PCIe (or device copies of them, small_path 2), and its device scratch
    // (the ticket word + 20 n leaf digests)
    // NKV_OPT_SIDE_GATE: the gated plan's input-order kernel on a second stream
    // (created on first use), forked after the range and joined before the levels
    int side_gate = 1;
    hipStream_t side = nullptr;
    hipEvent_t side_ev[2] = {nullptr, nullptr};
    int arena_coherent = 1;  // NKV_OPT_ARENA_COHERENT: nkv_host_alloc blocks host-coherent
    int small_path = 1;
    uint64_t small_max_n = 1024;
    uint64_t small_max_bytes = uint64_t(1) << 20;
    uint8_t* h_sin = nullptr;
    uint8_t* h_sout = nullptr;
    size_t h_sin_cap = 0, h_sout_cap = 0;
    nkv::DevBuf d_sin, d_sout, d_small;
    int last_path = 0;  // NKV_PATH_* of the latest host-buffer tree call
    uint32_t small_seq = 0;  // the small-tree kernel's completion word (per call)
    // NKV_OPT_SMALL_PATH 3: the resident service's mailbox and stream (created
    // on first use; the kernel leaves after kSvcIdleUs without a request or at
    // nkv_ctx_destroy)
    nkv::SmallMailbox* h_mbox = nullptr;
    uint8_t* h_svc_in = nullptr;  // host packing buffer of an inline request (kSmallSeg bytes, host-coherent)
    // NKV_OPT_SERVICE_MAILBOX 0 on a large-BAR GPU: the request side (doorbell,
    // request line) and the service's input buffer in fine-grained device memory
    // the host stores to directly (one block: the mailbox, then kSmallSeg bytes)
    uint8_t* d_svc_box = nullptr;
    int svc_mailbox = 0;      // NKV_OPT_SERVICE_MAILBOX
    // the one-launch path's packed input in fine-grained device memory the host
    // stores to (kSmallSeg bytes; NKV_OPT_SERVICE_MAILBOX 0 on a large-BAR GPU)
    uint8_t* d_sin_bar = nullptr;
    bool sin_bar_tried = false;
    bool svc_box_dev = false; // the live buffers are d_svc_box's (else h_mbox / h_svc_in)
    hipStream_t svc = nullptr;
    bool svc_live = false;   // a service launch was made and may still run
    bool svc_trace = false;  // nkv_ctx_small_service_trace: stamp each request's phases
    uint64_t svc_launches = 0;
};

namespace nkv {

int bind(nkv_ctx* c);
int grow_host(nkv_ctx* c, size_t bytes);
// Pack n host values into d_data at 16-byte aligned offsets and upload their
// offsets/lengths to d_off / d_len (or use the device mirror of the pinned
// block they lie in).  *d_base / *aligned: where the kernels read the values.
int stage_values(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                 const uint8_t** d_base, bool* aligned);
// Level 0 in the plan NKV_OPT_BUCKET picks (host_len: the lengths on the host, nullable)
int leaf_level(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
               bool aligned, uint8_t* nodes, const uint64_t* host_len);
int tree_from_device_values(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                            uint64_t n, bool aligned, uint8_t* nodes, const uint64_t* host_len = nullptr,
                            const unsigned int* dev_range = nullptr);
// After a tree call: image / nodes / root to the host (any nullable), then a sync.
int finish_tree(nkv_ctx* c, uint8_t* nodes, uint64_t n, uint8_t* root20, uint8_t* nodes_out, uint8_t* img_out);
// Record events around the leaf kernel and the reduce (which = 0, 1, 2).
int mark(nkv_ctx* c, int which);
// Events bracketing a host-buffer call (which = 0 before the upload, 1 after the download).
int host_mark(nkv_ctx* c, int which);

}  // namespace nkv
