// capi.cpp -- host side of libnkvmerkle.so: contexts, staging, launches and
// the C-ABI declared in include/nkv_merkle.h.
//
// There is deliberately no CPU compute path here: every digest is produced by
// the gfx950 kernels in kernels.hip.  A missing/unusable device is reported as
// NKV_ERR_DEVICE.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <new>
#include <vector>

#include "context.hpp"

using namespace nkv;

namespace nkv {

int bind(nkv_ctx* c) {
    if (!c) return NKV_ERR_INVALID;
    return st(hipSetDevice(c->device));
}

int grow(DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return NKV_OK;
    const size_t old = b.cap;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t want = std::max(bytes, old + old / 2);
    if (hipMalloc(&b.p, want) != hipSuccess) {
        (void)hipGetLastError();
        if (hipMalloc(&b.p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            b.p = nullptr;
            return NKV_ERR_NOMEM;
        }
        want = bytes;
    }
    b.cap = want;
    return NKV_OK;
}

// This call's pass flags and the set its leaf kernel resets for the next call
// (internal.hpp kPassFlagWords); flip_pass_flags once that kernel is launched.
void pass_flags(nkv_ctx* c, uint32_t** cur, uint32_t** next) {
    uint32_t* f = static_cast<uint32_t*>(c->d_flags.p);
    *cur = f + kPassFlagWords * c->flag_set;
    *next = f + kPassFlagWords * (1 - c->flag_set);
}
void flip_pass_flags(nkv_ctx* c) { c->flag_set ^= 1; }

// scratch for k_locate's per-workgroup partials
int locate_parts(nkv_ctx* c, uint64_t n, uint32_t** part) {
    TRY(grow(c->d_part, 4 * locate_part_words(n)));
    *part = static_cast<uint32_t*>(c->d_part.p);
    return NKV_OK;
}

int grow_host(nkv_ctx* c, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (c->h_cap >= bytes) return NKV_OK;
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->h_cap = 0;
    if (hipHostMalloc(&c->h_stage, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        c->h_stage = nullptr;
        return NKV_ERR_NOMEM;
    }
    c->h_cap = bytes;
    return NKV_OK;
}

uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

// sum(rec_size) <= stream_len, checked term by term so a wrapped sum cannot pass
bool records_fit(const uint64_t* rec_size, uint64_t n, uint64_t stream_len) {
    uint64_t left = stream_len;
    for (uint64_t i = 0; i < n; ++i) {
        if (rec_size[i] > left) return false;
        left -= rec_size[i];
    }
    return true;
}

// The pinned block (nkv_host_alloc on this context) that holds every value
// base + off[i] .. + len[i], or null; *lo / *hi: the values' extent relative
// to the block.
nkv_ctx::Pinned* pinned_extent(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                               uint64_t n, uint64_t* lo, uint64_t* hi) {
    if (c->pinned.empty() || n == 0) return nullptr;
    uint64_t a = ~uint64_t(0), b = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (len[i] > (uint64_t(1) << 62) || off[i] > (uint64_t(1) << 62)) return nullptr;
        a = std::min(a, off[i]);
        b = std::max(b, off[i] + len[i]);
    }
    const uintptr_t s = reinterpret_cast<uintptr_t>(base) + a, e = reinterpret_cast<uintptr_t>(base) + b;
    if (e < s) return nullptr;
    for (nkv_ctx::Pinned* blk : c->pinned) {
        const uintptr_t p = reinterpret_cast<uintptr_t>(blk->p);
        if (s >= p && e <= p + blk->bytes) {
            *lo = s - p;
            *hi = e - p;
            return blk;
        }
    }
    return nullptr;
}

// Queue bytes [from, to) of a pinned block to its device mirror on the
// context's stream (the block is library-owned memory, so the DMA may outlive
// the call).
int stream_block(nkv_ctx* c, nkv_ctx::Pinned* blk, uint64_t from, uint64_t to) {
    if (to <= from) return NKV_OK;
    if (!blk->d_arena.p) TRY(grow(blk->d_arena, blk->bytes));
    HIPTRY(hipMemcpyAsync(static_cast<uint8_t*>(blk->d_arena.p) + from, blk->p + from, to - from,
                          hipMemcpyHostToDevice, c->stream));
    return NKV_OK;
}

// Move n host values to the device and upload their offsets/lengths to d_off /
// d_len; *d_base / *aligned tell the kernels where the values are.
//  - Values inside one pinned block of this context (the deferred-NewLeaf
//    arena, nkv_host_alloc): one DMA straight from the block into its device
//    mirror, minus the prefix nkv_host_stream already queued; offsets are the
//    values' places in the block (aligned iff all are 16-byte aligned).
//  - Anything else: packed at 16-byte aligned offsets through the pipelined
//    pinned stager (a pool of host threads gathers chunk k+1 while chunk k is
//    in flight).
// No caller pointer is kept either way.
int stage_values(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
                 const uint8_t** d_base, bool* aligned) {
    uint64_t lo = 0, hi = 0;
    if (nkv_ctx::Pinned* blk = pinned_extent(c, base, off, len, n, &lo, &hi)) {
        TRY(grow_host(c, 16 * n));
        TRY(grow(c->d_off, 8 * n));
        TRY(grow(c->d_len, 8 * n));
        uint64_t* hoff = static_cast<uint64_t*>(c->h_stage);
        uint64_t* hlen = hoff + n;
        const uint64_t adj = uint64_t(base - blk->p);
        uint64_t ormask = 0;
        for (uint64_t i = 0; i < n; ++i) {
            hoff[i] = adj + off[i];
            hlen[i] = len[i];
            ormask |= hoff[i];
        }
        // the prefix nkv_host_stream queued is already on its way; the rest now
        TRY(stream_block(c, blk, std::max(lo, blk->streamed), hi));
        blk->streamed = 0;  // this call consumes the batch: a new one streams from 0
        HIPTRY(hipMemcpyAsync(c->d_off.p, hoff, 8 * n, hipMemcpyHostToDevice, c->stream));
        HIPTRY(hipMemcpyAsync(c->d_len.p, hlen, 8 * n, hipMemcpyHostToDevice, c->stream));
        *d_base = static_cast<const uint8_t*>(blk->d_arena.p);
        *aligned = (ormask & 15) == 0;
        return NKV_OK;
    }
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (len[i] > (uint64_t(1) << 62) || total > (uint64_t(1) << 62)) return NKV_ERR_INVALID;
        total += align16(len[i]);
    }
    *d_base = nullptr;
    *aligned = true;
    TRY(grow_host(c, 16 * n));
    TRY(grow(c->d_data, total));
    TRY(grow(c->d_off, 8 * n));
    TRY(grow(c->d_len, 8 * n));
    uint64_t* hoff = static_cast<uint64_t*>(c->h_stage);
    uint64_t* hlen = hoff + n;
    uint64_t p = 0;
    for (uint64_t i = 0; i < n; ++i) {
        hoff[i] = p;
        hlen[i] = len[i];
        p += align16(len[i]);
    }
    const Segments seg{base, off, len, hoff, n};
    HIPTRY(c->stage.upload(seg, total, static_cast<uint8_t*>(c->d_data.p), c->stream));
    HIPTRY(hipMemcpyAsync(c->d_off.p, hoff, 8 * n, hipMemcpyHostToDevice, c->stream));
    HIPTRY(hipMemcpyAsync(c->d_len.p, hlen, 8 * n, hipMemcpyHostToDevice, c->stream));
    *d_base = static_cast<const uint8_t*>(c->d_data.p);
    return NKV_OK;
}

// Contiguous host bytes -> d (bulk path) plus n u64 -> d64 (through h_stage).
int stage_stream(nkv_ctx* c, const uint8_t* src, uint64_t bytes, DevBuf& d, const uint64_t* v64,
                 uint64_t n, DevBuf& d64) {
    TRY(grow(d, bytes));
    TRY(grow(d64, 8 * n));
    TRY(grow_host(c, 8 * n));
    HIPTRY(c->stage.upload(src, bytes, static_cast<uint8_t*>(d.p), c->stream));
    memcpy(c->h_stage, v64, 8 * n);
    HIPTRY(hipMemcpyAsync(d64.p, c->h_stage, 8 * n, hipMemcpyHostToDevice, c->stream));
    return NKV_OK;
}

// A host-coherent pinned buffer of at least `bytes` (contents not kept): the
// small-tree kernel reads / writes it across PCIe, uncached on the GPU side.
int grow_coherent(uint8_t** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return NKV_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t want = std::max(bytes, size_t(64) << 10);
    if (hipHostMalloc(reinterpret_cast<void**>(p), want, hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return NKV_ERR_NOMEM;
    }
    *cap = want;
    return NKV_OK;
}

// The reference engine's own flush and compaction sizes (coreconf.go:33-34,
// :39: 10-record memtables, 4 runs) hash a few KiB per call, where the grid
// path's copies and per-level launches cost far more than the work.  A batch
// of at most small_max_n values and small_max_bytes of (16-byte aligned)
// payload instead goes as ONE launch (k_small_tree): the values are packed into
// a host-coherent pinned buffer that the kernel reads across PCIe
// (NKV_OPT_SMALL_PATH 1) or that is copied to HBM first (2), the kernel writes
// nodes + image into a pinned output buffer (or HBM, then one copy back), and
// the call synchronizes once.  *taken = false: not eligible, nothing done.
constexpr uint64_t kSmallMaxExtent = 0xFFFFFFF0ull;  // the kernel's 32-bit extent of in-place values
constexpr int64_t kSmallSpinUs = 2000;  // host spin on the completion word before the runtime's wait
constexpr uint64_t kSvcIdleUs = 20000;   // the resident service leaves after this long without a request
constexpr uint64_t kSvcLifeUs = 200000;  // ... or, between requests, once it has run this long
constexpr int64_t kSvcTimeoutUs = 10000000;  // a request unanswered this long (service alive) is an error

// Device memory the host may store to directly: fine-grained memory of a
// large-BAR GPU is mapped into the host's address space at the address the GPU
// uses (tools/bar_probe.hip on MI355X: hostBaseAddress == the pointer, host
// stores and loads work, no grant needed).
bool host_mapped(const void* p) {
    hsa_amd_pointer_info_t info;
    memset(&info, 0, sizeof info);
    info.size = sizeof info;
    if (hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
    return info.hostBaseAddress == p;
}

// Host stores to device memory through the BAR may be write-combined: drained
// before the doorbell (the request's bytes land first: PCIe keeps posted writes
// in order) and after it (so it leaves now, not when the buffer fills).
inline void store_fence() { asm volatile("sfence" ::: "memory"); }

// The service's mailbox, its input buffer and its stream (created on first
// use, and again after svc_stop).  The answer side (served, done, refused,
// stamps) is host-coherent memory, where the host spins.  The request side
// (doorbell, request line) and the service's input buffer go, with
// NKV_OPT_SERVICE_MAILBOX 0 on a large-BAR GPU, to fine-grained device memory
// the host stores to: the service then polls and reads local memory instead of
// crossing PCIe for each poll and for the input (tools/bar_probe.hip: a 4 KiB
// request's round trip 7.7 -> 5.8 us); otherwise they share the host mailbox.
int svc_buffers(nkv_ctx* c) {
    if (!c->h_mbox) {
        uint8_t* p = nullptr;
        size_t cap = 0;
        TRY(grow_coherent(&p, &cap, sizeof(SmallMailbox)));
        memset(p, 0, sizeof(SmallMailbox));
        c->h_mbox = reinterpret_cast<SmallMailbox*>(p);
        c->svc_box_dev = false;
        int large = 0;
        void* d = nullptr;
        if (c->svc_mailbox == 0 && hipDeviceGetAttribute(&large, hipDeviceAttributeIsLargeBar, c->device) == hipSuccess &&
            large && hipExtMallocWithFlags(&d, sizeof(SmallMailbox) + kSmallSeg, hipDeviceMallocFinegrained) == hipSuccess) {
            if (host_mapped(d)) {
                memset(d, 0, sizeof(SmallMailbox));  // doorbell 0 == served 0
                store_fence();
                c->d_svc_box = static_cast<uint8_t*>(d);
                c->svc_box_dev = true;
            } else {
                (void)hipFree(d);
            }
        }
        (void)hipGetLastError();
    }
    if (!c->h_svc_in) {
        size_t cap = 0;
        TRY(grow_coherent(&c->h_svc_in, &cap, kSmallSeg));
    }
    if (!c->svc) HIPTRY(hipStreamCreateWithFlags(&c->svc, hipStreamNonBlocking));
    return NKV_OK;
}

// The one-launch path's input buffer in device memory the host stores to
// (made once, on a large-BAR GPU with NKV_OPT_SERVICE_MAILBOX 0), or nullptr:
// a packed input of at most kSmallSeg bytes is copied there, so the kernel
// stages it from local memory instead of across PCIe.
uint8_t* small_input_bar(nkv_ctx* c) {
    if (c->svc_mailbox != 0) return nullptr;
    if (!c->d_sin_bar && !c->sin_bar_tried) {
        c->sin_bar_tried = true;
        int large = 0;
        void* d = nullptr;
        if (hipDeviceGetAttribute(&large, hipDeviceAttributeIsLargeBar, c->device) == hipSuccess && large &&
            hipExtMallocWithFlags(&d, kSmallSeg, hipDeviceMallocFinegrained) == hipSuccess) {
            if (host_mapped(d))
                c->d_sin_bar = static_cast<uint8_t*>(d);
            else
                (void)hipFree(d);
        }
        (void)hipGetLastError();
    }
    return c->d_sin_bar;
}

// The request side as the host stores to it (the device's address too).
SmallMailbox* svc_request_side(nkv_ctx* c) {
    return c->svc_box_dev ? reinterpret_cast<SmallMailbox*>(c->d_svc_box) : c->h_mbox;
}

// One request to the resident service: an inline request's packed input
// (descriptors + values at h_svc_in, in_bytes) moved to the device buffer when
// that is where the service reads it, the request line, then the doorbell
// (release: x86 keeps the stores in order; the fences drain a write-combined
// mapping; the service reads them after its system-scope acquire), then a
// spin on `done`.  Each 256 polls look at the service stream: a service that
// has left is started again.
int small_service_call(nkv_ctx* c, const uint64_t* d_desc, const uint8_t* d_vals, uint32_t vbytes, uint32_t n,
                       uint8_t* d_out, uint32_t img_at, uint32_t seq, bool inline_in) {
    TRY(svc_buffers(c));
    SmallMailbox* mb = c->h_mbox;
    SmallMailbox* rb = svc_request_side(c);
    void *dmb = nullptr, *din = nullptr;
    HIPTRY(hipHostGetDevicePointer(&dmb, mb, 0));
    const SmallMailbox* drb = c->svc_box_dev ? rb : static_cast<const SmallMailbox*>(dmb);
    if (c->svc_box_dev) {
        din = c->d_svc_box + sizeof(SmallMailbox);
        if (inline_in) {
            memcpy(din, c->h_svc_in, 16 * size_t(n) + vbytes);
            d_desc = static_cast<const uint64_t*>(din);
            d_vals = static_cast<const uint8_t*>(din) + 16 * size_t(n);
        }
    } else {
        HIPTRY(hipHostGetDevicePointer(&din, c->h_svc_in, 0));
    }
    const uint8_t* fixed_in = static_cast<const uint8_t*>(din);
    SmallRequest r;
    memset(&r, 0, sizeof r);
    r.n = n;
    r.vbytes = vbytes;
    r.img_at = img_at;
    r.trace = c->svc_trace ? 1u : 0u;
    r.desc = reinterpret_cast<uintptr_t>(d_desc);
    r.vals = reinterpret_cast<uintptr_t>(d_vals);
    r.out = reinterpret_cast<uintptr_t>(d_out);
    r.inline_in = inline_in ? 1u : 0u;
    memcpy(&rb->req, &r, sizeof r);
    if (c->svc_box_dev) store_fence();
    __atomic_store_n(&rb->doorbell, seq, __ATOMIC_RELEASE);
    if (c->svc_box_dev) store_fence();
    if (!c->svc_live) {
        HIPTRY(launch_small_service(static_cast<SmallMailbox*>(dmb), drb, fixed_in, kSvcIdleUs * 100, kSvcLifeUs * 100,
                                    c->svc));
        c->svc_live = true;
        ++c->svc_launches;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 1;; ++k) {
        if (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) == seq) {
            if (__atomic_load_n(&mb->refused, __ATOMIC_ACQUIRE) == seq) return NKV_ERR_DEVICE;
            break;
        }
        if ((k & 255u) == 0u) {
            const hipError_t q = hipStreamQuery(c->svc);
            if (q == hipSuccess) {  // the service has left (idle): start it again, unless it answered
                if (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) == seq) {
                    if (__atomic_load_n(&mb->refused, __ATOMIC_ACQUIRE) == seq) return NKV_ERR_DEVICE;
                    break;
                }
                HIPTRY(launch_small_service(static_cast<SmallMailbox*>(dmb), drb, fixed_in, kSvcIdleUs * 100,
                                            kSvcLifeUs * 100, c->svc));
                ++c->svc_launches;
            } else if (q != hipErrorNotReady) {
                return st_at(q, "k_small_service", __FILE__, __LINE__);
            } else if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSvcTimeoutUs)) {
                return NKV_ERR_DEVICE;
            }
        }
        __builtin_ia32_pause();
    }
    return NKV_OK;
}

// Stop the resident service (nkv_ctx_destroy, a change of
// NKV_OPT_SERVICE_MAILBOX): the exit doorbell, then wait for the kernel to
// leave; its buffers are made again on the next request.
void svc_stop(nkv_ctx* c) {
    if (c->svc_live && c->h_mbox) {
        SmallMailbox* rb = svc_request_side(c);
        __atomic_store_n(&rb->doorbell, kSvcExit, __ATOMIC_RELEASE);
        if (c->svc_box_dev) store_fence();
        // the service leaves at its next poll (or its idle timeout); never wait
        // unboundedly in a destructor: a service that has not left after 2 s
        // keeps its mailbox and stream (leaked) rather than hang the caller
        const auto t0 = std::chrono::steady_clock::now();
        while (hipStreamQuery(c->svc) == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                if (debug_on()) fprintf(stderr, "nkv: the small-tree service did not leave; mailbox leaked\n");
                c->svc_live = false;
                c->svc = nullptr;
                c->h_mbox = nullptr;
                c->h_svc_in = nullptr;
                c->d_svc_box = nullptr;
                c->svc_box_dev = false;
                return;
            }
            usleep(50);
        }
    }
    c->svc_live = false;
    if (c->svc) (void)hipStreamDestroy(c->svc);
    c->svc = nullptr;
    if (c->h_mbox) (void)hipHostFree(c->h_mbox);
    c->h_mbox = nullptr;
    if (c->h_svc_in) (void)hipHostFree(c->h_svc_in);
    c->h_svc_in = nullptr;
    if (c->d_svc_box) (void)hipFree(c->d_svc_box);
    c->d_svc_box = nullptr;
    c->svc_box_dev = false;
}
int small_tree(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
               uint8_t* root20, uint8_t* nodes_out, uint8_t* img_out, bool* taken) {
    *taken = false;
    if (c->small_path == 0 || n == 0 || n > c->small_max_n || n > kSmallMaxN) return NKV_OK;
    uint64_t vbytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (len[i] > c->small_max_bytes) return NKV_OK;
        vbytes += align16(len[i]);
        if (vbytes > c->small_max_bytes) return NKV_OK;
    }
    const uint64_t tot = total_of(n);
    const uint64_t img_len = layout_of(counts_of(n)).total;
    // img_at 0 tells the kernel to build no image: a caller that asked for none
    // (the mirrors' New, whose Serialize walks the live tree) pays none
    const uint64_t img_at = img_out ? align16(20 * tot) : 0;
    const uint64_t out_bytes = img_out ? img_at + align16(img_len) : align16(20 * tot);
    uint64_t lo = 0, hi = 0;
    nkv_ctx::Pinned* blk = pinned_extent(c, base, off, len, n, &lo, &hi);
    if (blk) blk->streamed = 0;  // a call over a pinned block ends its batch (nkv_host_stream)
    // values in a host-coherent arena block at 16-byte aligned places (the
    // mirrors' NewLeaf arena) are read where they lie: no pack, no copy
    // (only while their extent in the block, gaps included, stays within the
    // small bound: the kernel takes the extent as a 32-bit byte count)
    bool in_place = blk && blk->coherent && c->small_path != 2 && (lo & 15) == 0 &&
                    align16(hi) - lo <= std::min<uint64_t>(c->small_max_bytes, kSmallMaxExtent);
    const uint64_t adj = blk ? uint64_t(base - blk->p) : 0;
    for (uint64_t i = 0; in_place && i < n; ++i) in_place = ((adj + off[i]) & 15) == 0;
    // the resident service: a request whose descriptors and values fit its own
    // input buffer is packed there (a host copy of at most 16 KiB), so the
    // service reads it with the request line instead of one round trip later,
    // values in the arena included
    const bool svc = c->small_path == 3 && n <= kSvcMaxN;
    const bool svc_inline = svc && 16 * n + vbytes <= kSmallSeg;
    if (svc_inline) {
        in_place = false;
        TRY(svc_buffers(c));
    }
    // likewise the one-launch path (1): an input that fits 16 KiB is packed and
    // stored into BAR-mapped device memory (small_input_bar), arena values
    // included, rather than read across PCIe where it lies
    uint8_t* const bar = !svc && c->small_path == 1 && 16 * n + vbytes <= kSmallSeg ? small_input_bar(c) : nullptr;
    if (bar) in_place = false;
    const uint64_t vext = in_place ? align16(hi) - lo : vbytes;  // the values' extent
    const uint64_t in_bytes = 16 * n + (in_place ? 0 : vbytes);
    if (!svc_inline) TRY(grow_coherent(&c->h_sin, &c->h_sin_cap, in_bytes));
    uint8_t* const h_in = svc_inline ? c->h_svc_in : c->h_sin;
    TRY(grow_coherent(&c->h_sout, &c->h_sout_cap, out_bytes + 64));  // + the completion word
    const size_t small_cap = c->d_small.cap;
    TRY(grow(c->d_small, 64 + 20 * kSmallMaxN));
    if (c->d_small.cap != small_cap) HIPTRY(hipMemsetAsync(c->d_small.p, 0, 64, c->stream));  // the ticket
    uint64_t* desc = reinterpret_cast<uint64_t*>(h_in);
    if (in_place) {
        for (uint64_t i = 0; i < n; ++i) {
            desc[2 * i] = adj + off[i] - lo;
            desc[2 * i + 1] = len[i];
        }
    } else {
        uint8_t* vals = h_in + 16 * n;
        uint64_t p = 0;
        for (uint64_t i = 0; i < n; ++i) {
            desc[2 * i] = p;
            desc[2 * i + 1] = len[i];
            if (len[i]) memcpy(vals + p, base + off[i], len[i]);
            p += align16(len[i]);
        }
    }
    uint8_t* scratch = static_cast<uint8_t*>(c->d_small.p) + 64;
    unsigned int* ticket = static_cast<unsigned int*>(c->d_small.p);
    volatile unsigned int* hdone = reinterpret_cast<volatile unsigned int*>(c->h_sout + out_bytes);
    uint32_t seq = ++c->small_seq;
    if (seq == 0 || seq == kSvcExit) seq = c->small_seq = 1;  // 0 is the word's cleared state
    *hdone = 0;
    if (svc) {  // the resident service: no launch, no runtime completion
        void *din = nullptr, *dout = nullptr, *dblk = nullptr;
        HIPTRY(hipHostGetDevicePointer(&din, h_in, 0));
        HIPTRY(hipHostGetDevicePointer(&dout, c->h_sout, 0));
        if (in_place) HIPTRY(hipHostGetDevicePointer(&dblk, blk->p, 0));
        const uint8_t* d_vals = in_place ? static_cast<const uint8_t*>(dblk) + lo
                                         : static_cast<const uint8_t*>(din) + 16 * n;
        TRY(small_service_call(c, static_cast<const uint64_t*>(din), d_vals, uint32_t(vext), uint32_t(n),
                               static_cast<uint8_t*>(dout), uint32_t(img_at), seq, svc_inline));
    } else if (c->small_path == 2) {  // through HBM: one copy in, one launch, one copy out
        TRY(grow(c->d_sin, in_bytes));
        TRY(grow(c->d_sout, out_bytes));
        HIPTRY(hipMemcpyAsync(c->d_sin.p, c->h_sin, in_bytes, hipMemcpyHostToDevice, c->stream));
        const uint64_t* d_desc = static_cast<const uint64_t*>(c->d_sin.p);
        HIPTRY(launch_small_tree(d_desc, reinterpret_cast<const uint8_t*>(d_desc + 2 * n), uint32_t(vext),
                                 uint32_t(n), static_cast<uint8_t*>(c->d_sout.p), uint32_t(img_at), scratch, ticket,
                                 nullptr, 0, c->stream));
        HIPTRY(hipMemcpyAsync(c->h_sout, c->d_sout.p, out_bytes, hipMemcpyDeviceToHost, c->stream));
        HIPTRY(hipStreamSynchronize(c->stream));
    } else {  // the kernel reads the values and writes its results across PCIe
        void *din = nullptr, *dout = nullptr, *dblk = nullptr;
        HIPTRY(hipHostGetDevicePointer(&din, c->h_sin, 0));
        HIPTRY(hipHostGetDevicePointer(&dout, c->h_sout, 0));
        if (in_place) HIPTRY(hipHostGetDevicePointer(&dblk, blk->p, 0));
        const uint64_t* d_desc = static_cast<const uint64_t*>(din);
        const uint8_t* d_vals = in_place ? static_cast<const uint8_t*>(dblk) + lo
                                         : reinterpret_cast<const uint8_t*>(d_desc + 2 * n);
        // a packed input that fits the kernel's LDS stage goes to device memory
        // over the large BAR (posted writes: they land before the launch's
        // doorbell), so the kernel stages it without a PCIe read round trip
        if (bar) {
            memcpy(bar, c->h_sin, in_bytes);
            store_fence();
            d_desc = reinterpret_cast<const uint64_t*>(bar);
            d_vals = bar + 16 * n;
        }
        HIPTRY(launch_small_tree(d_desc, d_vals, uint32_t(vext), uint32_t(n), static_cast<uint8_t*>(dout),
                                 uint32_t(img_at), scratch, ticket,
                                 reinterpret_cast<unsigned int*>(static_cast<uint8_t*>(dout) + out_bytes), seq,
                                 c->stream));
        // the kernel's last store is seq into the completion word, after every
        // output byte: spin on it (a few us sooner than the runtime's
        // completion wait); every 256 polls ask the stream whether it failed.
        // The spin is bounded (kSmallSpinUs): a kernel queued behind other work
        // on a caller's stream is waited for by the runtime instead, so no
        // host core spins for the length of someone else's queue.
        const auto t_spin = std::chrono::steady_clock::now();
        for (uint32_t k = 1;; ++k) {
            if (__atomic_load_n(hdone, __ATOMIC_ACQUIRE) == seq) break;
            if ((k & 255u) == 0u) {
                const hipError_t q = hipStreamQuery(c->stream);
                if (q == hipSuccess) {  // finished: the word is there now
                    if (__atomic_load_n(hdone, __ATOMIC_ACQUIRE) != seq) return NKV_ERR_DEVICE;
                    break;
                }
                if (q != hipErrorNotReady) return st_at(q, "k_small_tree", __FILE__, __LINE__);
                if (std::chrono::steady_clock::now() - t_spin > std::chrono::microseconds(kSmallSpinUs)) {
                    HIPTRY(hipStreamSynchronize(c->stream));
                    if (__atomic_load_n(hdone, __ATOMIC_ACQUIRE) != seq) return NKV_ERR_DEVICE;
                    break;
                }
            }
            __builtin_ia32_pause();
        }
    }
    if (nodes_out) memcpy(nodes_out, c->h_sout, 20 * tot);
    if (root20) memcpy(root20, c->h_sout + 20 * (tot - 1), 20);
    if (img_out) memcpy(img_out, c->h_sout + img_at, img_len);
    c->last_path = NKV_PATH_SMALL;
    c->host_timed = false;
    *taken = true;
    return NKV_OK;
}

int finish_tree(nkv_ctx* c, uint8_t* nodes, uint64_t n, uint8_t* root20, uint8_t* nodes_out,
                uint8_t* img_out) {
    const uint64_t tot = total_of(n);
    if (img_out) {
        BfsLayout lay = layout_of(counts_of(n));
        TRY(grow(c->d_img, lay.total));
        HIPTRY(launch_bfs_image(nodes, lay, static_cast<uint8_t*>(c->d_img.p), c->stream));
        HIPTRY(c->stage.download(img_out, static_cast<const uint8_t*>(c->d_img.p), lay.total, c->stream));
    }
    if (nodes_out) HIPTRY(c->stage.download(nodes_out, nodes, 20 * tot, c->stream));
    if (root20)
        HIPTRY(hipMemcpyAsync(root20, nodes + 20 * (tot - 1), 20, hipMemcpyDeviceToHost, c->stream));
    HIPTRY(hipStreamSynchronize(c->stream));
    return NKV_OK;
}

// Events around the leaf kernel and the reduce of one tree call; kept per
// call (no host sync) so a timed loop can be summarised afterwards.
int mark(nkv_ctx* c, int which) {
    if (!c->timing) return NKV_OK;
    if (which == 0) c->sampled = c->timing_calls++ % uint64_t(c->timing_every) == 0;
    if (!c->sampled) return NKV_OK;
    if (which == 0) {
        if (c->ring_used + 3 > nkv_ctx::kTimingRing) c->ring_used = 0;  // restart the window
        if (c->ring_used + 3 > c->ring.size()) {
            for (int i = 0; i < 3; ++i) {
                hipEvent_t e;
                HIPTRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));  // timing only: no cache writeback per record
                c->ring.push_back(e);
            }
        }
        c->ring_used += 3;
    }
    // one event per mark: each record is a timestamp packet on the stream
    // (a few us of GPU time), so the timed loop carries three per tree
    HIPTRY(hipEventRecord(c->ring[c->ring_used - 3 + which], c->stream));
    if (which == 2) c->timed = true;
    return NKV_OK;
}

// Events around a host-buffer tree call (which = 0 before the upload, 1 after
// the outputs are back): with the three mark() events of the same call they
// split it into upload, kernels and download (nkv_ctx_last_host_timing).
int host_mark(nkv_ctx* c, int which) {
    if (!c->timing) return NKV_OK;
    // which 0 comes before the call's mark(0): the call is sampled when the
    // count it is about to take is
    const bool sampled = which == 0 ? c->timing_calls % uint64_t(c->timing_every) == 0 : c->sampled;
    if (!sampled) {
        c->host_timed = false;
        return NKV_OK;
    }
    if (!c->host_ev[which]) HIPTRY(hipEventCreate(&c->host_ev[which]));
    HIPTRY(hipEventRecord(c->host_ev[which], c->stream));
    if (which == 1) c->host_timed = c->timed;
    return NKV_OK;
}

// Order of a ragged batch for the leaf kernel (NKV_OPT_BUCKET): input order
// (no sort), length-sorted (work queue), or both kernels
// launched behind a device-side Gate.  Auto mode (2) sorts batches of fewer than
// 4096 values; for larger ones a narrow range of full-block counts
// (max <= min + max(1, min / 16), e.g. SSTable records of one size) gains
// nothing from sorting.  With the lengths on the host the choice is made here;
// with device lengths only, k_len_range measures the range and the two leaf
// kernels read it (no host read-back, so device-resident calls stay
// asynchronous; the sort then runs either way).
enum Plan { kInputOrder = 0, kSorted = 1, kGated = 2 };

// dev_range (nullable): the batch's range already on the device (k_locate wrote it)
int plan_of(nkv_ctx* c, const uint64_t* len, const uint64_t* host_len, uint64_t n, int* plan, Gate* gate,
            const unsigned int* dev_range = nullptr) {
    *plan = (c->bucket != 0 && n > 64) ? kSorted : kInputOrder;
    *gate = Gate{};
    if (c->bucket != 2 || n < 4096) return NKV_OK;
    if (host_len) {
        uint64_t lo = ~uint64_t(0), hi = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t b = host_len[i] >> 6;
            lo = std::min(lo, b);
            hi = std::max(hi, b);
        }
        *plan = hi <= lo + std::max<uint64_t>(1, lo / 16) ? kInputOrder : kSorted;
        return NKV_OK;
    }
    if (dev_range) {
        gate->range = dev_range;
        *plan = kGated;
        return NKV_OK;
    }
    TRY(grow(c->d_range, 8));
    unsigned int* d = static_cast<unsigned int*>(c->d_range.p);
    uint32_t* part = nullptr;
    TRY(locate_parts(c, n, &part));
    const size_t tcap = c->d_ticket.cap;
    TRY(grow(c->d_ticket, 16));
    if (c->d_ticket.cap != tcap) HIPTRY(hipMemsetAsync(c->d_ticket.p, 0, 16, c->stream));
    HIPTRY(launch_len_range(len, n, d, part, static_cast<unsigned int*>(c->d_ticket.p), c->stream));
    gate->range = d;
    *plan = kGated;
    return NKV_OK;
}

// The context's second stream and its fork / join events (NKV_OPT_SIDE_GATE).
int side_ready(nkv_ctx* c) {
    if (!c->side) HIPTRY(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    for (hipEvent_t& e : c->side_ev)
        if (!e) HIPTRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return NKV_OK;
}

// Level 0 in the order plan_of chose.  Gated plans also launch the input-order
// kernel (it runs when the range is narrow) unless the caller has its own
// (narrow_kernel = false: k_leaf_verify).
int leaf_level(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
               bool aligned, uint8_t* nodes, int plan, Gate range, bool narrow_kernel = true,
               CopyWords cw = CopyWords{}) {
    if (plan == kInputOrder && cw.n) return NKV_ERR_INVALID;  // the copy rides on the sort
    if (plan == kInputOrder) return st(launch_leaf_offsets(base, off, len, n, aligned, c->leaf_load, nodes, c->stream));
    if (n > 0x7fffffffull) return NKV_ERR_INVALID;
    const Gate wide{range.range, plan == kGated ? 2 : 0};
    const size_t keys_cap = c->d_keys.cap;
    TRY(grow(c->d_keys, 4 * sort_hist_words(n)));
    // (re)allocated scratch, or a sort cut short by an error: the sort's bucket
    // totals must start at zero (its last workgroup leaves them zero again)
    if (c->d_keys.cap != keys_cap || c->sort_dirty) {
        HIPTRY(hipMemsetAsync(c->d_keys.p, 0, 4 * sort_head_words(), c->stream));
        c->sort_dirty = false;
    }
    c->sort_dirty = true;  // until the sort and the kernels behind it are queued
    TRY(grow(c->d_perm, 4 * n));
    uint32_t* perm = static_cast<uint32_t*>(c->d_perm.p);
    TRY(grow(c->d_queue, 4 * queue_words(n)));
    const QueueInit qi{static_cast<uint32_t*>(c->d_queue.p), queue_words(n), uint32_t(c->queue_split)};
    // the gated input-order kernel writes level 0 only when the range is narrow,
    // the sort and the queue only when it is wide: on the side stream it runs
    // beside them, so the closed ones cost the batch no launch slot
    const bool narrow = plan == kGated && narrow_kernel;
    const bool forked = narrow && c->side_gate;
    if (forked) {
        TRY(side_ready(c));
        HIPTRY(hipEventRecord(c->side_ev[0], c->stream));
        HIPTRY(hipStreamWaitEvent(c->side, c->side_ev[0], 0));
        HIPTRY(launch_leaf_offsets(base, off, len, n, aligned, c->leaf_load, nodes, c->side, Gate{range.range, 1}));
        HIPTRY(hipEventRecord(c->side_ev[1], c->side));
    }
    int rc = st(sort_by_length_desc(len, n, perm, static_cast<uint32_t*>(c->d_keys.p), c->stream, wide, qi, cw));
    if (rc == NKV_OK)
        rc = st(launch_leaf_queue(base, off, len, perm, n, static_cast<uint32_t*>(c->d_queue.p), c->simds,
                                  uint32_t(c->queue_waves), nodes, c->stream, wide));
    if (forked) {  // joined whatever happened above: nothing on the stream may pass it
        const int j = st(hipStreamWaitEvent(c->stream, c->side_ev[1], 0));
        if (rc == NKV_OK) rc = j;
    } else if (rc == NKV_OK && narrow) {
        rc = st(launch_leaf_offsets(base, off, len, n, aligned, c->leaf_load, nodes, c->stream, Gate{range.range, 1}));
    }
    TRY(rc);
    c->sort_dirty = false;
    return NKV_OK;
}

int leaf_level(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, uint64_t n,
               bool aligned, uint8_t* nodes, const uint64_t* host_len) {
    int plan = kInputOrder;
    Gate g;
    TRY(plan_of(c, len, host_len, n, &plan, &g));
    return leaf_level(c, base, off, len, n, aligned, nodes, plan, g);
}

// host_len (nullable): the value lengths on the host, when the caller has them.
// Every order leaves level 0 complete, so one reduce sequence follows.
int tree_from_device_values(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                            uint64_t n, bool aligned, uint8_t* nodes, const uint64_t* host_len,
                            const unsigned int* dev_range) {
    int plan = kInputOrder;
    Gate g;
    TRY(plan_of(c, len, host_len, n, &plan, &g, dev_range));
    TRY(mark(c, 0));
    TRY(leaf_level(c, base, off, len, n, aligned, nodes, plan, g));
    TRY(mark(c, 1));
    HIPTRY(launch_reduce(nodes, n, 0, levels_of(n) - 1, c->stream));
    return mark(c, 2);
}

// The Merkle step of a device-resident Data table: one k_leaf_records launch
// locates every record's value and hashes it in input order -- all of them
// (NKV_OPT_BUCKET 0), or (auto) the waves whose block counts are narrow, the
// others deferred -- then the length-sorted work queue takes what was deferred
// (behind a device Gate: on a table of one record size it is never opened),
// then the levels.  err (device u32) = 1 if a header points outside the stream.
int records_tree(nkv_ctx* c, const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_off, uint64_t n,
                 uint8_t* nodes, unsigned int* err) {
    TRY(grow(c->d_off, 8 * n));
    TRY(grow(c->d_len, 8 * n));
    TRY(grow(c->d_range, 8));
    uint64_t* voff = static_cast<uint64_t*>(c->d_off.p);
    uint64_t* vlen = static_cast<uint64_t*>(c->d_len.p);
    unsigned int* range = static_cast<unsigned int*>(c->d_range.p);
    uint32_t* part = nullptr;
    TRY(locate_parts(c, n, &part));
    if (!c->records_fused) {  // NKV_OPT_RECORDS_FUSED 0: separate locate pass, then the leaf plan
        const bool gated = c->bucket == 2 && n >= 4096;
        HIPTRY(launch_locate(stream, stream_len, rec_off, n, voff, vlen, err, gated ? range : nullptr, part,
                             c->stream));
        return tree_from_device_values(c, stream, voff, vlen, n, false, nodes, nullptr, gated ? range : nullptr);
    }
    // plan_of's rule: input order without bucketing or for tiny batches; auto
    // for >= 4096 values; else everything sorted
    const int policy = (c->bucket == 0 || n <= 64) ? 0 : ((c->bucket == 2 && n >= 4096) ? 1 : 2);
    TRY(mark(c, 0));
    if (policy == 0) {
        HIPTRY(launch_leaf_records(stream, stream_len, rec_off, n, policy, voff, vlen, nodes, err, range, part,
                                   c->stream));
    } else {  // deferred plan: the pass flags gate the sorted pass, whose first launch copies err out
        uint32_t *flags, *next;
        pass_flags(c, &flags, &next);
        HIPTRY(launch_leaf_records(stream, stream_len, rec_off, n, policy, voff, vlen, nodes, nullptr, nullptr,
                                   nullptr, c->stream, flags, next));
        flip_pass_flags(c);
        TRY(leaf_level(c, stream, voff, vlen, n, false, nodes, policy == 2 ? kSorted : kGated, Gate{flags, 0},
                       false, CopyWords{flags + 2, err, 1}));
    }
    TRY(mark(c, 1));
    HIPTRY(launch_reduce(nodes, n, 0, levels_of(n) - 1, c->stream));
    return mark(c, 2);
}

}  // namespace nkv

#ifndef NKV_SRC_HASH
#define NKV_SRC_HASH "unknown"
#endif

extern "C" {

const char* nkv_build_id(void) { return "nkv-src-sha256:" NKV_SRC_HASH; }

int nkv_abi_version(void) { return NKV_ABI_VERSION; }

const char* nkv_strerror(int s) {
    switch (s) {
        case NKV_OK: return "ok";
        case NKV_ERR_EMPTY: return "cannot build Merkle Tree from 0 nodes";
        case NKV_ERR_INVALID: return "invalid argument";
        case NKV_ERR_DEVICE: return "HIP device error";
        case NKV_ERR_NOMEM: return "out of memory";
        case NKV_ERR_IO: return "file I/O error";
        default: return "unknown error";
    }
}

int nkv_device_count(int* count) try {
    if (!count) return NKV_ERR_INVALID;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *count = 0;
        return NKV_ERR_DEVICE;
    }
    *count = n;
    return NKV_OK;
} NKV_CATCH

int nkv_ctx_create(int device, nkv_ctx** out) try {
    if (!out) return NKV_ERR_INVALID;
    *out = nullptr;
    int cnt = 0;
    if (nkv_device_count(&cnt) != NKV_OK || device < 0 || device >= cnt) return NKV_ERR_DEVICE;
    nkv_ctx* c = new nkv_ctx();
    c->device = device;
    int rc = st(hipSetDevice(device));
    if (rc == NKV_OK) rc = st(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
    if (rc == NKV_OK) rc = st(hipHostMalloc(reinterpret_cast<void**>(&c->h_small), 64, hipHostMallocDefault));
    if (rc == NKV_OK) rc = grow(c->d_flags, 4 * 2 * kPassFlagWords);
    if (rc == NKV_OK) {  // both pass-flag sets start reset (each records call resets the other)
        uint32_t init[2 * kPassFlagWords] = {};
        for (uint32_t k = 0; k < 2; ++k) init[kPassFlagWords * k + 6] = init[kPassFlagWords * k + 7] = ~0u;
        rc = st(hipMemcpy(c->d_flags.p, init, sizeof(init), hipMemcpyHostToDevice));
    }
    if (rc != NKV_OK) {
        nkv_ctx_destroy(c);
        return rc;
    }
    c->stream = c->own;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->simds = uint32_t(prop.multiProcessorCount) * 4;
    *out = c;
    return NKV_OK;
} NKV_CATCH

void nkv_ctx_destroy(nkv_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->own) (void)hipStreamSynchronize(c->own);
    svc_stop(c);  // the resident small-tree service leaves before anything it reads is freed
    if (c->clock_probe) (void)set_clock_probe(nullptr, c->own);  // kernels must not add into freed memory
    for (nkv_ctx* l : c->lanes) nkv_ctx_destroy(l);
    (void)hipSetDevice(c->device);
    for (DevBuf* b : {&c->d_data, &c->d_off, &c->d_len, &c->d_nodes, &c->d_img, &c->d_tmp,
                      &c->d_err, &c->d_aux, &c->d_keys, &c->d_perm, &c->d_stmp, &c->d_queue, &c->d_stats,
                      &c->d_range, &c->d_part, &c->d_tmp2, &c->d_flags, &c->d_clk, &c->d_sin, &c->d_sout,
                      &c->d_small, &c->d_ticket})
        if (b->p) (void)hipFree(b->p);
    for (nkv_ctx::Pinned* blk : c->pinned) {
        if (blk->d_arena.p) (void)hipFree(blk->d_arena.p);
        (void)hipHostFree(blk->p);
        delete blk;
    }
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_sin) (void)hipHostFree(c->h_sin);
    if (c->d_sin_bar) (void)hipFree(c->d_sin_bar);
    if (c->h_sout) (void)hipHostFree(c->h_sout);
    for (hipEvent_t e : c->ring) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->join_ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->host_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->side) (void)hipStreamSynchronize(c->side);
    for (hipEvent_t e : c->side_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->switch_ev) (void)hipEventDestroy(c->switch_ev);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

// Stream hand-over: work already queued on the old stream (an asynchronous
// *_dev call) is ordered before anything the context queues on the new one --
// the records entries' pass flags and the sort scratch carry state from one
// call to the next on a context.
static int switch_stream(nkv_ctx* c, hipStream_t s) {
    if (s == c->stream) return NKV_OK;
    if (!c->switch_ev) HIPTRY(hipEventCreateWithFlags(&c->switch_ev, hipEventDisableTiming));
    HIPTRY(hipEventRecord(c->switch_ev, c->stream));
    HIPTRY(hipStreamWaitEvent(s, c->switch_ev, 0));
    c->stream = s;
    return NKV_OK;
}

int nkv_ctx_set_stream(nkv_ctx* c, void* s) try {
    TRY(bind(c));
    return switch_stream(c, static_cast<hipStream_t>(s));  // NULL = the device's null stream
} NKV_CATCH

int nkv_ctx_use_own_stream(nkv_ctx* c) try {
    TRY(bind(c));
    return switch_stream(c, c->own);
} NKV_CATCH

int nkv_ctx_set_option(nkv_ctx* c, int key, int64_t value) try {
    TRY(bind(c));
    switch (key) {
        case NKV_OPT_LEAF_LOAD:
            if (value != 4 && value != 11) return NKV_ERR_INVALID;
            c->leaf_load = int(value);
            return NKV_OK;
        case NKV_OPT_BUCKET:
            if (value < 0 || value > 2) return NKV_ERR_INVALID;
            c->bucket = int(value);
            return NKV_OK;
        case NKV_OPT_QUEUE_SPLIT:
            if (value < 0 || value > 0xFFFFFFFFll) return NKV_ERR_INVALID;
            c->queue_split = int(std::min<int64_t>(value, 0x7FFFFFFF));
            return NKV_OK;
        case NKV_OPT_CRC_LOAD:
            if (value != 0 && value != 8) return NKV_ERR_INVALID;
            c->crc_load = int(value);
            return NKV_OK;
        case NKV_OPT_BLOOM_PATH:
            if (value < 0 || value > 2) return NKV_ERR_INVALID;
            c->bloom_path = int(value);
            return NKV_OK;
        case NKV_OPT_HOST_THREADS:
            if (value < 0 || value > 256) return NKV_ERR_INVALID;
            c->stage.want_threads = int(value);
            return NKV_OK;
        case NKV_OPT_STAGE_CHUNK:
            if (value < 4096 || value > (int64_t(1) << 32) || (value & 4095)) return NKV_ERR_INVALID;
            if (c->stage.drain() != hipSuccess) return NKV_ERR_DEVICE;
            c->stage.chunk = size_t(value);
            return NKV_OK;
        case NKV_OPT_RECORDS_FUSED:
            if (value < 0 || value > 1) return NKV_ERR_INVALID;
            c->records_fused = int(value);
            return NKV_OK;
        case NKV_OPT_QUEUE_WAVES:
            if (value < 1 || value > 3) return NKV_ERR_INVALID;  // 12 KiB ring per wave: <= 13 per CU
            c->queue_waves = int(value);
            return NKV_OK;
        case NKV_OPT_TABLE_LANES:
            if (value < 1 || value > 8) return NKV_ERR_INVALID;
            c->table_lanes = int(value);
            return NKV_OK;
        case NKV_OPT_TIMING_EVERY:
            if (value < 1 || value > 1000000) return NKV_ERR_INVALID;
            c->timing_every = int(value);
            c->timing_calls = 0;
            return NKV_OK;
        case NKV_OPT_SMALL_PATH:
            if (value < 0 || value > 3) return NKV_ERR_INVALID;
            c->small_path = int(value);
            return NKV_OK;
        case NKV_OPT_SMALL_MAX_N:
            if (value < 0 || value > int64_t(kSmallMaxN)) return NKV_ERR_INVALID;
            c->small_max_n = uint64_t(value);
            return NKV_OK;
        case NKV_OPT_ARENA_COHERENT:
            if (value < 0 || value > 1) return NKV_ERR_INVALID;
            c->arena_coherent = int(value);
            return NKV_OK;
        case NKV_OPT_SIDE_GATE:
            if (value < 0 || value > 1) return NKV_ERR_INVALID;
            c->side_gate = int(value);
            return NKV_OK;
        case NKV_OPT_SERVICE_MAILBOX:
            if (value < 0 || value > 1) return NKV_ERR_INVALID;
            if (int(value) != c->svc_mailbox) {
                TRY(bind(c));
                svc_stop(c);  // the next request makes the buffers in the new place
                c->svc_mailbox = int(value);
            }
            return NKV_OK;
        case NKV_OPT_QUEUE_PAIR:  // retired: one wave per group (the pair kernel failed its GPU parity run)
            return value == 0 ? NKV_OK : NKV_ERR_INVALID;
        case NKV_OPT_SMALL_MAX_BYTES:
            if (value < 0 || value > (int64_t(1) << 30)) return NKV_ERR_INVALID;
            c->small_max_bytes = uint64_t(value);
            return NKV_OK;
        case NKV_OPT_DEEP_PREFETCH:  // retired: the one path left (ABI version 1)
            return value == 3 ? NKV_OK : NKV_ERR_INVALID;
        case NKV_OPT_QUEUE_RING:  // retired: the 3-slot ring (ABI version 1)
            return value == 13 ? NKV_OK : NKV_ERR_INVALID;
        default:
            return NKV_ERR_INVALID;
    }
} NKV_CATCH

int nkv_ctx_small_service_state(nkv_ctx* c, uint64_t out[8]) try {
    if (!c || !out) return NKV_ERR_INVALID;
    for (int k = 0; k < 8; ++k) out[k] = 0;
    if (c->h_mbox) {
        out[0] = __atomic_load_n(&svc_request_side(c)->doorbell, __ATOMIC_ACQUIRE);
        out[6] = c->svc_box_dev ? 1u : 0u;
        out[7] = (uint64_t(__atomic_load_n(&c->h_mbox->xcc_id, __ATOMIC_ACQUIRE)) << 32) |
                 __atomic_load_n(&c->h_mbox->hw_id, __ATOMIC_ACQUIRE);
        out[1] = __atomic_load_n(&c->h_mbox->served, __ATOMIC_ACQUIRE);
        out[2] = __atomic_load_n(&c->h_mbox->done, __ATOMIC_ACQUIRE);
    }
    out[3] = c->svc_launches;
    out[4] = c->svc_live ? 1u : 0u;
    if (c->svc) {
        TRY(bind(c));
        out[5] = hipStreamQuery(c->svc) == hipErrorNotReady ? 1u : 0u;
    }
    return NKV_OK;
} NKV_CATCH

int nkv_ctx_small_service_trace(nkv_ctx* c, int enable, uint64_t out[14]) try {
    if (!c || enable < 0 || enable > 1) return NKV_ERR_INVALID;
    if (out) {
        for (int k = 0; k < kSvcStamps; ++k)
            out[k] = c->h_mbox ? __atomic_load_n(&c->h_mbox->stamps[k], __ATOMIC_ACQUIRE) : 0u;
    }
    c->svc_trace = enable != 0;
    return NKV_OK;
} NKV_CATCH

int nkv_ctx_last_path(nkv_ctx* c, int* path) try {
    if (!c || !path) return NKV_ERR_INVALID;
    *path = c->last_path;
    return NKV_OK;
} NKV_CATCH

int nkv_ctx_sync(nkv_ctx* c) try {
    TRY(bind(c));
    return st(hipStreamSynchronize(c->stream));
} NKV_CATCH

int nkv_ctx_set_timing(nkv_ctx* c, int enable) try {
    TRY(bind(c));
    if (enable & ~(NKV_TIMING_EVENTS | NKV_TIMING_CLOCK)) return NKV_ERR_INVALID;
    c->timing = (enable & NKV_TIMING_EVENTS) != 0;
    c->timed = false;
    c->ring_used = 0;
    c->timing_calls = 0;
    for (nkv_ctx* l : c->lanes) {
        l->timing = c->timing;
        l->timed = false;
        l->ring_used = 0;
        l->timing_calls = 0;
    }
    if (enable & NKV_TIMING_CLOCK) {
        TRY(grow(c->d_clk, kClockWords * sizeof(unsigned long long)));
        HIPTRY(hipMemsetAsync(c->d_clk.p, 0, kClockWords * sizeof(unsigned long long), c->stream));
        HIPTRY(set_clock_probe(static_cast<unsigned long long*>(c->d_clk.p), c->stream));
        c->clock_probe = true;
    } else if (c->clock_probe) {
        HIPTRY(set_clock_probe(nullptr, c->stream));
        c->clock_probe = false;
    }
    return NKV_OK;
} NKV_CATCH

int nkv_ctx_clock(nkv_ctx* c, double* mhz, uint64_t* waves) try {
    TRY(bind(c));
    if (!mhz || !waves) return NKV_ERR_INVALID;
    if (!c->d_clk.p) return NKV_ERR_INVALID;
    std::vector<unsigned long long> h(kClockWords);
    HIPTRY(hipStreamSynchronize(c->stream));
    for (nkv_ctx* l : c->lanes) HIPTRY(hipStreamSynchronize(l->stream));
    HIPTRY(hipMemcpy(h.data(), c->d_clk.p, kClockWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // per slot: [0] shader-clock cycles, [1] 100 MHz reference ticks, summed over waves; [2] waves
    double cyc = 0, ticks = 0;
    uint64_t w = 0;
    for (uint32_t s = 0; s < kClockWords; s += 32) {
        cyc += double(h[s]);
        ticks += double(h[s + 1]);
        w += h[s + 2];
    }
    *mhz = ticks > 0 ? 100.0 * cyc / ticks : 0.0;
    *waves = w;
    return NKV_OK;
} NKV_CATCH

static int timing_sum(nkv_ctx* c, int* calls, double* a, double* b) {
    const size_t k = c->ring_used / 3;
    if (k) HIPTRY(hipEventSynchronize(c->ring[c->ring_used - 1]));
    for (size_t i = 0; i < k; ++i) {
        float x = 0.f, y = 0.f;
        HIPTRY(hipEventElapsedTime(&x, c->ring[3 * i], c->ring[3 * i + 1]));
        HIPTRY(hipEventElapsedTime(&y, c->ring[3 * i + 1], c->ring[3 * i + 2]));
        *a += x;
        *b += y;
    }
    *calls += int(k);
    return NKV_OK;
}

int nkv_ctx_timing_summary(nkv_ctx* c, int* calls, float* leaf_ms_total, float* reduce_ms_total) try {
    TRY(bind(c));
    if (!calls || !leaf_ms_total || !reduce_ms_total) return NKV_ERR_INVALID;
    int k = 0;
    double a = 0, b = 0;
    TRY(timing_sum(c, &k, &a, &b));
    for (nkv_ctx* l : c->lanes) TRY(timing_sum(l, &k, &a, &b));  // nkv_trees_dev's lanes
    *calls = k;
    *leaf_ms_total = float(a);
    *reduce_ms_total = float(b);
    return NKV_OK;
} NKV_CATCH

int nkv_ctx_last_host_timing(nkv_ctx* c, float* upload_ms, float* kernels_ms, float* download_ms) try {
    TRY(bind(c));
    if (!c->host_timed || !c->timed) return NKV_ERR_INVALID;
    hipEvent_t* ev = &c->ring[c->ring_used - 3];
    HIPTRY(hipEventSynchronize(c->host_ev[1]));
    float a = 0.f, b = 0.f, d = 0.f;
    HIPTRY(hipEventElapsedTime(&a, c->host_ev[0], ev[0]));
    HIPTRY(hipEventElapsedTime(&b, ev[0], ev[2]));
    HIPTRY(hipEventElapsedTime(&d, ev[2], c->host_ev[1]));
    if (upload_ms) *upload_ms = a;
    if (kernels_ms) *kernels_ms = b;
    if (download_ms) *download_ms = d;
    return NKV_OK;
} NKV_CATCH

int nkv_ctx_last_timing(nkv_ctx* c, float* leaf_ms, float* reduce_ms) try {
    TRY(bind(c));
    if (!c->timed) return NKV_ERR_INVALID;
    hipEvent_t* ev = &c->ring[c->ring_used - 3];
    HIPTRY(hipEventSynchronize(ev[2]));
    float a = 0.f, b = 0.f;
    HIPTRY(hipEventElapsedTime(&a, ev[0], ev[1]));
    HIPTRY(hipEventElapsedTime(&b, ev[1], ev[2]));
    if (leaf_ms) *leaf_ms = a;
    if (reduce_ms) *reduce_ms = b;
    return NKV_OK;
} NKV_CATCH

// ---- shape ----
int nkv_num_levels(uint64_t n) { return levels_of(n); }
uint64_t nkv_level_count(uint64_t n, int L) {
    return (n == 0 || L < 0 || L >= levels_of(n)) ? 0 : count_of(n, L);
}
uint64_t nkv_level_start(uint64_t n, int L) {
    return (n == 0 || L < 0 || L >= levels_of(n)) ? 0 : start_of(n, L);
}
uint64_t nkv_total_nodes(uint64_t n) { return total_of(n); }
uint64_t nkv_bfs_size(uint64_t n) { return n == 0 ? 0 : layout_of(counts_of(n)).total; }

// ---- pinned arena ----
constexpr uint64_t kEagerMirrorBytes = uint64_t(64) << 20;
int nkv_host_alloc(nkv_ctx* c, uint64_t bytes, void** out) try {
    if (!out) return NKV_ERR_INVALID;
    *out = nullptr;
    TRY(bind(c));
    void* p = nullptr;
    // host-coherent by default (NKV_OPT_ARENA_COHERENT): DMA reads it as any
    // pinned block, and the small-tree kernel may read it in place (uncached on
    // the GPU side, so a block rewritten flush after flush is never stale there)
    const unsigned flags = c->arena_coherent ? hipHostMallocCoherent : hipHostMallocDefault;
    if (hipHostMalloc(&p, bytes ? bytes : 1, flags) != hipSuccess) {
        (void)hipGetLastError();
        return NKV_ERR_NOMEM;
    }
    nkv_ctx::Pinned* blk = new (std::nothrow)
        nkv_ctx::Pinned{static_cast<uint8_t*>(p), bytes ? bytes : 1, 0, {}, c->arena_coherent != 0};
    if (!blk) {
        (void)hipHostFree(p);
        return NKV_ERR_NOMEM;
    }
    // a large block's device mirror now, not inside the first flush that
    // streams into it (an arena reserved at engine start costs a flush
    // nothing); small blocks, and any block whose mirror does not fit the HBM
    // free right now, get theirs on first use (stream_block): a caller whose
    // values only ever take the small path never needs it
    if (blk->bytes >= kEagerMirrorBytes && grow(blk->d_arena, blk->bytes) != NKV_OK) (void)hipGetLastError();
    c->pinned.push_back(blk);
    *out = p;
    return NKV_OK;
} NKV_CATCH

int nkv_host_free(nkv_ctx* c, void* p) try {
    TRY(bind(c));
    if (!p) return NKV_OK;
    for (size_t i = 0; i < c->pinned.size(); ++i) {
        nkv_ctx::Pinned* blk = c->pinned[i];
        if (blk->p != p) continue;
        // copies from the block (nkv_host_stream, a tree call) may still be queued
        HIPTRY(hipStreamSynchronize(c->stream));
        if (blk->d_arena.p) (void)hipFree(blk->d_arena.p);
        c->pinned.erase(c->pinned.begin() + long(i));
        delete blk;
        break;
    }
    return st(hipHostFree(p));
} NKV_CATCH

int nkv_host_stream(nkv_ctx* c, const void* block, uint64_t upto) try {
    TRY(bind(c));
    if (!block) return NKV_ERR_INVALID;
    for (nkv_ctx::Pinned* blk : c->pinned) {
        if (blk->p != block) continue;
        if (upto > blk->bytes) return NKV_ERR_INVALID;
        if (upto < blk->streamed) blk->streamed = 0;  // a new batch: its bytes replace the old ones
        TRY(stream_block(c, blk, blk->streamed, upto));
        blk->streamed = std::max(blk->streamed, upto);
        return NKV_OK;
    }
    return NKV_ERR_INVALID;  // not a block nkv_host_alloc returned on this context
} NKV_CATCH

// ---- host-buffer API ----
int nkv_leaf_hash(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                  uint64_t n, uint8_t* out20) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!base || !off || !len || !out20) return NKV_ERR_INVALID;
    const uint8_t* d_base = nullptr;
    bool aligned = true;
    TRY(stage_values(c, base, off, len, n, &d_base, &aligned));
    TRY(grow(c->d_nodes, 20 * n));
    uint8_t* nodes = static_cast<uint8_t*>(c->d_nodes.p);
    TRY(leaf_level(c, d_base, static_cast<const uint64_t*>(c->d_off.p), static_cast<const uint64_t*>(c->d_len.p), n,
                   aligned, nodes, len));
    HIPTRY(c->stage.download(out20, nodes, 20 * n, c->stream));
    return st(hipStreamSynchronize(c->stream));
} NKV_CATCH

int nkv_tree_build(nkv_ctx* c, const uint8_t* leaf20, uint64_t n, uint8_t* root20,
                   uint8_t* nodes_out, uint8_t* img_out) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!leaf20) return NKV_ERR_INVALID;
    TRY(grow(c->d_nodes, 20 * total_of(n)));
    uint8_t* nodes = static_cast<uint8_t*>(c->d_nodes.p);
    HIPTRY(c->stage.upload(leaf20, 20 * n, nodes, c->stream));
    HIPTRY(launch_reduce(nodes, n, 0, levels_of(n) - 1, c->stream));
    return finish_tree(c, nodes, n, root20, nodes_out, img_out);
} NKV_CATCH

int nkv_tree_from_values(nkv_ctx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                         uint64_t n, uint8_t* root20, uint8_t* nodes_out, uint8_t* img_out) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!base || !off || !len) return NKV_ERR_INVALID;
    bool small = false;
    TRY(small_tree(c, base, off, len, n, root20, nodes_out, img_out, &small));
    if (small) return NKV_OK;
    c->last_path = NKV_PATH_GRID;
    TRY(host_mark(c, 0));
    const uint8_t* d_base = nullptr;
    bool aligned = true;
    TRY(stage_values(c, base, off, len, n, &d_base, &aligned));
    TRY(grow(c->d_nodes, 20 * total_of(n)));
    uint8_t* nodes = static_cast<uint8_t*>(c->d_nodes.p);
    TRY(tree_from_device_values(c, d_base, static_cast<const uint64_t*>(c->d_off.p),
                                static_cast<const uint64_t*>(c->d_len.p), n, aligned, nodes, len));
    TRY(finish_tree(c, nodes, n, root20, nodes_out, img_out));
    return host_mark(c, 1);
} NKV_CATCH

uint64_t nkv_generic_bfs_size(const uint64_t* len, uint64_t n) {
    if (n == 0 || !len) return 0;
    // levels 1..top are 20-byte nodes; level 0 is the raw leaves
    uint64_t s = nkv_bfs_size(n) - 21 * n;
    for (uint64_t i = 0; i < n; ++i) s += len[i] ? 1 + len[i] : 1;
    return s;
}

int nkv_tree_generic(nkv_ctx* c, const uint8_t* data, const uint64_t* off, const uint64_t* len,
                     uint64_t n, uint8_t* root20, uint8_t* upper_out, uint8_t* img_out) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!data || !off || !len) return NKV_ERR_INVALID;
    // Level 1 node i = SHA-1(leaf[2i].Data || leaf[2i+1].Data) (merkletree.go:44-46;
    // the pad of an odd level contributes no bytes).  Stage each parent's
    // message contiguously and hash the messages with the leaf kernel; the
    // rest of the tree is the 20-byte reduce over the n1 level-1 nodes.
    const uint64_t n1 = (n + 1) / 2;
    std::vector<uint64_t> moff(n1), mlen(n1);
    std::vector<uint8_t> tmp;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n1; ++i) {
        mlen[i] = len[2 * i] + (2 * i + 1 < n ? len[2 * i + 1] : 0);
        total += mlen[i];
    }
    tmp.resize(total ? total : 1);
    uint64_t p = 0;
    for (uint64_t i = 0; i < n1; ++i) {
        moff[i] = p;
        memcpy(tmp.data() + p, data + off[2 * i], len[2 * i]);
        p += len[2 * i];
        if (2 * i + 1 < n) {
            memcpy(tmp.data() + p, data + off[2 * i + 1], len[2 * i + 1]);
            p += len[2 * i + 1];
        }
    }
    const uint8_t* d_base = nullptr;
    bool aligned = true;
    TRY(stage_values(c, tmp.data(), moff.data(), mlen.data(), n1, &d_base, &aligned));
    const uint64_t up_total = n1 == 1 ? 1 : total_of(n1);
    TRY(grow(c->d_nodes, 20 * up_total));
    uint8_t* up = static_cast<uint8_t*>(c->d_nodes.p);
    TRY(leaf_level(c, d_base, static_cast<const uint64_t*>(c->d_off.p), static_cast<const uint64_t*>(c->d_len.p), n1,
                   aligned, up, mlen.data()));
    if (n1 > 1) HIPTRY(launch_reduce(up, n1, 0, levels_of(n1) - 1, c->stream));
    if (upper_out) HIPTRY(c->stage.download(upper_out, up, 20 * up_total, c->stream));
    if (root20)
        HIPTRY(hipMemcpyAsync(root20, up + 20 * (up_total - 1), 20, hipMemcpyDeviceToHost,
                              c->stream));
    uint64_t upper_img = 0;
    if (img_out) {
        // levels top..1 from the device, level 0 (raw leaf Data) appended here
        std::vector<uint64_t> cnt = n1 == 1 ? std::vector<uint64_t>{1} : counts_of(n1);
        BfsLayout lay = layout_of(cnt);
        // the bottom of this sub-image is level 1 of the whole tree, which is
        // never the top when n1 > 1; its pad is already handled by layout_of
        upper_img = lay.total;
        TRY(grow(c->d_img, lay.total));
        HIPTRY(launch_bfs_image(up, lay, static_cast<uint8_t*>(c->d_img.p), c->stream));
        HIPTRY(c->stage.download(img_out, static_cast<const uint8_t*>(c->d_img.p), lay.total, c->stream));
    }
    HIPTRY(hipStreamSynchronize(c->stream));
    if (img_out) {
        uint8_t* q = img_out + upper_img;
        for (uint64_t i = 0; i < n; ++i) {
            if (len[i] == 0) {
                *q++ = NKV_MERKLE_NODE_EMPTY;
            } else {
                *q++ = 0;
                memcpy(q, data + off[i], len[i]);
                q += len[i];
            }
        }
        if (n & 1) *q++ = NKV_MERKLE_NODE_EMPTY;
    }
    return NKV_OK;
} NKV_CATCH

int nkv_tree_validate(nkv_ctx* c, const uint8_t* leaf_data, const uint64_t* off, const uint64_t* len,
                      uint64_t n, const uint8_t* root20, int* ok) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (!ok) return NKV_ERR_INVALID;
    *ok = 0;
    if (n == 0) return NKV_ERR_EMPTY;  // New never builds an empty tree (merkletree.go:19-21)
    if (!leaf_data || !off || !len || !root20) return NKV_ERR_INVALID;
    bool all20 = true;
    for (uint64_t i = 0; i < n && all20; ++i) all20 = len[i] == NKV_DIGEST_SIZE;
    uint8_t got[NKV_DIGEST_SIZE];
    if (all20) {
        // NewLeaf leaves: gather the digests into level 0 and reduce to the root
        TRY(grow_host(c, 8 * n));
        uint64_t* dst = static_cast<uint64_t*>(c->h_stage);
        for (uint64_t i = 0; i < n; ++i) dst[i] = NKV_DIGEST_SIZE * i;
        TRY(grow(c->d_nodes, NKV_DIGEST_SIZE * total_of(n)));
        uint8_t* nodes = static_cast<uint8_t*>(c->d_nodes.p);
        const Segments seg{leaf_data, off, len, dst, n};
        HIPTRY(c->stage.upload(seg, NKV_DIGEST_SIZE * n, nodes, c->stream));
        HIPTRY(launch_reduce(nodes, n, 0, levels_of(n) - 1, c->stream));
        HIPTRY(hipMemcpyAsync(c->h_small, nodes + NKV_DIGEST_SIZE * (total_of(n) - 1), NKV_DIGEST_SIZE,
                              hipMemcpyDeviceToHost, c->stream));
        HIPTRY(hipStreamSynchronize(c->stream));
        memcpy(got, c->h_small, NKV_DIGEST_SIZE);
    } else {
        TRY(nkv_tree_generic(c, leaf_data, off, len, n, got, nullptr, nullptr));
    }
    *ok = memcmp(got, root20, NKV_DIGEST_SIZE) == 0;
    return NKV_OK;
} NKV_CATCH

int nkv_tree_from_records(nkv_ctx* c, const uint8_t* stream, uint64_t stream_len,
                          const uint64_t* rec_size, uint64_t n, uint8_t* root20,
                          uint8_t* nodes_out, uint8_t* img_out) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!stream || !rec_size) return NKV_ERR_INVALID;
    if (!records_fit(rec_size, n, stream_len)) return NKV_ERR_INVALID;
    if (c->small_path != 0 && n <= c->small_max_n && n <= kSmallMaxN && stream_len <= c->small_max_bytes) {
        // a small table (one lsm_run_max compaction at the default sizes): the
        // values' places from the headers here (record.go:191-199, the same
        // bounds k_locate applies), then the one-launch path
        std::vector<uint64_t> voff(n), vlen(n);
        uint64_t r = 0;
        for (uint64_t i = 0; i < n; ++i) {
            if (!header_in(r, stream_len)) return NKV_ERR_INVALID;
            uint64_t ks = 0, vs = 0;
            memcpy(&ks, stream + r + 14, 8);
            memcpy(&vs, stream + r + 22, 8);
            if (ks > stream_len || vs > stream_len || r + 30 + ks + vs > stream_len) return NKV_ERR_INVALID;
            voff[i] = r + 30 + ks;
            vlen[i] = vs;
            r += rec_size[i];
        }
        bool small = false;
        TRY(small_tree(c, stream, voff.data(), vlen.data(), n, root20, nodes_out, img_out, &small));
        if (small) return NKV_OK;
    }
    c->last_path = NKV_PATH_GRID;
    TRY(stage_stream(c, stream, stream_len, c->d_data, rec_size, n, c->d_aux));
    // record offsets in their own scratch (records_tree uses d_off / d_len)
    TRY(grow(c->d_tmp2, 8 * n));
    uint64_t* rec_off = static_cast<uint64_t*>(c->d_tmp2.p);
    TRY(nkv_record_offsets_dev(c, static_cast<const uint64_t*>(c->d_aux.p), n, rec_off));
    TRY(grow(c->d_nodes, 20 * total_of(n)));
    uint8_t* nodes = static_cast<uint8_t*>(c->d_nodes.p);
    TRY(grow(c->d_err, 4));
    unsigned int* err = static_cast<unsigned int*>(c->d_err.p);
    TRY(records_tree(c, static_cast<const uint8_t*>(c->d_data.p), stream_len, rec_off, n, nodes, err));
    unsigned int h = 0;
    HIPTRY(hipMemcpyAsync(&h, err, 4, hipMemcpyDeviceToHost, c->stream));
    HIPTRY(hipStreamSynchronize(c->stream));
    if (h) return NKV_ERR_INVALID;
    return finish_tree(c, nodes, n, root20, nodes_out, img_out);
} NKV_CATCH

int nkv_record_crc(nkv_ctx* c, const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_size,
                   uint64_t n, uint32_t* crc_out, uint64_t* n_bad, uint64_t* first_bad) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n_bad) *n_bad = 0;
    if (first_bad) *first_bad = ~0ull;
    if (n == 0) return NKV_OK;
    if (!stream || !rec_size) return NKV_ERR_INVALID;
    if (!records_fit(rec_size, n, stream_len)) return NKV_ERR_INVALID;
    TRY(stage_stream(c, stream, stream_len, c->d_data, rec_size, n, c->d_aux));
    TRY(grow(c->d_len, 8 * n));
    TRY(grow(c->d_off, 4 * n));
    uint64_t* rec_off = static_cast<uint64_t*>(c->d_len.p);
    TRY(nkv_record_offsets_dev(c, static_cast<const uint64_t*>(c->d_aux.p), n, rec_off));
    TRY(grow(c->d_stats, 24));
    uint32_t* d_crc = static_cast<uint32_t*>(c->d_off.p);
    uint64_t* d_stats = static_cast<uint64_t*>(c->d_stats.p);
    TRY(nkv_record_crc_dev(c, c->d_data.p, stream_len, rec_off, n, d_crc, d_stats));
    // the rec_size copy in h_stage has been consumed once the stream reaches here
    uint64_t* hs = static_cast<uint64_t*>(c->h_stage);
    HIPTRY(hipMemcpyAsync(hs, d_stats, 24, hipMemcpyDeviceToHost, c->stream));
    HIPTRY(hipStreamSynchronize(c->stream));
    if (hs[2]) return NKV_ERR_INVALID;
    if (n_bad) *n_bad = hs[0];
    if (first_bad) *first_bad = hs[1];
    if (crc_out) HIPTRY(c->stage.download(reinterpret_cast<uint8_t*>(crc_out), reinterpret_cast<const uint8_t*>(d_crc),
                                          4 * n, c->stream));
    return NKV_OK;
} NKV_CATCH

int nkv_bloom_params(uint64_t n, double p, uint32_t* m, uint32_t* k) try {
    if (!m || !k || n == 0 || !(p > 0.0 && p < 1.0)) return NKV_ERR_INVALID;
    const double ln2 = std::log(2.0);  // bloomfilter.go:18-24
    const double mm = std::ceil(double(n) * std::fabs(std::log(p)) / std::pow(ln2, 2.0));
    if (!(mm >= 1.0 && mm <= 4294967295.0)) return NKV_ERR_INVALID;
    *m = uint32_t(mm);
    *k = uint32_t(std::ceil((double(*m) / double(n)) * ln2));
    return NKV_OK;
} NKV_CATCH

static uint64_t bloom_words(uint32_t m) { return (uint64_t(m) + 31) / 32; }

int nkv_bloom_build(nkv_ctx* c, const uint8_t* keys, const uint64_t* off, const uint64_t* len, uint64_t n,
                    uint32_t m, uint32_t k, uint32_t seed0, uint8_t* bits_out) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (m == 0 || !bits_out || (n && (!keys || !off || !len))) return NKV_ERR_INVALID;
    const uint64_t nbytes = (uint64_t(m) + 7) / 8, wbytes = 4 * bloom_words(m);
    TRY(grow(c->d_img, wbytes));
    HIPTRY(hipMemsetAsync(c->d_img.p, 0, wbytes, c->stream));
    if (n) {
        uint64_t total = 0;
        for (uint64_t i = 0; i < n; ++i) total = std::max(total, off[i] + len[i]);
        TRY(grow_host(c, 16 * n));
        TRY(grow(c->d_data, total + 1));
        TRY(grow(c->d_off, 8 * n));
        TRY(grow(c->d_len, 8 * n));
        uint8_t* h = static_cast<uint8_t*>(c->h_stage);
        HIPTRY(c->stage.upload(keys, total, static_cast<uint8_t*>(c->d_data.p), c->stream));
        memcpy(h, off, 8 * n);
        memcpy(h + 8 * n, len, 8 * n);
        HIPTRY(hipMemcpyAsync(c->d_off.p, h, 8 * n, hipMemcpyHostToDevice, c->stream));
        HIPTRY(hipMemcpyAsync(c->d_len.p, h + 8 * n, 8 * n, hipMemcpyHostToDevice, c->stream));
        TRY(nkv_bloom_insert_dev(c, c->d_data.p, static_cast<const uint64_t*>(c->d_off.p),
                                 static_cast<const uint64_t*>(c->d_len.p), n, m, k, seed0, c->d_img.p));
    }
    HIPTRY(c->stage.download(bits_out, static_cast<const uint8_t*>(c->d_img.p), nbytes, c->stream));
    return st(hipStreamSynchronize(c->stream));
} NKV_CATCH

int nkv_bloom_from_records(nkv_ctx* c, const uint8_t* stream, uint64_t stream_len, const uint64_t* rec_size,
                           uint64_t n, uint32_t m, uint32_t k, uint32_t seed0, uint8_t* bits_out) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (m == 0 || !bits_out || (n && (!stream || !rec_size))) return NKV_ERR_INVALID;
    const uint64_t nbytes = (uint64_t(m) + 7) / 8, wbytes = 4 * bloom_words(m);
    TRY(grow(c->d_img, wbytes));
    HIPTRY(hipMemsetAsync(c->d_img.p, 0, wbytes, c->stream));
    if (n) {
        if (!records_fit(rec_size, n, stream_len)) return NKV_ERR_INVALID;
        TRY(stage_stream(c, stream, stream_len, c->d_data, rec_size, n, c->d_aux));
        TRY(grow(c->d_len, 8 * n));
        uint64_t* rec_off = static_cast<uint64_t*>(c->d_len.p);
        TRY(nkv_record_offsets_dev(c, static_cast<const uint64_t*>(c->d_aux.p), n, rec_off));
        TRY(nkv_bloom_insert_records_dev(c, c->d_data.p, stream_len, rec_off, n, m, k, seed0, c->d_img.p));
    }
    HIPTRY(c->stage.download(bits_out, static_cast<const uint8_t*>(c->d_img.p), nbytes, c->stream));
    return st(hipStreamSynchronize(c->stream));
} NKV_CATCH

int nkv_write_file(const char* fname, const uint8_t* data, uint64_t len) try {
    if (!fname || (!data && len)) return NKV_ERR_INVALID;
    int fd = open(fname, O_WRONLY | O_CREAT, 0666);  // no O_TRUNC: merkletree.go:68
    if (fd < 0) return NKV_ERR_IO;
    // one sequential write (positioned writes from several threads measured no
    // faster: buffered writes to one file serialise on its inode lock)
    uint64_t done = 0;
    while (done < len) {
        ssize_t w = write(fd, data + done, size_t(std::min<uint64_t>(len - done, 1ull << 30)));
        if (w <= 0) {
            close(fd);
            return NKV_ERR_IO;
        }
        done += uint64_t(w);
    }
    return close(fd) == 0 ? NKV_OK : NKV_ERR_IO;
} NKV_CATCH

// ---- device-resident API ----
int nkv_leaf_hash_dev(nkv_ctx* c, const void* d_base, const uint64_t* d_off,
                      const uint64_t* d_len, uint64_t n, void* d_nodes) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_base || !d_off || !d_len || !d_nodes) return NKV_ERR_INVALID;
    return leaf_level(c, static_cast<const uint8_t*>(d_base), d_off, d_len, n, false,
                      static_cast<uint8_t*>(d_nodes), nullptr);
} NKV_CATCH

int nkv_leaf_hash_strided_dev(nkv_ctx* c, const void* d_base, uint64_t stride, uint64_t len,
                              uint64_t n, void* d_nodes) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_base || !d_nodes) return NKV_ERR_INVALID;
    return st(launch_leaf_strided(static_cast<const uint8_t*>(d_base), stride, len, n,
                                  c->leaf_load, static_cast<uint8_t*>(d_nodes), c->stream));
} NKV_CATCH

int nkv_tree_reduce_dev(nkv_ctx* c, void* d_nodes, uint64_t n) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!d_nodes) return NKV_ERR_INVALID;
    return st(launch_reduce(static_cast<uint8_t*>(d_nodes), n, 0, levels_of(n) - 1, c->stream));
} NKV_CATCH

int nkv_tree_from_values_dev(nkv_ctx* c, const void* d_base, const uint64_t* d_off,
                             const uint64_t* d_len, uint64_t n, void* d_nodes) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!d_base || !d_off || !d_len || !d_nodes) return NKV_ERR_INVALID;
    return tree_from_device_values(c, static_cast<const uint8_t*>(d_base), d_off, d_len, n, false,
                                   static_cast<uint8_t*>(d_nodes));
} NKV_CATCH

int nkv_tree_from_strided_dev(nkv_ctx* c, const void* d_base, uint64_t stride, uint64_t len,
                              uint64_t n, void* d_nodes) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!d_base || !d_nodes) return NKV_ERR_INVALID;
    uint8_t* nodes = static_cast<uint8_t*>(d_nodes);
    const int top = levels_of(n) - 1;
    TRY(mark(c, 0));
    HIPTRY(launch_leaf_strided(static_cast<const uint8_t*>(d_base), stride, len, n,
                               c->leaf_load, nodes, c->stream));
    TRY(mark(c, 1));
    HIPTRY(launch_reduce(nodes, n, 0, top, c->stream));
    return mark(c, 2);
} NKV_CATCH

int nkv_bfs_image_dev(nkv_ctx* c, const void* d_nodes, uint64_t n, void* d_img) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!d_nodes || !d_img) return NKV_ERR_INVALID;
    BfsLayout lay = layout_of(counts_of(n));
    return st(launch_bfs_image(static_cast<const uint8_t*>(d_nodes), lay,
                               static_cast<uint8_t*>(d_img), c->stream));
} NKV_CATCH

int nkv_record_offsets_dev(nkv_ctx* c, const uint64_t* d_rec_size, uint64_t n,
                           uint64_t* d_rec_off) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_rec_size || !d_rec_off || n > 0x7fffffffull) return NKV_ERR_INVALID;
    size_t tb = 0;
    HIPTRY(scan_exclusive_u64(d_rec_size, d_rec_off, n, nullptr, &tb, c->stream));
    TRY(grow(c->d_tmp, tb));
    return st(scan_exclusive_u64(d_rec_size, d_rec_off, n, c->d_tmp.p, &tb, c->stream));
} NKV_CATCH

int nkv_locate_values_dev(nkv_ctx* c, const void* d_stream, uint64_t stream_len,
                          const uint64_t* d_rec_off, uint64_t n, uint64_t* d_voff,
                          uint64_t* d_vlen) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_stream || !d_rec_off || !d_voff || !d_vlen) return NKV_ERR_INVALID;
    TRY(grow(c->d_err, 4));
    unsigned int* err = static_cast<unsigned int*>(c->d_err.p);
    uint32_t* part = nullptr;
    TRY(locate_parts(c, n, &part));
    HIPTRY(launch_locate(static_cast<const uint8_t*>(d_stream), stream_len, d_rec_off, n, d_voff,
                         d_vlen, err, nullptr, part, c->stream));
    unsigned int h = 0;
    HIPTRY(hipMemcpyAsync(&h, err, 4, hipMemcpyDeviceToHost, c->stream));
    HIPTRY(hipStreamSynchronize(c->stream));
    return h ? NKV_ERR_INVALID : NKV_OK;
} NKV_CATCH

int nkv_tree_from_records_dev(nkv_ctx* c, const void* d_stream, uint64_t stream_len, const uint64_t* d_rec_off,
                              uint64_t n, void* d_nodes, uint32_t* d_err) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!d_stream || !d_rec_off || !d_nodes) return NKV_ERR_INVALID;
    unsigned int* err = reinterpret_cast<unsigned int*>(d_err);
    if (!err) {
        TRY(grow(c->d_err, 4));
        err = static_cast<unsigned int*>(c->d_err.p);
    }
    TRY(records_tree(c, static_cast<const uint8_t*>(d_stream), stream_len, d_rec_off, n,
                     static_cast<uint8_t*>(d_nodes), err));
    if (d_err) return NKV_OK;
    unsigned int h = 0;
    HIPTRY(hipMemcpyAsync(&h, err, 4, hipMemcpyDeviceToHost, c->stream));
    HIPTRY(hipStreamSynchronize(c->stream));
    return h ? NKV_ERR_INVALID : NKV_OK;
} NKV_CATCH

// Compaction read in one pass: the Merkle tree of the records' Values and the
// check of every record's Crc.  k_leaf_verify parses the headers, checks every
// Crc and hashes the waves whose value sizes are narrow (the range rule of
// plan_of), reading each record once for both; it defers ragged waves (after
// their checksums) to the length-sorted leaf pass behind a device Gate, as
// records_tree does.
int nkv_tree_verify_records_dev(nkv_ctx* c, const void* d_stream, uint64_t stream_len, const uint64_t* d_rec_off,
                                uint64_t n, void* d_nodes, uint32_t* d_crc, uint64_t* d_stats) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (!d_stream || !d_rec_off || !d_nodes) return NKV_ERR_INVALID;
    const uint8_t* stream = static_cast<const uint8_t*>(d_stream);
    uint8_t* nodes = static_cast<uint8_t*>(d_nodes);
    unsigned long long* stats = reinterpret_cast<unsigned long long*>(d_stats);
    if (!stats) {
        TRY(grow(c->d_stats, 24));
        stats = static_cast<unsigned long long*>(c->d_stats.p);
    }
    // records_tree's policy rule: input order without bucketing or for tiny
    // batches; auto for >= 4096 records; else everything sorted
    const int policy = (c->bucket == 0 || n <= 64) ? 0 : ((c->bucket == 2 && n >= 4096) ? 1 : 2);
    if (policy == 0) {  // else the stats start in the pass flags (reset by the previous call)
        HIPTRY(hipMemsetAsync(stats, 0, 24, c->stream));
        HIPTRY(hipMemsetAsync(stats + 1, 0xFF, 8, c->stream));
    }
    TRY(grow(c->d_off, 8 * n));
    TRY(grow(c->d_len, 8 * n));
    TRY(grow(c->d_range, 8));
    uint64_t* voff = static_cast<uint64_t*>(c->d_off.p);
    uint64_t* vlen = static_cast<uint64_t*>(c->d_len.p);
    unsigned int* range = static_cast<unsigned int*>(c->d_range.p);
    uint32_t* part = nullptr;
    TRY(locate_parts(c, n, &part));
    TRY(mark(c, 0));
    if (policy == 0) {
        HIPTRY(launch_leaf_verify(stream, stream_len, d_rec_off, n, policy, voff, vlen, nodes, d_crc, stats, range,
                                  part, c->stream));
    } else {  // as records_tree: the pass flags, the stats copied out by the sort's first launch
        uint32_t *flags, *next;
        pass_flags(c, &flags, &next);
        HIPTRY(launch_leaf_verify(stream, stream_len, d_rec_off, n, policy, voff, vlen, nodes, d_crc, stats,
                                  nullptr, nullptr, c->stream, flags, next));
        flip_pass_flags(c);
        TRY(leaf_level(c, stream, voff, vlen, n, false, nodes, policy == 2 ? kSorted : kGated, Gate{flags, 0},
                       false, CopyWords{flags + 4, reinterpret_cast<uint32_t*>(stats), 6}));
    }
    TRY(mark(c, 1));
    HIPTRY(launch_reduce(nodes, n, 0, levels_of(n) - 1, c->stream));
    return mark(c, 2);
} NKV_CATCH

int nkv_crc32_dev(nkv_ctx* c, const void* d_base, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                  uint32_t* d_crc) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_base || !d_off || !d_len || !d_crc) return NKV_ERR_INVALID;
    return st(launch_crc_spans(static_cast<const uint8_t*>(d_base), d_off, d_len, n, d_crc, c->crc_load, c->stream));
} NKV_CATCH

int nkv_record_crc_dev(nkv_ctx* c, const void* d_stream, uint64_t stream_len, const uint64_t* d_rec_off,
                       uint64_t n, uint32_t* d_crc, uint64_t* d_stats) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (!d_stream && n) return NKV_ERR_INVALID;
    if (n && !d_rec_off) return NKV_ERR_INVALID;
    if (n == 0) {
        if (d_stats) {
            HIPTRY(hipMemsetAsync(d_stats, 0, 24, c->stream));
            HIPTRY(hipMemsetAsync(d_stats + 1, 0xFF, 8, c->stream));
        }
        return NKV_OK;
    }
    unsigned long long* stats = reinterpret_cast<unsigned long long*>(d_stats);
    if (!stats) {
        TRY(grow(c->d_stats, 24));
        stats = static_cast<unsigned long long*>(c->d_stats.p);
    }
    return st(launch_record_crc(static_cast<const uint8_t*>(d_stream), stream_len, d_rec_off, n, d_crc, stats,
                                c->crc_load, c->stream));
} NKV_CATCH

// Filter inserts: the range-privatised build (bloom.hip) for batches of at least
// 4096 keys when its scratch applies, else one device atomicOr per bit.
static int bloom_insert(nkv_ctx* c, int mode, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                        uint64_t stream_len, uint64_t n, uint32_t m, uint32_t k, uint32_t seed0, uint32_t* bits,
                        unsigned int* err) {
    const uint64_t staged = c->bloom_path == 2 && n >= 4096 ? bloom_staged_scratch_words(n, m, k) : 0;
    if (staged) {
        TRY(grow(c->d_tmp, 4 * staged));
        return st(launch_bloom_staged(mode, base, off, len, stream_len, n, m, k, seed0, bits, err,
                                      static_cast<uint32_t*>(c->d_tmp.p), c->stream));
    }
    const uint64_t words = c->bloom_path >= 1 && n >= 4096 ? bloom_ranges_scratch_words(n, m, k) : 0;
    if (words) {
        TRY(grow(c->d_tmp, 4 * words));
        return st(launch_bloom_ranges(mode, base, off, len, stream_len, n, m, k, seed0, bits, err,
                                      static_cast<uint32_t*>(c->d_tmp.p), c->stream));
    }
    return st(launch_bloom(mode, false, base, off, len, stream_len, n, m, k, seed0, bits, nullptr, err, c->stream));
}

int nkv_bloom_insert_dev(nkv_ctx* c, const void* d_keys, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                         uint32_t m, uint32_t k, uint32_t seed0, void* d_bits) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (m == 0 || !d_bits) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_keys || !d_off || !d_len) return NKV_ERR_INVALID;
    return bloom_insert(c, 0, static_cast<const uint8_t*>(d_keys), d_off, d_len, 0, n, m, k, seed0,
                        static_cast<uint32_t*>(d_bits), nullptr);
} NKV_CATCH

int nkv_bloom_insert_records_dev(nkv_ctx* c, const void* d_stream, uint64_t stream_len, const uint64_t* d_rec_off,
                                 uint64_t n, uint32_t m, uint32_t k, uint32_t seed0, void* d_bits) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (m == 0 || !d_bits) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_stream || !d_rec_off) return NKV_ERR_INVALID;
    TRY(grow(c->d_err, 4));
    unsigned int* err = static_cast<unsigned int*>(c->d_err.p);
    HIPTRY(hipMemsetAsync(err, 0, 4, c->stream));
    TRY(bloom_insert(c, 1, static_cast<const uint8_t*>(d_stream), d_rec_off, nullptr, stream_len, n, m, k, seed0,
                     static_cast<uint32_t*>(d_bits), err));
    unsigned int h = 0;
    HIPTRY(hipMemcpyAsync(&h, err, 4, hipMemcpyDeviceToHost, c->stream));
    HIPTRY(hipStreamSynchronize(c->stream));
    return h ? NKV_ERR_INVALID : NKV_OK;
} NKV_CATCH

int nkv_bloom_query_dev(nkv_ctx* c, const void* d_keys, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                        uint32_t m, uint32_t k, uint32_t seed0, const void* d_bits, uint8_t* d_out) try {
    TRY(bind(c));
    if (n > kMaxN) return NKV_ERR_INVALID;
    if (m == 0 || !d_bits) return NKV_ERR_INVALID;
    if (n == 0) return NKV_OK;
    if (!d_keys || !d_off || !d_len || !d_out) return NKV_ERR_INVALID;
    if (k == 0) return st(hipMemsetAsync(d_out, 1, n, c->stream));  // Query with no hashes: true
    return st(launch_bloom(0, true, static_cast<const uint8_t*>(d_keys), d_off, d_len, 0, n, m, k, seed0,
                           const_cast<uint32_t*>(static_cast<const uint32_t*>(d_bits)), d_out, nullptr,
                           c->stream));
} NKV_CATCH

int nkv_fill_splitmix64_dev(nkv_ctx* c, void* d_buf, uint64_t nbytes, uint64_t seed) try {
    TRY(bind(c));
    if (nbytes == 0) return NKV_OK;
    if (!d_buf) return NKV_ERR_INVALID;
    return st(launch_fill(static_cast<uint8_t*>(d_buf), nbytes, seed, c->stream));
} NKV_CATCH

}  // extern "C"
