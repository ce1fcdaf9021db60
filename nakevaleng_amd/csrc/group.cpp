// group.cpp -- several tables per call and several GPUs per process (SURVEY.md
// section 8e), behind the C-ABI in include/nkv_merkle.h.
//
// The reference compacts a level by merging its runs into one output table
// (core/lsmtree/lsmtree.go:71-128; leaves collected at :211) and builds that
// table's tree in MakeTableSecondaries (core/sstable/sstable.go:35-47).
// Independent tables are independent trees, so:
//   - nkv_trees_dev spreads the tables of one call over a few streams of one
//     device (the next table's leaf kernel fills the CUs while the previous
//     one drains and reduces);
//   - a group is one host process driving g GPUs: one nkv_ctx per device and
//     one RCCL communicator (ncclCommInitAll); tables go to members round-robin
//     and the only collective is the all-gather of the 20-byte roots;
//   - one table too large for one GPU splits at 2^k-aligned leaf ranges
//     (padding only happens at a level's end, merkletree.go:32-34), the
//     level-k sub-roots are all-gathered and every member reduces the top
//     levels, so every member holds the root.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <exception>
#include <thread>
#include <vector>

#include "context.hpp"

using namespace nkv;

namespace {

// Options a lane inherits from the context it serves (per call: the caller may
// have changed them since the lane was made).
void copy_options(const nkv_ctx* from, nkv_ctx* to) {
    to->leaf_load = from->leaf_load;
    to->bucket = from->bucket;
    to->queue_split = from->queue_split;
    to->queue_waves = from->queue_waves;
    to->crc_load = from->crc_load;
    to->records_fused = from->records_fused;
    if (to->timing != from->timing || to->timing_every != from->timing_every) {
        to->timing = from->timing;
        to->timing_every = from->timing_every;
        to->timed = false;
        to->ring_used = 0;
        to->timing_calls = 0;
    }
}

// One table through its single-table entry on context c (asynchronous; err
// substitutes a device word for a RECORDS table whose err is NULL).
int one_table(nkv_ctx* c, const nkv_table& t, uint32_t* err) {
    switch (t.kind) {
        case NKV_TABLE_STRIDED:
            return nkv_tree_from_strided_dev(c, t.base, t.stride, t.len, t.n, t.nodes);
        case NKV_TABLE_VALUES:
            return nkv_tree_from_values_dev(c, t.base, t.off, t.lens, t.n, t.nodes);
        case NKV_TABLE_RECORDS:
            return nkv_tree_from_records_dev(c, t.base, t.base_len, t.off, t.n, t.nodes, t.err ? t.err : err);
        case NKV_TABLE_VERIFY:
            return nkv_tree_verify_records_dev(c, t.base, t.base_len, t.off, t.n, t.nodes, t.crc, t.stats);
        default:
            return NKV_ERR_INVALID;
    }
}

int make_event(hipEvent_t* e) {
    if (!*e) HIPTRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return NKV_OK;
}

// ptr is device memory of `device` (a table handed to the wrong member would
// make its kernels read another GPU's memory)
bool on_device(const void* p, int device) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.device == device;
}

int nccl_st(ncclResult_t r) { return r == ncclSuccess ? NKV_OK : NKV_ERR_DEVICE; }

// Every pointer the table's kind hands to a kernel lives on `device` (ADVICE
// r03: offsets or stats on another GPU would become peer reads or faults
// instead of NKV_ERR_INVALID).  Optional outputs may be NULL.
bool table_on_device(const nkv_table& t, int device) {
    auto opt = [&](const void* p) { return !p || on_device(p, device); };
    if (!on_device(t.nodes, device) || !on_device(t.base, device)) return false;
    switch (t.kind) {
        case NKV_TABLE_STRIDED:
            return true;
        case NKV_TABLE_VALUES:
            return on_device(t.off, device) && on_device(t.lens, device);
        case NKV_TABLE_RECORDS:
            return on_device(t.off, device) && opt(t.err);
        case NKV_TABLE_VERIFY:
            return on_device(t.off, device) && opt(t.crc) && opt(t.stats);
        default:
            return true;  // the build refuses the kind itself
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// several tables on one device

extern "C" int nkv_trees_dev(nkv_ctx* c, const nkv_table* tables, int k) try {
    TRY(bind(c));
    if (k < 0 || (k > 0 && !tables)) return NKV_ERR_INVALID;
    if (k == 0) return NKV_OK;
    int nrec = 0;  // RECORDS tables without an err word get one of ours
    for (int t = 0; t < k; ++t) nrec += tables[t].kind == NKV_TABLE_RECORDS && !tables[t].err;
    uint32_t* errs = nullptr;
    if (nrec) {
        TRY(grow(c->d_err, 4 * size_t(k)));
        errs = static_cast<uint32_t*>(c->d_err.p);
    }
    const int nl = std::min(k, c->table_lanes);
    int rc = NKV_OK;
    if (nl <= 1) {
        for (int t = 0; t < k && rc == NKV_OK; ++t) rc = one_table(c, tables[t], errs ? errs + t : nullptr);
    } else {
        while (int(c->lanes.size()) < nl) {
            nkv_ctx* l = nullptr;
            TRY(nkv_ctx_create(c->device, &l));
            c->lanes.push_back(l);
            c->join_ev.push_back(nullptr);
        }
        TRY(bind(c));
        TRY(make_event(&c->fork_ev));
        for (int i = 0; i < nl; ++i) TRY(make_event(&c->join_ev[i]));
        HIPTRY(hipEventRecord(c->fork_ev, c->stream));
        for (int i = 0; i < nl; ++i) {
            copy_options(c, c->lanes[i]);
            HIPTRY(hipStreamWaitEvent(c->lanes[i]->stream, c->fork_ev, 0));
        }
        for (int t = 0; t < k && rc == NKV_OK; ++t)
            rc = one_table(c->lanes[t % nl], tables[t], errs ? errs + t : nullptr);
        // join every lane whatever happened: the context's stream orders after
        // all work this call queued
        for (int i = 0; i < nl; ++i) {
            const int jr = st(hipEventRecord(c->join_ev[i], c->lanes[i]->stream));
            const int wr = jr == NKV_OK ? st(hipStreamWaitEvent(c->stream, c->join_ev[i], 0)) : jr;
            if (rc == NKV_OK) rc = wr;
        }
        TRY(bind(c));
    }
    TRY(rc);
    if (nrec) {  // the single-table rule for err == NULL: synchronize and report
        std::vector<uint32_t> h(k);
        HIPTRY(hipMemcpyAsync(h.data(), errs, 4 * size_t(k), hipMemcpyDeviceToHost, c->stream));
        HIPTRY(hipStreamSynchronize(c->stream));
        for (int t = 0; t < k; ++t)
            if (tables[t].kind == NKV_TABLE_RECORDS && !tables[t].err && h[t]) return NKV_ERR_INVALID;
    }
    return NKV_OK;
} NKV_CATCH

// ---------------------------------------------------------------------------
// group

struct nkv_group {
    int g = 0;
    int transport = NKV_TRANSPORT_COPY;
    std::vector<int> dev;
    std::vector<nkv_ctx*> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<DevBuf> slot, gathered;  // per member: roots to send, g x roots received
    std::vector<hipEvent_t> ev, ev2;     // per member (copy transport, split-tree joins)
    // the latest split tree (nkv_group_tree_dev / _from_values); n == 0: none
    // (a refused or failed split call leaves none, so fetch refuses)
    uint64_t n = 0, span = 0, G = 0;
    int k = 0;
    std::vector<uint64_t> nr;      // leaves per member
    std::vector<DevBuf> levels;    // per member: levels 0..k of its range, level-major
    std::vector<DevBuf> top;       // per member: the top tree over the G sub-roots
    DevBuf full, img;              // member 0: the whole tree, its image
    std::vector<int> peer;         // g x g: NKV_PEER_* of member i's device to member j's
};

namespace {

int member_bind(nkv_group* grp, int i) { return st(hipSetDevice(grp->dev[i])); }

// xGMI peer mappings between every pair of the members' GPUs (VERDICT r04 item
// 5): nkv_group_tree_fetch and the copy transport move bytes GPU to GPU with
// hipMemcpyPeerAsync, which without a mapping takes whatever path the runtime
// picks (staged through the host).  A pair already enabled (by another group,
// or by torch in the same process) counts as enabled; a pair the hardware
// cannot map stays NKV_PEER_NONE and its copies still work.  Mappings are
// process-wide and are left in place when the group is destroyed (another
// group of the process may use them).
int enable_peers(nkv_group* grp) {
    const int g = grp->g;
    grp->peer.assign(size_t(g) * g, NKV_PEER_NONE);
    for (int i = 0; i < g; ++i) {
        for (int j = 0; j < g; ++j) {
            int& s = grp->peer[size_t(i) * g + j];
            if (grp->dev[i] == grp->dev[j]) {
                s = NKV_PEER_SAME;
                continue;
            }
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, grp->dev[i], grp->dev[j]) != hipSuccess) {
                (void)hipGetLastError();
                continue;
            }
            if (!can) continue;
            TRY(member_bind(grp, i));
            const hipError_t e = hipDeviceEnablePeerAccess(grp->dev[j], 0);
            if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) s = NKV_PEER_ENABLED;
            (void)hipGetLastError();  // an already-enabled pair leaves its error behind
        }
    }
    return NKV_OK;
}

// bytes from member j's device memory to member i's, on member i's stream (a
// plain device copy when both are the same GPU, else a peer copy over xGMI)
hipError_t copy_between(nkv_group* grp, int i, void* dst, int j, const void* src, size_t bytes) {
    if (grp->dev[i] == grp->dev[j])
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, grp->ctx[i]->stream);
    return hipMemcpyPeerAsync(dst, grp->dev[i], src, grp->dev[j], bytes, grp->ctx[i]->stream);
}

// All-gather `bytes` from src[i] (member i) into dst[i] (g * bytes on member i),
// on the members' streams.
int allgather(nkv_group* grp, const void* const* src, void* const* dst, size_t bytes) {
    const int g = grp->g;
    if (grp->transport == NKV_TRANSPORT_RCCL) {
        TRY(nccl_st(ncclGroupStart()));
        int rc = NKV_OK;
        for (int i = 0; i < g && rc == NKV_OK; ++i) {
            rc = member_bind(grp, i);
            if (rc == NKV_OK)
                rc = nccl_st(ncclAllGather(src[i], dst[i], bytes, ncclUint8, grp->comm[i], grp->ctx[i]->stream));
        }
        const int er = nccl_st(ncclGroupEnd());
        TRY(rc);
        return er;
    }
    // copy transport (a device listed twice): every member's stream first waits
    // for every source, copies, and then every stream waits for every copy
    // before it may overwrite its source
    for (int j = 0; j < g; ++j) {
        TRY(member_bind(grp, j));
        TRY(make_event(&grp->ev[j]));
        HIPTRY(hipEventRecord(grp->ev[j], grp->ctx[j]->stream));
    }
    for (int i = 0; i < g; ++i) {
        TRY(member_bind(grp, i));
        for (int j = 0; j < g; ++j) {
            HIPTRY(hipStreamWaitEvent(grp->ctx[i]->stream, grp->ev[j], 0));
            HIPTRY(copy_between(grp, i, static_cast<uint8_t*>(dst[i]) + bytes * j, j, src[j], bytes));
        }
        TRY(make_event(&grp->ev2[i]));
        HIPTRY(hipEventRecord(grp->ev2[i], grp->ctx[i]->stream));
    }
    for (int j = 0; j < g; ++j) {
        TRY(member_bind(grp, j));
        for (int i = 0; i < g; ++i) HIPTRY(hipStreamWaitEvent(grp->ctx[j]->stream, grp->ev2[i], 0));
    }
    return NKV_OK;
}

int group_sync(nkv_group* grp) {
    for (int i = 0; i < grp->g; ++i) {
        TRY(member_bind(grp, i));
        HIPTRY(hipStreamSynchronize(grp->ctx[i]->stream));
    }
    return NKV_OK;
}

// Nodes in levels 0..k of a range of m leaves (the levels above its natural
// top are its lone node re-hashed, one node each).
uint64_t range_nodes(uint64_t m, int k) { return m ? start_of(m, k + 1) : 0; }

// The split plan for n leaves over g members: span 2^k, G ranges, member r's
// range length.  Computed apart from the group and committed only once the
// call's arguments passed (a refused call must not change the plan
// a later nkv_group_tree_fetch reads).
struct SplitPlan {
    uint64_t n = 0, span = 0, G = 0;
    int k = 0;
    std::vector<uint64_t> nr;
};

SplitPlan split_plan(uint64_t n, int g) {
    SplitPlan p;
    p.n = n;
    p.span = nkv_split_span(n, g);
    while ((uint64_t(1) << p.k) < p.span) ++p.k;
    p.G = (n + p.span - 1) / p.span;
    p.nr.assign(g, 0);
    for (int r = 0; r < g; ++r) {
        const uint64_t lo = std::min(n, uint64_t(r) * p.span);
        p.nr[r] = std::min(n, lo + p.span) - lo;
    }
    return p;
}

void commit_plan(nkv_group* grp, const SplitPlan& p) {
    grp->n = p.n;
    grp->span = p.span;
    grp->k = p.k;
    grp->G = p.G;
    grp->nr = p.nr;
}

// After every member built levels 0..k of its range into levels[r]: all-gather
// the level-k sub-roots and reduce the top ceil(log2 G) levels on EVERY member
// into its own top[r] (every rank computes the top levels; G <= 64
// nodes, one single-wave chain per member, the members' chains run
// concurrently), then put member r's root at d_roots[r] (nullable array and
// entries, each on member r's device) and member 0's at root20 (host, nullable).
int split_top(nkv_group* grp, void* const* d_roots, uint8_t* root20) {
    const int g = grp->g;
    std::vector<const void*> src(g);
    std::vector<void*> dst(g);
    for (int r = 0; r < g; ++r) {
        TRY(member_bind(grp, r));
        TRY(grow(grp->slot[r], 20));
        TRY(grow(grp->gathered[r], 20 * size_t(g)));
        nkv_ctx* c = grp->ctx[r];
        if (grp->nr[r]) {
            const uint8_t* sub = static_cast<const uint8_t*>(grp->levels[r].p) + 20 * start_of(grp->nr[r], grp->k);
            HIPTRY(hipMemcpyAsync(grp->slot[r].p, sub, 20, hipMemcpyDeviceToDevice, c->stream));
        } else {
            HIPTRY(hipMemsetAsync(grp->slot[r].p, 0, 20, c->stream));  // an idle member sends zeros
        }
        // fetch reads the member's levels on member 0's stream after this event
        TRY(make_event(&grp->ev2[r]));
        src[r] = grp->slot[r].p;
        dst[r] = grp->gathered[r].p;
    }
    // (the copy transport records its own events; the RCCL kernels order the
    // streams themselves)
    TRY(allgather(grp, src.data(), dst.data(), 20));
    const uint64_t G = grp->G;
    const uint64_t tn = G == 1 ? 1 : total_of(G);
    for (int r = 0; r < g; ++r) {
        TRY(member_bind(grp, r));
        nkv_ctx* c = grp->ctx[r];
        TRY(grow(grp->top[r], 20 * tn));
        uint8_t* top = static_cast<uint8_t*>(grp->top[r].p);
        HIPTRY(hipMemcpyAsync(top, grp->gathered[r].p, 20 * G, hipMemcpyDeviceToDevice, c->stream));
        if (G > 1) HIPTRY(launch_reduce(top, G, 0, levels_of(G) - 1, c->stream));
        if (d_roots && d_roots[r])
            HIPTRY(hipMemcpyAsync(d_roots[r], top + 20 * (tn - 1), 20, hipMemcpyDeviceToDevice, c->stream));
    }
    TRY(member_bind(grp, 0));
    nkv_ctx* c0 = grp->ctx[0];
    const uint8_t* root = static_cast<const uint8_t*>(grp->top[0].p) + 20 * (tn - 1);
    if (root20) {
        HIPTRY(hipMemcpyAsync(c0->h_small, root, 20, hipMemcpyDeviceToHost, c0->stream));
        HIPTRY(hipStreamSynchronize(c0->stream));
        memcpy(root20, c0->h_small, 20);
    }
    return NKV_OK;
}

// Member r's levels 0..k from its leaves already on its device (kind STRIDED:
// base/stride/len; VALUES: base/off/lens), on its stream.
int build_range(nkv_group* grp, int r, const nkv_table& t, bool aligned, const uint64_t* host_len) {
    nkv_ctx* c = grp->ctx[r];
    const uint64_t m = grp->nr[r];
    TRY(grow(grp->levels[r], 20 * range_nodes(m, grp->k)));
    uint8_t* lv = static_cast<uint8_t*>(grp->levels[r].p);
    TRY(mark(c, 0));
    if (t.kind == NKV_TABLE_STRIDED) {
        if (!t.base) return NKV_ERR_INVALID;
        HIPTRY(launch_leaf_strided(static_cast<const uint8_t*>(t.base), t.stride, t.len, m, c->leaf_load, lv,
                                   c->stream));
    } else if (t.kind == NKV_TABLE_VALUES) {
        if (!t.base || !t.off || !t.lens) return NKV_ERR_INVALID;
        TRY(leaf_level(c, static_cast<const uint8_t*>(t.base), t.off, t.lens, m, aligned, lv, host_len));
    } else {
        return NKV_ERR_INVALID;
    }
    TRY(mark(c, 1));
    // k >= the range's natural top: the levels above it re-hash the lone node
    HIPTRY(launch_reduce(lv, m, 0, grp->k, c->stream));
    return mark(c, 2);
}

}  // namespace

extern "C" {

uint64_t nkv_split_span(uint64_t n, int g) {
    if (n == 0 || g < 1) return 0;
    const uint64_t per = (n + uint64_t(g) - 1) / uint64_t(g);
    int k = 1;
    while ((uint64_t(1) << k) < per) ++k;
    return uint64_t(1) << k;
}

int nkv_group_create(const int* devices, int g, nkv_group** out) try {
    if (!out) return NKV_ERR_INVALID;
    *out = nullptr;
    if (!devices || g < 1 || g > 64) return NKV_ERR_INVALID;
    int cnt = 0;
    if (nkv_device_count(&cnt) != NKV_OK) return NKV_ERR_DEVICE;
    for (int i = 0; i < g; ++i)
        if (devices[i] < 0 || devices[i] >= cnt) return NKV_ERR_DEVICE;
    nkv_group* grp = new nkv_group();
    grp->g = g;
    grp->dev.assign(devices, devices + g);
    grp->ctx.assign(g, nullptr);
    grp->slot.resize(g);
    grp->gathered.resize(g);
    grp->levels.resize(g);
    grp->top.resize(g);
    grp->ev.assign(g, nullptr);
    grp->ev2.assign(g, nullptr);
    int rc = NKV_OK;
    for (int i = 0; i < g && rc == NKV_OK; ++i) rc = nkv_ctx_create(devices[i], &grp->ctx[i]);
    std::vector<int> sorted(grp->dev);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (rc == NKV_OK && distinct) {
        grp->comm.assign(g, nullptr);
        rc = nccl_st(ncclCommInitAll(grp->comm.data(), g, grp->dev.data()));
        if (rc != NKV_OK) grp->comm.clear();
        grp->transport = NKV_TRANSPORT_RCCL;
    }
    if (rc == NKV_OK) rc = enable_peers(grp);  // after RCCL's own setup (it may have enabled them)
    if (rc != NKV_OK) {
        nkv_group_destroy(grp);
        return rc;
    }
    *out = grp;
    return NKV_OK;
} NKV_CATCH

void nkv_group_destroy(nkv_group* grp) {
    if (!grp) return;
    for (int i = 0; i < grp->g; ++i) {
        if (!grp->ctx[i]) continue;
        (void)hipSetDevice(grp->dev[i]);
        (void)hipStreamSynchronize(grp->ctx[i]->stream);
    }
    for (ncclComm_t cm : grp->comm)
        if (cm) (void)ncclCommDestroy(cm);
    for (int i = 0; i < grp->g; ++i) {
        (void)hipSetDevice(grp->dev[i]);
        for (DevBuf* b : {&grp->slot[i], &grp->gathered[i], &grp->levels[i], &grp->top[i]})
            if (b->p) (void)hipFree(b->p);
        if (grp->ev[i]) (void)hipEventDestroy(grp->ev[i]);
        if (grp->ev2[i]) (void)hipEventDestroy(grp->ev2[i]);
    }
    if (!grp->dev.empty()) {
        (void)hipSetDevice(grp->dev[0]);
        for (DevBuf* b : {&grp->full, &grp->img})
            if (b->p) (void)hipFree(b->p);
    }
    for (nkv_ctx* c : grp->ctx) nkv_ctx_destroy(c);
    delete grp;
}

int nkv_group_peer_access(const nkv_group* grp, int i, int j, int* state) try {
    if (!grp || !state || i < 0 || j < 0 || i >= grp->g || j >= grp->g) return NKV_ERR_INVALID;
    *state = grp->peer[size_t(i) * grp->g + j];
    return NKV_OK;
} NKV_CATCH

int nkv_group_size(const nkv_group* grp) { return grp ? grp->g : 0; }

int nkv_group_transport(const nkv_group* grp) { return grp ? grp->transport : 0; }

int nkv_group_ctx(nkv_group* grp, int i, nkv_ctx** out) try {
    if (!grp || !out || i < 0 || i >= grp->g) return NKV_ERR_INVALID;
    *out = grp->ctx[i];
    return NKV_OK;
} NKV_CATCH

int nkv_group_sync(nkv_group* grp) try {
    if (!grp) return NKV_ERR_INVALID;
    return group_sync(grp);
} NKV_CATCH

int nkv_group_roots_allgather(nkv_group* grp, const void* const* d_roots, void* const* d_out,
                              uint8_t* roots_out) try {
    if (!grp || !d_roots) return NKV_ERR_INVALID;
    const int g = grp->g;
    std::vector<void*> dst(g);
    for (int i = 0; i < g; ++i) {
        // each member's buffers must live on its device (RCCL and the copies
        // read and write them there)
        if (!on_device(d_roots[i], grp->dev[i])) return NKV_ERR_INVALID;
        if (d_out && d_out[i] && !on_device(d_out[i], grp->dev[i])) return NKV_ERR_INVALID;
        if (d_out && d_out[i]) {
            dst[i] = d_out[i];
        } else {
            TRY(member_bind(grp, i));
            TRY(grow(grp->gathered[i], 20 * size_t(g)));
            dst[i] = grp->gathered[i].p;
        }
    }
    TRY(allgather(grp, d_roots, dst.data(), 20));
    if (roots_out) {
        TRY(member_bind(grp, 0));
        HIPTRY(hipMemcpyAsync(roots_out, dst[0], 20 * size_t(g), hipMemcpyDeviceToHost, grp->ctx[0]->stream));
        HIPTRY(hipStreamSynchronize(grp->ctx[0]->stream));
    }
    return NKV_OK;
} NKV_CATCH

int nkv_group_trees_dev(nkv_group* grp, const nkv_table* tables, int k, uint8_t* roots_out) try {
    if (!grp || k < 0 || (k > 0 && !tables)) return NKV_ERR_INVALID;
    if (k == 0) return NKV_OK;
    const int g = grp->g;
    for (int t = 0; t < k; ++t)
        if (!table_on_device(tables[t], grp->dev[t % g])) return NKV_ERR_INVALID;
    const int per = (k + g - 1) / g;  // roots per member (the last slots of some stay unused)
    std::vector<const void*> src(g);
    std::vector<void*> dst(g);
    for (int m = 0; m < g; ++m) {
        std::vector<nkv_table> mine;
        for (int t = m; t < k; t += g) mine.push_back(tables[t]);
        nkv_ctx* c = grp->ctx[m];
        TRY(member_bind(grp, m));
        TRY(grow(grp->slot[m], 20 * size_t(per)));
        TRY(grow(grp->gathered[m], 20 * size_t(per) * size_t(g)));
        if (!mine.empty()) TRY(nkv_trees_dev(c, mine.data(), int(mine.size())));
        TRY(member_bind(grp, m));
        uint8_t* slot = static_cast<uint8_t*>(grp->slot[m].p);
        for (size_t j = 0; j < mine.size(); ++j) {
            const uint8_t* root = static_cast<const uint8_t*>(mine[j].nodes) + 20 * (total_of(mine[j].n) - 1);
            HIPTRY(hipMemcpyAsync(slot + 20 * j, root, 20, hipMemcpyDeviceToDevice, c->stream));
        }
        if (int(mine.size()) < per)
            HIPTRY(hipMemsetAsync(slot + 20 * mine.size(), 0, 20 * (per - mine.size()), c->stream));
        src[m] = grp->slot[m].p;
        dst[m] = grp->gathered[m].p;
    }
    TRY(allgather(grp, src.data(), dst.data(), 20 * size_t(per)));
    if (roots_out) {
        TRY(member_bind(grp, 0));
        std::vector<uint8_t> h(20 * size_t(per) * size_t(g));
        HIPTRY(hipMemcpyAsync(h.data(), dst[0], h.size(), hipMemcpyDeviceToHost, grp->ctx[0]->stream));
        HIPTRY(hipStreamSynchronize(grp->ctx[0]->stream));
        for (int t = 0; t < k; ++t)  // member t % g, its slot t / g
            memcpy(roots_out + 20 * size_t(t), h.data() + 20 * (size_t(t % g) * per + t / g), 20);
    }
    return NKV_OK;
} NKV_CATCH

int nkv_group_trees_from_values(nkv_group* grp, const nkv_values* tables, int k) try {
    if (!grp || k < 0 || (k > 0 && !tables)) return NKV_ERR_INVALID;
    const int g = std::min(grp->g, k);
    std::vector<int> rc(g, NKV_OK);
    // one host thread per member: each stages and builds its own tables (the
    // staging of one GPU overlaps the others'); roots come back per table
    auto work = [&](int m) {
        try {
            for (int t = m; t < k && rc[m] == NKV_OK; t += grp->g) {
                const nkv_values& v = tables[t];
                rc[m] = nkv_tree_from_values(grp->ctx[m], v.base, v.off, v.len, v.n, v.root20, v.nodes_out,
                                             v.img_out);
            }
        } catch (const std::bad_alloc&) {
            rc[m] = NKV_ERR_NOMEM;
        } catch (...) {
            rc[m] = NKV_ERR_DEVICE;
        }
    };
    std::vector<std::thread> th;
    for (int m = 1; m < g; ++m) th.emplace_back(work, m);
    if (g > 0) work(0);
    for (auto& x : th) x.join();
    for (int m = 0; m < g; ++m) TRY(rc[m]);
    return NKV_OK;
} NKV_CATCH

int nkv_group_tree_dev(nkv_group* grp, const nkv_table* parts, uint64_t n, void* const* d_roots,
                       uint8_t* root20) try {
    if (!grp) return NKV_ERR_INVALID;
    grp->n = 0;  // this call replaces the latest tree, refused or not (fetch then refuses)
    if (!parts) return NKV_ERR_INVALID;
    if (n == 0) return NKV_ERR_EMPTY;
    if (n > kMaxN * uint64_t(grp->g)) return NKV_ERR_INVALID;
    const SplitPlan plan = split_plan(n, grp->g);
    for (int r = 0; r < grp->g; ++r) {
        if (parts[r].n != plan.nr[r]) return NKV_ERR_INVALID;
        if (plan.nr[r]) {
            if (parts[r].kind != NKV_TABLE_STRIDED && parts[r].kind != NKV_TABLE_VALUES) return NKV_ERR_INVALID;
            nkv_table t = parts[r];
            t.nodes = const_cast<void*>(t.base);  // nodes are the group's: check the rest
            if (!table_on_device(t, grp->dev[r])) return NKV_ERR_INVALID;
        }
        if (d_roots && d_roots[r] && !on_device(d_roots[r], grp->dev[r])) return NKV_ERR_INVALID;
    }
    commit_plan(grp, plan);
    grp->n = 0;  // until the whole tree stands
    int rc = NKV_OK;
    for (int r = 0; r < grp->g && rc == NKV_OK; ++r) {
        if (!grp->nr[r]) continue;
        rc = member_bind(grp, r);
        if (rc == NKV_OK) rc = build_range(grp, r, parts[r], false, nullptr);
    }
    if (rc == NKV_OK) rc = split_top(grp, d_roots, root20);
    if (rc == NKV_OK) grp->n = n;
    return rc;
} NKV_CATCH

int nkv_group_tree_from_values(nkv_group* grp, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                               uint64_t n, uint8_t* root20, uint8_t* nodes_out, uint8_t* img_out) try {
    if (!grp) return NKV_ERR_INVALID;
    grp->n = 0;  // set again once the whole tree stands
    if (n == 0) return NKV_ERR_EMPTY;
    if (!base || !off || !len) return NKV_ERR_INVALID;
    if (n > kMaxN * uint64_t(grp->g)) return NKV_ERR_INVALID;
    commit_plan(grp, split_plan(n, grp->g));
    grp->n = 0;
    const int g = grp->g;
    std::vector<int> rc(g, NKV_OK);
    // one host thread per member stages its leaf range and builds its levels
    auto work = [&](int r) {
        try {
            const uint64_t m = grp->nr[r];
            if (!m) return;
            nkv_ctx* c = grp->ctx[r];
            rc[r] = bind(c);
            const uint64_t lo = uint64_t(r) * grp->span;
            const uint8_t* d_base = nullptr;
            bool aligned = true;
            if (rc[r] == NKV_OK) rc[r] = stage_values(c, base, off + lo, len + lo, m, &d_base, &aligned);
            nkv_table t{};
            t.kind = NKV_TABLE_VALUES;
            t.base = d_base;
            t.off = static_cast<const uint64_t*>(c->d_off.p);
            t.lens = static_cast<const uint64_t*>(c->d_len.p);
            t.n = m;
            if (rc[r] == NKV_OK) rc[r] = build_range(grp, r, t, aligned, len + lo);
        } catch (const std::bad_alloc&) {
            rc[r] = NKV_ERR_NOMEM;
        } catch (...) {
            rc[r] = NKV_ERR_DEVICE;
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < g; ++r) th.emplace_back(work, r);
    work(0);
    for (auto& x : th) x.join();
    for (int r = 0; r < g; ++r) TRY(rc[r]);
    TRY(split_top(grp, nullptr, root20));
    grp->n = n;
    if (nodes_out || img_out) {
        const int fr = nkv_group_tree_fetch(grp, nodes_out, img_out);
        if (fr != NKV_OK) {
            grp->n = 0;
            return fr;
        }
    }
    return group_sync(grp);
} NKV_CATCH

int nkv_group_tree_fetch(nkv_group* grp, uint8_t* nodes_out, uint8_t* img_out) try {
    if (!grp) return NKV_ERR_INVALID;
    if (grp->n == 0) return NKV_ERR_INVALID;  // no split tree built yet
    if (!nodes_out && !img_out) return NKV_OK;
    const uint64_t n = grp->n;
    const int k = grp->k;
    // assemble the whole tree, level-major, on member 0: levels 0..k from every
    // member's range (xGMI peer copies), the levels above from the top tree
    for (int r = 0; r < grp->g; ++r) {
        TRY(member_bind(grp, r));
        HIPTRY(hipEventRecord(grp->ev2[r], grp->ctx[r]->stream));
    }
    TRY(member_bind(grp, 0));
    nkv_ctx* c0 = grp->ctx[0];
    TRY(grow(grp->full, 20 * total_of(n)));
    uint8_t* full = static_cast<uint8_t*>(grp->full.p);
    for (int r = 0; r < grp->g; ++r) {
        const uint64_t m = grp->nr[r];
        if (!m) continue;
        HIPTRY(hipStreamWaitEvent(c0->stream, grp->ev2[r], 0));
        const uint8_t* lv = static_cast<const uint8_t*>(grp->levels[r].p);
        for (int L = 0; L <= k; ++L) {
            const uint64_t dst = start_of(n, L) + uint64_t(r) * (grp->span >> L);
            HIPTRY(copy_between(grp, 0, full + 20 * dst, r, lv + 20 * start_of(m, L), 20 * count_of(m, L)));
        }
    }
    if (grp->G > 1) {
        const uint8_t* top = static_cast<const uint8_t*>(grp->top[0].p);
        for (int L = k + 1; L < levels_of(n); ++L)
            HIPTRY(hipMemcpyAsync(full + 20 * start_of(n, L), top + 20 * start_of(grp->G, L - k),
                                  20 * count_of(grp->G, L - k), hipMemcpyDeviceToDevice, c0->stream));
    }
    if (img_out) {
        const BfsLayout lay = layout_of(counts_of(n));
        TRY(grow(grp->img, lay.total));
        HIPTRY(launch_bfs_image(full, lay, static_cast<uint8_t*>(grp->img.p), c0->stream));
        HIPTRY(c0->stage.download(img_out, static_cast<const uint8_t*>(grp->img.p), lay.total, c0->stream));
    }
    if (nodes_out) HIPTRY(c0->stage.download(nodes_out, full, 20 * total_of(n), c0->stream));
    HIPTRY(hipStreamSynchronize(c0->stream));
    return NKV_OK;
} NKV_CATCH

}  // extern "C"
