// launch_floor.hip -- the per-call floor of a small host-buffer Merkle step on
// this box ("The small-flush floor"): what one launch,
// one copy and one completion wait cost before any hashing, beside the
// library's one-launch path (nkv_tree_from_values, NKV_OPT_SMALL_PATH) on the
// reference's default flush (10 values <= 200 B).  Microseconds, median and p10
// / p90 of REPS calls each:
//   launch_sync        empty kernel + hipStreamSynchronize
//   launch_flag        empty kernel that stores a sequence number into
//                      host-coherent pinned memory (system-scope release) +
//                      the host spinning on it (no runtime completion wait)
//   h2d_sync, d2h_sync 1 KiB pinned copy + hipStreamSynchronize
//   event_sync         empty kernel + hipEventRecord + hipEventSynchronize
//   abi_small          nkv_tree_from_values, 10 values, small path
//   abi_grid           the same, NKV_OPT_SMALL_PATH 0
// Usage: launch_floor [REPS]; one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nkv_merkle.h"

using clk = std::chrono::steady_clock;

__global__ void k_empty() {}

__global__ void k_flag(unsigned int* flag, unsigned int seq) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

struct St {
    double med, p10, p90;
};
static St stats(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    auto at = [&](double q) { return v[std::min(v.size() - 1, size_t(q * double(v.size() - 1) + 0.5))]; };
    return {at(0.5), at(0.1), at(0.9)};
}

template <class F>
static St time_us(int reps, F f) {
    for (int i = 0; i < 20; ++i) f(i);
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
        const auto a = clk::now();
        f(i);
        t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
    }
    return stats(t);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned int* hflag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hflag), 64, hipHostMallocCoherent));
    unsigned int* dflag = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), hflag, 0));
    *hflag = 0;
    uint8_t *hbuf = nullptr, *dbuf = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hbuf), 1024, hipHostMallocDefault));
    CK(hipMalloc(reinterpret_cast<void**>(&dbuf), 1024));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));

    const St launch_sync = time_us(reps, [&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        CK(hipStreamSynchronize(s));
    });
    unsigned int seq = 0;
    const St launch_flag = time_us(reps, [&](int) {
        ++seq;
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, dflag, seq);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
    });
    CK(hipStreamSynchronize(s));
    const St event_sync = time_us(reps, [&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
    });
    const St h2d = time_us(reps, [&](int) {
        CK(hipMemcpyAsync(dbuf, hbuf, 1024, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    });
    const St d2h = time_us(reps, [&](int) {
        CK(hipMemcpyAsync(hbuf, dbuf, 1024, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    });

    // the reference's default flush: 10 values of 1..200 bytes
    const uint64_t n = 10;
    std::vector<uint64_t> off(n), len(n);
    uint64_t tot = 0;
    for (uint64_t i = 0; i < n; ++i) {
        len[i] = 1 + (i * 73) % 200;
        off[i] = tot;
        tot += len[i];
    }
    std::vector<uint8_t> vals(tot + 1);
    for (uint64_t j = 0; j < tot; ++j) vals[j] = uint8_t(j * 131 + 7);
    nkv_ctx* ctx = nullptr;
    if (nkv_ctx_create(0, &ctx) != NKV_OK) return 2;
    uint8_t root[20];
    std::vector<uint8_t> nodes(20 * nkv_total_nodes(n)), img(nkv_bfs_size(n));
    auto call = [&](int) {
        if (nkv_tree_from_values(ctx, vals.data(), off.data(), len.data(), n, root, nodes.data(), img.data()) != NKV_OK)
            std::exit(3);
    };
    const St abi_small = time_us(reps, call);
    nkv_ctx_set_option(ctx, NKV_OPT_SMALL_PATH, 0);
    const St abi_grid = time_us(reps, call);
    nkv_ctx_destroy(ctx);

    auto pr = [](const char* k, const St& x, bool last = false) {
        std::printf("\"%s\": [%.2f, %.2f, %.2f]%s", k, x.med, x.p10, x.p90, last ? "" : ", ");
    };
    std::printf("{\"reps\": %d, \"unit\": \"us [median, p10, p90]\", ", reps);
    pr("launch_sync", launch_sync);
    pr("launch_flag", launch_flag);
    pr("event_sync", event_sync);
    pr("h2d_sync", h2d);
    pr("d2h_sync", d2h);
    pr("abi_small", abi_small);
    pr("abi_grid", abi_grid, true);
    std::printf("}\n");
    return 0;
}
