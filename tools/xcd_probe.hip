// xcd_probe.hip -- does the resident service's request round trip depend on
// the XCD its one workgroup lands on?
//
// tools/svc_ab.py showed the service's per-call time changing by up to 4.5 us
// from one launch to the next and staying put within a launch: a placement
// effect.  Here a kernel of 8 workgroups (one per XCD: the dispatcher deals
// workgroups round-robin over the XCDs) reads each workgroup's XCC_ID; only the
// workgroup on the target XCD answers the host's requests, the rest leave at
// once.  For each target XCD and each doorbell place (host-coherent memory, or
// fine-grained device memory the host stores to through the large BAR) it
// reports the median round trip of `iters` requests: doorbell store -> the
// workgroup's poll sees it -> 512 B of output + the acknowledgement into host
// memory -> the host sees it.  Every wait on either side is bounded.
//
//   hipcc --offload-arch=gfx950 -O2 tools/xcd_probe.hip -o tools/xcd_probe.bin
//   tools/xcd_probe.bin [iters]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

constexpr uint32_t kFail = 0xFFFFFFFFu;
// s_getreg_b32 of HW_REG_XCC_ID (id 20 on gfx940+), bits [3:0]
constexpr int kXccIdReg = 20 | (0 << 6) | ((4 - 1) << 11);

__global__ __launch_bounds__(64) void k_xcd_pingpong(const uint32_t* bell, uint32_t* ack, uint4* out,
                                                     uint32_t* ids, uint32_t target, uint32_t iters,
                                                     uint64_t timeout_ticks) {
    const uint32_t xcc = uint32_t(__builtin_amdgcn_s_getreg(kXccIdReg)) & 15u;
    if (threadIdx.x == 0) ids[blockIdx.x] = xcc;
    if (xcc != target) return;  // (two workgroups on one XCD would both answer: same values)
    for (uint32_t k = 1; k <= iters; ++k) {
        const uint64_t t0 = wall_clock64();
        bool give_up = false;
        for (;;) {
            const uint32_t v = uint32_t(__builtin_amdgcn_readfirstlane(
                int(__hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM))));
            if (v == k) break;
            if (wall_clock64() - t0 > timeout_ticks) {
                give_up = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (give_up) {
            if (threadIdx.x == 0) __hip_atomic_store(ack, kFail, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        // 512 B of "output" (a default flush's nodes are ~400 B), then the ack
        if (threadIdx.x < 32) out[threadIdx.x] = make_uint4(k, k, k, xcc);
        if (threadIdx.x == 0) __hip_atomic_store(ack, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double run(uint32_t* bell, uint32_t* d_bell, uint32_t* ack, uint32_t* d_ack, uint4* out_dev, uint32_t* ids, uint32_t target,
                  uint32_t iters, bool wc, bool* ok) {
    volatile uint32_t* vb = bell;
    *vb = 0;
    __atomic_store_n(ack, 0u, __ATOMIC_RELEASE);
    asm volatile("sfence" ::: "memory");
    *ok = false;
    hipLaunchKernelGGL(k_xcd_pingpong, dim3(8), dim3(64), 0, 0, d_bell, d_ack, out_dev, ids, target, iters,
                       uint64_t(200000000));
    if (hipGetLastError() != hipSuccess) return -1;
    std::vector<double> us;
    for (uint32_t k = 1; k <= iters; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(bell, k, __ATOMIC_RELEASE);
        if (wc) asm volatile("sfence" ::: "memory");
        bool failed = false;
        for (;;) {
            const uint32_t a = __atomic_load_n(ack, __ATOMIC_ACQUIRE);
            if (a == k) break;
            if (a == kFail || std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3)) {
                failed = true;
                break;
            }
        }
        if (failed) {
            (void)hipDeviceSynchronize();
            return -1;
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    std::sort(us.begin() + 0, us.end());
    *ok = true;
    return us[us.size() / 2];
}

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? uint32_t(atoi(argv[1])) : 2000;
    CK(hipSetDevice(0));
    uint32_t *hbell = nullptr, *hack = nullptr, *hids = nullptr;
    uint4* hout = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hbell), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hack), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hids), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hout), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    uint32_t* dbell = nullptr;
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&dbell), 4096, hipDeviceMallocFinegrained));
    void *d_hbell, *d_hack, *d_hids, *d_hout;
    CK(hipHostGetDevicePointer(&d_hbell, hbell, 0));
    CK(hipHostGetDevicePointer(&d_hack, hack, 0));
    CK(hipHostGetDevicePointer(&d_hids, hids, 0));
    CK(hipHostGetDevicePointer(&d_hout, hout, 0));
    int rc = 0;
    for (int rep = 0; rep < 2; ++rep) {
        for (uint32_t target = 0; target < 8; ++target) {
            double med[2];
            for (int form = 0; form < 2; ++form) {
                memset(hids, 0xff, 64);
                bool ok = false;
                med[form] = run(form == 0 ? hbell : dbell, form == 0 ? static_cast<uint32_t*>(d_hbell) : dbell, hack, static_cast<uint32_t*>(d_hack),
                                static_cast<uint4*>(d_hout), static_cast<uint32_t*>(d_hids), target, iters, form == 1,
                                &ok);
                if (!ok) {
                    printf("target %u form %d FAILED\n", target, form);
                    fflush(stdout);
                    return 1;
                }
            }
            printf("{\"rep\": %d, \"xcd\": %u, \"bell_host_us\": %.2f, \"bell_device_us\": %.2f, "
                   "\"workgroup_xccs\": [%u, %u, %u, %u, %u, %u, %u, %u]}\n",
                   rep, target, med[0], med[1], hids[0], hids[1], hids[2], hids[3], hids[4], hids[5], hids[6],
                   hids[7]);
            fflush(stdout);
        }
    }
    (void)hipFree(dbell);
    printf("done rc=%d\n", rc);
    return rc;
}
