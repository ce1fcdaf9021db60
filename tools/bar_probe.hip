// bar_probe.hip -- can the host write the resident service's doorbell and input
// straight into device memory, and does that shorten a request's round trip?
//
// The service (k_small_service, NKV_OPT_SMALL_PATH 3) polls a host-coherent
// mailbox across PCIe and reads its input from host memory: one PCIe read round
// trip per poll and one for the input (DESIGN section 5, 3.4 us of a default
// flush's 14.8 on the device).  If fine-grained device memory is mapped into the
// host's address space (a large BAR), the host's stores reach HBM as posted
// writes and the kernel polls and reads local memory instead.
//
// Modes, each a ping-pong of `iters` requests against one resident workgroup:
//   host:   doorbell + input in host-coherent memory (the current form)
//   device: doorbell + input in fine-grained device memory written by the host
// For each: input 0 B (doorbell only) and 4 KiB (256 threads x 16 B, xor-folded
// into the acknowledgement, which the host checks).  The acknowledgement always
// goes to host memory.  Every wait on either side is bounded.
//
//   hipcc --offload-arch=gfx950 -O2 tools/bar_probe.hip -o tools/bar_probe.bin -lhsa-runtime64
//   tools/bar_probe.bin [iters]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <x86intrin.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr uint32_t kFail = 0xFFFFFFFFu;

// One 256-thread workgroup serving `iters` requests: every wave polls the
// doorbell with a wave-uniform test, a barrier, then each thread reads its 16 B
// of the input, the words are xor-folded in LDS and thread 0 acknowledges
// (seq in ack[0], the fold in ack[1]) behind one system release.
__global__ __launch_bounds__(256) void k_pingpong(const uint32_t* bell, const uint4* in, uint32_t in_words,
                                                  uint32_t* ack, uint32_t iters, uint64_t timeout_ticks) {
    __shared__ uint32_t fold;
    __shared__ uint32_t give_up;
    for (uint32_t k = 1; k <= iters; ++k) {
        if (threadIdx.x == 0) {
            fold = 0;
            give_up = 0;
        }
        __syncthreads();
        const uint64_t t0 = wall_clock64();
        for (;;) {
            const uint32_t b = uint32_t(__builtin_amdgcn_readfirstlane(
                int(__hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM))));
            if (b == k) break;
            if (wall_clock64() - t0 > timeout_ticks) {
                give_up = 1;  // every lane of every wave writes the same value
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();
        if (give_up) {
            if (threadIdx.x == 0) __hip_atomic_store(ack, kFail, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        if (threadIdx.x < in_words) {
            const uint4 v = in[threadIdx.x];
            atomicXor(&fold, v.x ^ v.y ^ v.z ^ v.w);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(ack + 1, fold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(ack, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

// The CPU agent (to grant it access to a device allocation).
static hsa_status_t find_cpu(hsa_agent_t a, void* data) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        *static_cast<hsa_agent_t*>(data) = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

// Can this process's CPU store to and load from p?  (A fault is caught.)
static bool host_can_touch(volatile uint32_t* p) {
    struct sigaction sa, old_segv, old_bus;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_jb, 1) == 0) {
        p[0] = 0x12345678u;
        _mm_sfence();
        ok = p[0] == 0x12345678u;
        p[0] = 0;
        _mm_sfence();
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

static int run(const char* name, uint32_t* bell, uint32_t* in_host_view, const uint4* in_dev_view, uint32_t* ack,
               uint32_t iters, uint32_t in_words, bool wc) {
    volatile uint32_t* vb = bell;
    volatile uint32_t* va = ack;
    *vb = 0;
    va[0] = 0;
    va[1] = 0;
    _mm_sfence();
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // 2 s per request on the device side, 5 s on the host side
    hipLaunchKernelGGL(k_pingpong, dim3(1), dim3(256), 0, s, bell, in_dev_view, in_words, ack, iters,
                       uint64_t(200000000));
    CK(hipGetLastError());
    std::vector<double> us;
    us.reserve(iters);
    uint32_t x = 0x9e3779b9u, bad = 0;
    static uint32_t buf[1024];
    bool failed = false;
    for (uint32_t k = 1; k <= iters; ++k) {
        uint32_t want = 0;
        for (uint32_t i = 0; i < 4 * in_words; ++i) {  // fresh input every request
            x = x * 1664525u + 1013904223u;
            want ^= x;
            buf[i] = x;
        }
        // timed: the copy into the mailbox's input (as the service's host side
        // packs it), the doorbell, the wait for the acknowledgement
        const auto t0 = std::chrono::steady_clock::now();
        if (in_words) memcpy(in_host_view, buf, 16 * in_words);
        if (wc) _mm_sfence();  // the input lands before the doorbell (write-combined mapping)
        __atomic_store_n(bell, k, __ATOMIC_RELEASE);
        if (wc) _mm_sfence();
        for (;;) {
            const uint32_t a = __atomic_load_n(ack, __ATOMIC_ACQUIRE);
            if (a == k) break;
            if (a == kFail ||
                std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                failed = true;
                break;
            }
        }
        if (failed) break;
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        if (va[1] != want) ++bad;
    }
    if (failed) {
        printf("%s in=%u B: FAILED after %zu requests (device gave up or host timed out)\n", name, 16 * in_words,
               us.size());
        fflush(stdout);
        // the kernel leaves on its own timeout; wait for it
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
        return 1;
    }
    CK(hipStreamSynchronize(s));
    CK(hipStreamDestroy(s));
    std::vector<double> v(us.begin() + std::min<size_t>(50, us.size() / 4), us.end());
    std::sort(v.begin(), v.end());
    printf("{\"mode\": \"%s\", \"input_bytes\": %u, \"requests\": %u, \"round_trip_us\": {\"p10\": %.2f, "
           "\"median\": %.2f, \"p90\": %.2f}, \"bad_folds\": %u}\n",
           name, 16 * in_words, iters, v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], bad);
    fflush(stdout);
    return bad ? 1 : 0;
}

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? uint32_t(atoi(argv[1])) : 2000;
    CK(hipSetDevice(0));
    // host-coherent mailbox, input and acknowledgement (the service's current form)
    uint32_t *hbell = nullptr, *hin = nullptr, *hack = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hbell), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hin), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hack), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    void *dbell_h = nullptr, *din_h = nullptr;
    CK(hipHostGetDevicePointer(&dbell_h, hbell, 0));
    CK(hipHostGetDevicePointer(&din_h, hin, 0));
    int rc = 0;
    for (uint32_t words : {0u, 256u})
        rc |= run("host", hbell, hin, static_cast<const uint4*>(din_h), hack, iters, words, false);

    // fine-grained device memory, granted to the CPU agent
    uint32_t *dbell = nullptr, *din = nullptr;
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&dbell), 4096, hipDeviceMallocFinegrained));
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&din), 4096, hipDeviceMallocFinegrained));
    hipPointerAttribute_t at;
    CK(hipPointerGetAttributes(&at, dbell));
    printf("device bell %p: type %d, device %d, hostPointer %p, devicePointer %p\n", (void*)dbell, int(at.type),
           at.device, at.hostPointer, at.devicePointer);
    int large_bar = -1;
    CK(hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, 0));
    {
        hsa_amd_pointer_info_t info;
        memset(&info, 0, sizeof info);
        info.size = sizeof info;
        uint32_t na = 0;
        hsa_agent_t* acc = nullptr;
        hsa_status_t st = hsa_amd_pointer_info(dbell, &info, malloc, &na, &acc);
        int ncpu = 0;
        for (uint32_t i = 0; i < na; ++i) {
            hsa_device_type_t t;
            if (hsa_agent_get_info(acc[i], HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU)
                ++ncpu;
        }
        free(acc);
        printf("isLargeBar %d; hsa_amd_pointer_info %d: type %d, agentBase %p, hostBase %p, size %zu, "
               "accessible agents %u (cpu %d)\n",
               large_bar, int(st), int(info.type), info.agentBaseAddress, info.hostBaseAddress, info.sizeInBytes, na,
               ncpu);
    }
    bool touch = host_can_touch(dbell);
    printf("host store/load on the device allocation before any grant: %s\n", touch ? "ok" : "fault");
    if (!touch) {
        hsa_agent_t cpu{0};
        hsa_status_t st = hsa_iterate_agents(find_cpu, &cpu);
        printf("cpu agent: %s\n", cpu.handle ? "found" : "missing");
        if (cpu.handle) {
            hsa_status_t s1 = hsa_amd_agents_allow_access(1, &cpu, nullptr, dbell);
            hsa_status_t s2 = hsa_amd_agents_allow_access(1, &cpu, nullptr, din);
            printf("hsa_amd_agents_allow_access: %d %d (iterate %d)\n", int(s1), int(s2), int(st));
            touch = s1 == HSA_STATUS_SUCCESS && s2 == HSA_STATUS_SUCCESS && host_can_touch(dbell) &&
                    host_can_touch(din);
            printf("host store/load after the grant: %s\n", touch ? "ok" : "fault");
        }
    }
    fflush(stdout);
    if (touch) {
        for (uint32_t words : {0u, 256u})
            rc |= run("device", dbell, din, reinterpret_cast<const uint4*>(din), hack, iters, words, true);
        // mixed: the doorbell in host memory, the input in device memory, and the reverse
        rc |= run("bell_host_input_device", hbell, din, reinterpret_cast<const uint4*>(din), hack, iters, 256, true);
        rc |= run("bell_device_input_host", dbell, hin, static_cast<const uint4*>(din_h), hack, iters, 256, true);
    }
    (void)hipFree(dbell);
    (void)hipFree(din);
    (void)hipHostFree(hbell);
    (void)hipHostFree(hin);
    (void)hipHostFree(hack);
    printf("done rc=%d\n", rc);
    return rc;
}
