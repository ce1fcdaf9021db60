// cu_speed.hip -- does a lone wave's SHA-1 chain run at the same speed on
// every CU?
//
// tools/svc_ab.py found the resident service's compute phases (leaves, levels:
// LDS and VALU only, no instruction-cache misses by the SQC counters) taking
// 5.5 to 7.3 us for the same request depending on the CU its workgroup landed
// on, at one shader clock by s_memtime.  Here one 64-lane workgroup per CU
// (96 KiB of LDS each, so no two share a CU) runs the same dependent chain of
// SHA-1 compressions and reports its wall time (s_memrealtime, 100 MHz), its
// s_memtime cycles and where it ran (HW_ID, XCC_ID); the host prints the
// distribution over CUs.
//
//   hipcc --offload-arch=gfx950 -O3 tools/cu_speed.hip -o tools/cu_speed.bin
//   tools/cu_speed.bin [rounds] [passes]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <map>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

constexpr int kHwId = 4 | (0 << 6) | (31 << 11);
constexpr int kXccId = 20 | (0 << 6) | (15 << 11);

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_rotateleft32(x, n); }

// one SHA-1 compression of w[16] into h[5]
__device__ __forceinline__ void compress(uint32_t h[5], const uint32_t m[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = m[i];
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(w[(t + 13) & 15] ^ w[(t + 8) & 15] ^ w[(t + 2) & 15] ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) {
            f = (b & c) | (~b & d);
            k = 0x5A827999u;
        } else if (t < 40) {
            f = b ^ c ^ d;
            k = 0x6ED9EBA1u;
        } else if (t < 60) {
            f = (b & c) | (b & d) | (c & d);
            k = 0x8F1BBCDCu;
        } else {
            f = b ^ c ^ d;
            k = 0xCA62C1D6u;
        }
        const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
}

struct Rec {
    uint32_t hw, xcc, sink, pad;
    uint64_t rt, mt;
};

// MODE 0: the block stays in registers; 1: each block is read from LDS with ds
// loads; 2: the same LDS bytes through a generic pointer (flat loads, as the
// small-tree kernels read their staged values); the block's place depends on
// the previous digest, so it is a chain either way.
template <int MODE>
__global__ __launch_bounds__(64) void k_chain(Rec* out, uint32_t rounds, const uint4* not_lds) {
    extern __shared__ uint4 lds4[];  // 96 KiB: one workgroup per CU
    uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u ^ threadIdx.x};
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 16u + uint32_t(i);
    for (uint32_t i = threadIdx.x; i < 4096; i += 64) lds4[i] = make_uint4(i, i * 3u, i * 5u, i * 7u);
    if (threadIdx.x == 0) lds[0] = 1;
    __syncthreads();
    // generic view of LDS (the compiler cannot tell: not_lds is null at run time)
    const uint4* gen = not_lds ? not_lds : lds4;
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t mt0 = __builtin_amdgcn_s_memtime();
    for (uint32_t r = 0; r < rounds; ++r) {
        if (MODE != 0) {
            const uint32_t at = ((h[0] + threadIdx.x) & 63u) * 4u;
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = MODE == 1 ? lds4[at + k] : gen[at + k];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                m[4 * k] = v[k].x;
                m[4 * k + 1] = v[k].y;
                m[4 * k + 2] = v[k].z;
                m[4 * k + 3] = v[k].w;
            }
        }
        compress(h, m);
        m[r & 15] ^= h[0];  // the next block depends on this one: a chain
    }
    const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t mt1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        Rec r;
        r.hw = uint32_t(__builtin_amdgcn_s_getreg(kHwId));
        r.xcc = uint32_t(__builtin_amdgcn_s_getreg(kXccId));
        r.sink = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4] ^ lds[0];
        r.pad = 0;
        r.rt = rt1 - rt0;
        r.mt = mt1 - mt0;
        out[blockIdx.x] = r;
    }
}

int main(int argc, char** argv) {
    const uint32_t rounds = argc > 1 ? uint32_t(atoi(argv[1])) : 400;
    const int passes = argc > 2 ? atoi(argv[2]) : 3;
    CK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int G = prop.multiProcessorCount;
    const size_t lds = 96 * 1024;
    for (const void* f : {reinterpret_cast<const void*>(k_chain<0>), reinterpret_cast<const void*>(k_chain<1>),
                          reinterpret_cast<const void*>(k_chain<2>)})
        CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    Rec* d = nullptr;
    CK(hipMalloc(&d, sizeof(Rec) * G));
    std::vector<Rec> h(G);
    printf("CUs %d, rounds %u per lane (dependent SHA-1 compressions)\n", G, rounds);
    for (int p = 0; p < passes; ++p) {
        CK(hipMemset(d, 0, sizeof(Rec) * G));
        hipLaunchKernelGGL(k_chain<0>, dim3(G), dim3(64), lds, 0, d, rounds, nullptr);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), d, sizeof(Rec) * G, hipMemcpyDeviceToHost));
        std::vector<double> us(G), cyc(G);
        for (int i = 0; i < G; ++i) {
            us[i] = h[i].rt / 100.0;
            cyc[i] = double(h[i].mt) / rounds;
        }
        std::vector<double> s = us;
        std::sort(s.begin(), s.end());
        printf("pass %d: us per workgroup min %.1f p10 %.1f median %.1f p90 %.1f max %.1f; "
               "s_memtime cycles per compression min %.0f max %.0f\n",
               p, s[0], s[G / 10], s[G / 2], s[G * 9 / 10], s[G - 1], *std::min_element(cyc.begin(), cyc.end()),
               *std::max_element(cyc.begin(), cyc.end()));
        // by CU id within its shader array, and by XCD
        std::map<int, std::vector<double>> by_cu, by_xcc;
        for (int i = 0; i < G; ++i) {
            by_cu[(h[i].hw >> 8) & 15].push_back(us[i]);
            by_xcc[h[i].xcc & 15].push_back(us[i]);
        }
        printf("  by CU id:");
        for (auto& kv : by_cu) {
            std::sort(kv.second.begin(), kv.second.end());
            printf(" %d:%.1f(n%zu)", kv.first, kv.second[kv.second.size() / 2], kv.second.size());
        }
        printf("\n  by XCD:");
        for (auto& kv : by_xcc) {
            std::sort(kv.second.begin(), kv.second.end());
            printf(" %d:%.1f..%.1f", kv.first, kv.second.front(), kv.second.back());
        }
        printf("\n");
        if (p == passes - 1) {
            printf("  XCD 0 workgroups (se sh cu : us):");
            for (int i = 0; i < G; ++i)
                if ((h[i].xcc & 15) == 0)
                    printf(" %u.%u.%u:%.1f", (h[i].hw >> 13) & 7, (h[i].hw >> 12) & 1, (h[i].hw >> 8) & 15, us[i]);
            printf("\n");
        }
        fflush(stdout);
    }
    // lone workgroups, one launch at a time (the resident service's case: one
    // busy CU on an idle GPU): time and place of each
    printf("lone workgroups (launch: mode xcc.se.sh.cu simd : us, s_memtime cycles per compression):\n");
    for (int l = 0; l < 48; ++l) {
        const int mode = l % 3;
        if (mode == 0) hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), lds, 0, d, rounds, nullptr);
        if (mode == 1) hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), lds, 0, d, rounds, nullptr);
        if (mode == 2) hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), lds, 0, d, rounds, nullptr);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        Rec r;
        CK(hipMemcpy(&r, d, sizeof r, hipMemcpyDeviceToHost));
        printf("  %d: mode %d %u.%u.%u.%u s%u : %.1f us, %.0f\n", l, mode, r.xcc & 15, (r.hw >> 13) & 7, (r.hw >> 12) & 1,
               (r.hw >> 8) & 15, (r.hw >> 4) & 3, r.rt / 100.0, double(r.mt) / rounds);
        fflush(stdout);
    }
    (void)hipFree(d);
    printf("done\n");
    return 0;
}
