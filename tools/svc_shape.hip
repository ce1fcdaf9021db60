// svc_shape.hip -- which part of the resident service's shape makes its compute
// time depend on the CU it lands on?
//
// tools/svc_ab.py: the service's leaves + levels take 11.3-14.6 us for the same
// request, fixed per launch, ordered by the CU (HW_ID); tools/cu_speed.hip: a
// lone 64-lane wave's SHA-1 chain (registers, ds or flat loads of LDS) runs at
// one speed on every CU.  This kernel keeps the service's shape and lets each
// ingredient be switched off: WG = 256 threads (waves 1-3 wait at a barrier
// while wave 0 works) or 64; IDLE = between "requests" wave 0 sleeps ~20 us in
// an s_sleep loop (as the service polls) or does not; each "request" is 8
// dependent compressions of blocks read from LDS, then 4 barriers (the tree
// levels).  Sequential one-workgroup launches (each lands on the next CU) print
// the median request time and the placement.
//
//   hipcc --offload-arch=gfx950 -O3 tools/svc_shape.hip -o tools/svc_shape.bin
//   tools/svc_shape.bin [launches] [bisect|lanes]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
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
constexpr int kReqs = 64;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_rotateleft32(x, n); }

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
    uint64_t req_ticks[kReqs];
};

// QUARTERS: LANES active lanes in each 16-lane quarter of wave 0 instead of the
// first LANES lanes
template <bool IDLE, int LANES, int LEVELS, bool QUARTERS = false>
__global__ __launch_bounds__(256) void k_shape(Rec* out) {
    __shared__ uint4 blk[1024];
    __shared__ uint32_t dig[5 * 64];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 1024; i += blockDim.x) blk[i] = make_uint4(i, 3 * i, 5 * i, 7 * i);
    __syncthreads();
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u ^ tid};
    uint32_t sink = 0;
    for (int q = 0; q < kReqs; ++q) {
        if (tid < 64) {  // wave 0: wait for the "request" (a fixed idle time), wave-uniform
            if (IDLE) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
        if (QUARTERS ? (tid < 64 && (tid & 15u) < uint32_t(LANES)) : tid < uint32_t(LANES)) {  // e.g. 10 lanes: a 10-value flush
            for (int b = 0; b < 8; ++b) {
                const uint32_t at = ((h[0] + tid + b) & 255u) * 4u;
                uint32_t m[16];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint4 v = blk[at + k];
                    m[4 * k] = v.x;
                    m[4 * k + 1] = v.y;
                    m[4 * k + 2] = v.z;
                    m[4 * k + 3] = v.w;
                }
                compress(h, m);
            }
#pragma unroll
            for (int k = 0; k < 5; ++k) dig[5 * tid + k] = h[k];
        }
        for (int lv = 0; lv < LEVELS; ++lv) {  // the levels' barriers
            __syncthreads();
            if (tid < (10u >> lv)) h[0] ^= dig[5 * tid];
        }
        __syncthreads();
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
        sink ^= h[0];
        if (tid == 0) out->req_ticks[q] = r1 - r0;
    }
    if (tid == 0) {
        out->hw = uint32_t(__builtin_amdgcn_s_getreg(kHwId));
        out->xcc = uint32_t(__builtin_amdgcn_s_getreg(kXccId));
        out->sink = sink;
    }
}

template <bool IDLE, int LANES, int LEVELS, bool QUARTERS = false>
static int series(const char* name, Rec* d, int launches, unsigned threads) {
    printf("%s (threads %u, lanes %d%s, level barriers %d, idle %d)\n", name, threads, LANES,
           QUARTERS ? " per quarter" : "", LEVELS, int(IDLE));
    for (int l = 0; l < launches; ++l) {
        hipLaunchKernelGGL((k_shape<IDLE, LANES, LEVELS, QUARTERS>), dim3(1), dim3(threads), 0, 0, d);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        Rec r;
        CK(hipMemcpy(&r, d, sizeof r, hipMemcpyDeviceToHost));
        std::vector<uint64_t> t(r.req_ticks + 4, r.req_ticks + kReqs);
        std::sort(t.begin(), t.end());
        printf("  launch %2d: xcc %u se %u cu %2u simd %u: request median %.2f us (min %.2f max %.2f)\n", l,
               r.xcc & 15, (r.hw >> 13) & 7, (r.hw >> 8) & 15, (r.hw >> 4) & 3, t[t.size() / 2] / 100.0,
               t.front() / 100.0, t.back() / 100.0);
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char** argv) {
    const int launches = argc > 1 ? atoi(argv[1]) : 8;
    CK(hipSetDevice(0));
    Rec* d = nullptr;
    CK(hipMalloc(&d, sizeof(Rec)));
    int rc = 0;
    const char* which = argc > 2 ? argv[2] : "bisect";
    if (which[0] == 'b') {  // round 6, first: which ingredient
        rc |= series<false, 10, 4>("A service shape", d, launches, 256);
        rc |= series<false, 10, 4>("B one wave", d, launches, 64);
        rc |= series<false, 64, 4>("C 256 threads, 64 lanes", d, launches, 256);
        rc |= series<false, 10, 0>("D 256 threads, no level barriers", d, launches, 256);
        rc |= series<false, 64, 0>("E one wave, 64 lanes, no barriers (cu_speed's shape)", d, launches, 64);
        rc |= series<false, 10, 0>("F one wave, 10 lanes, no level barriers", d, launches, 64);
    } else {  // second: which active-lane patterns are slow
        rc |= series<false, 1, 0>("G 1 lane", d, launches, 64);
        rc |= series<false, 16, 0>("H lanes 0-15 (one whole quarter)", d, launches, 64);
        rc |= series<false, 17, 0>("I lanes 0-16", d, launches, 64);
        rc |= series<false, 32, 0>("J lanes 0-31", d, launches, 64);
        rc |= series<false, 48, 0>("K lanes 0-47", d, launches, 64);
        rc |= series<false, 63, 0>("L lanes 0-62", d, launches, 64);
        rc |= series<false, 1, 0, true>("M one lane in each quarter", d, launches, 64);
        rc |= series<false, 3, 0, true>("N three lanes in each quarter", d, launches, 64);
    }
    (void)hipFree(d);
    printf("done rc=%d\n", rc);
    return rc;
}
