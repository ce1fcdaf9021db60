// lone_wave.hip -- cycles per 64-byte block of ONE wave alone on its SIMD,
// the rate that bounds a ragged batch's longest chain (DESIGN.md section 4,
// cfg3).  Each 64-thread workgroup hashes 64 values of NBLK full blocks with
// one of the leaf kernels' block loops; 256 workgroups = one wave per CU.
// L2 mode: every wave reads the same 64 values (4 MiB at 1,024 blocks);
// HBM mode: each wave its own.
//   hipcc --offload-arch=gfx950 -O3 -I nakevaleng_amd/csrc tools/lone_wave.hip -o tools/lone_wave.bin
#include "../nakevaleng_amd/csrc/kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <vector>

namespace nkv {

// Two independent messages per lane, their rounds interleaved (does a lone
// wave issue faster with twice the ILP?  If its rate is the issue cadence,
// a block pair costs twice a block).
__device__ __forceinline__ void sha1_compress2(uint32_t h[5], uint32_t w[16], uint32_t g[5], uint32_t x[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    uint32_t a2 = g[0], b2 = g[1], c2 = g[2], d2 = g[3], e2 = g[4];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt, xt;
        if (t < 16) {
            wt = w[t];
            xt = x[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
            xt = rotl(xor3(x[(t - 3) & 15], x[(t - 8) & 15], x[(t - 14) & 15]) ^ x[t & 15], 1);
            x[t & 15] = xt;
        }
        uint32_t f, f2, k;
        if (t < 20) { f = ch(b, c, d); f2 = ch(b2, c2, d2); k = 0x5A827999u; }
        else if (t < 40) { f = xor3(b, c, d); f2 = xor3(b2, c2, d2); k = 0x6ED9EBA1u; }
        else if (t < 60) { f = maj(b, c, d); f2 = maj(b2, c2, d2); k = 0x8F1BBCDCu; }
        else { f = xor3(b, c, d); f2 = xor3(b2, c2, d2); k = 0xCA62C1D6u; }
        const uint32_t tmp = add3(rotl(a, 5), f, add3k(e, wt, k));
        const uint32_t tmp2 = add3(rotl(a2, 5), f2, add3k(e2, xt, k));
        e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
        e2 = d2; d2 = c2; c2 = rotl(b2, 30); b2 = a2; a2 = tmp2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
    g[0] += a2; g[1] += b2; g[2] += c2; g[3] += d2; g[4] += e2;
}

template <int V>
__global__ __launch_bounds__(64, 1) void k_lone(const uint8_t* __restrict__ base, uint64_t vstride,
                                                uint32_t nblk, int hbm, unsigned long long* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[4 * 4096];
    const int lane = threadIdx.x;
    const uint64_t v = (hbm ? uint64_t(blockIdx.x) * 64 : 0) + uint64_t(lane);
    const uint8_t* p = base + v * vstride;
    uint32_t h[5];
    sha1_init(h);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (V == 0) {
        for (uint32_t b = 0; b < nblk; ++b) {
            uint32_t w[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = bswap32(uint32_t(v) + i * 0x9E3779B9u + b);
            sha1_compress(h, w);
        }
    } else if constexpr (V >= 1 && V <= 3) {
        sha1_blocks_ring_vc<V + 1>(smem, p, nblk, h);
    } else if constexpr (V == 7) {
        // nblk blocks as nblk / 2 interleaved pairs (two messages per lane)
        uint32_t g[5];
        sha1_init(g);
        for (uint32_t b = 0; b < nblk; b += 2) {
            uint32_t w[16], x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                w[i] = bswap32(uint32_t(v) + i * 0x9E3779B9u + b);
                x[i] = bswap32(uint32_t(v) * 3u + i * 0x7F4A7C15u + b);
            }
            sha1_compress2(h, w, g, x);
        }
        h[0] ^= g[0];
    } else if constexpr (V == 5 || V == 6) {
        // V 5: only lanes 0..31 active; V 6: only lanes 0..15 (does a lone
        // wave with a partial exec mask issue faster?)
        if (lane < (V == 5 ? 32 : 16)) {
            for (uint32_t b = 0; b < nblk; ++b) {
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] = bswap32(uint32_t(v) + i * 0x9E3779B9u + b);
                sha1_compress(h, w);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
    if (lane == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[blockIdx.x * 4 + 0] = t1 - t0;
        out[blockIdx.x * 4 + 1] = r1 - r0;
        out[blockIdx.x * 4 + 2] = (uint64_t(xcc) << 32) | hw;
    }
    if (x == 0x12345678u) out[blockIdx.x * 4 + 3] = x;
}


// The rounds alone, W[t] + K[t] precomputed: what a chain wave would issue if
// another wave of its workgroup expanded the schedule (VERDICT r04 item 7's
// mixed chain floor).  Per lane 80 words in LDS at a padded stride; the loop
// reads 16 of them (four ds_read_b128) one chunk ahead of the rounds using them.
constexpr int kWkStride = 84;  // words per lane row (80 + 4 pad)
__device__ __forceinline__ void rounds_wk(uint32_t h[5], const uint32_t* __restrict__ wk_row) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = reinterpret_cast<const uint4*>(wk_row)[q];
#pragma unroll
    for (int ch16 = 0; ch16 < 5; ++ch16) {
        if (ch16 < 4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) nxt[q] = reinterpret_cast<const uint4*>(wk_row + 16 * (ch16 + 1))[q];
        }
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[4 * q] = cur[q].x; w[4 * q + 1] = cur[q].y; w[4 * q + 2] = cur[q].z; w[4 * q + 3] = cur[q].w;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int t = 16 * ch16 + i;
            uint32_t f;
            if (t < 20) f = ch(b, c, d);
            else if (t < 40) f = xor3(b, c, d);
            else if (t < 60) f = maj(b, c, d);
            else f = xor3(b, c, d);
            const uint32_t tmp = add3(rotl(a, 5), f, e + w[i]);
            e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
        }
        if (ch16 < 4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
        }
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// W[0..79] + K of one block into a lane's row
__device__ __forceinline__ void schedule_wk(uint32_t w[16], uint32_t* __restrict__ row) {
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) wt = w[t];
        else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        const uint32_t k = t < 20 ? 0x5A827999u : t < 40 ? 0x6ED9EBA1u : t < 60 ? 0x8F1BBCDCu : 0xCA62C1D6u;
        row[t] = wt + k;
    }
}

// V 8: one wave, the rounds from a constant precomputed row (the chain's floor
// with the schedule elsewhere); V 9: two waves, wave 1 expands each block's
// schedule into one of two LDS slots while wave 0 runs the rounds from the
// other, LDS counters hand the slots over (the split as a kernel would run it)
template <int V>
__global__ __launch_bounds__(128, 1) void k_split(uint32_t nblk, unsigned long long* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t wk[2][64 * kWkStride];
    __shared__ uint32_t produced, consumed;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t v = blockIdx.x * 64u + uint32_t(lane);
    if (threadIdx.x == 0) { produced = 0; consumed = 0; }
    if (V == 8 && wave == 0) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = bswap32(v + i * 0x9E3779B9u);
        schedule_wk(w, &wk[0][lane * kWkStride]);
    }
    __syncthreads();
    uint32_t h[5];
    sha1_init(h);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (V == 8) {
        if (wave == 0)
            for (uint32_t b = 0; b < nblk; ++b) rounds_wk(h, &wk[0][lane * kWkStride]);
    } else {
        if (wave == 1) {  // producer
            for (uint32_t b = 0; b < nblk; ++b) {
                if (b >= 2)
                    while (__hip_atomic_load(&consumed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < b - 1)
                        __builtin_amdgcn_s_sleep(1);
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] = bswap32(v + i * 0x9E3779B9u + b);
                schedule_wk(w, &wk[b & 1][lane * kWkStride]);
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the row is in LDS
                if (lane == 0) __hip_atomic_store(&produced, b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else {  // chain
            for (uint32_t b = 0; b < nblk; ++b) {
                while (__hip_atomic_load(&produced, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < b + 1)
                    __builtin_amdgcn_s_sleep(1);
                rounds_wk(h, &wk[b & 1][lane * kWkStride]);
                __builtin_amdgcn_s_waitcnt(0xc07f);
                if (lane == 0) __hip_atomic_store(&consumed, b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
    if (threadIdx.x == 0) {
        out[blockIdx.x * 4 + 0] = t1 - t0;
        out[blockIdx.x * 4 + 1] = r1 - r0;
        out[blockIdx.x * 4 + 2] = 0;
    }
    if (x == 0x12345678u) out[blockIdx.x * 4 + 3] = x;
}

template <int V>
void run_split(const char* name, uint32_t nblk, int wgs) {
    unsigned long long* out;
    (void)hipMalloc(&out, size_t(wgs) * 32);
    hipLaunchKernelGGL(k_split<V>, dim3(wgs), dim3(V == 8 ? 64 : 128), 0, 0, nblk, out);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_split<V>, dim3(wgs), dim3(V == 8 ? 64 : 128), 0, 0, nblk, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> o(size_t(wgs) * 4);
    (void)hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0, ghz = 0;
    for (int w = 0; w < wgs; ++w) {
        cyc += double(o[4 * w]);
        ghz += double(o[4 * w]) / (double(o[4 * w + 1]) / 100e6) / 1e9;
    }
    printf("%-28s wgs=%4d nblk=%5u  %.3f ms  clk %.2f GHz  %.0f cycles/block  %.3f us/block\n", name, wgs, nblk, ms,
           ghz / wgs, cyc / wgs / nblk, ms * 1e3 / nblk);
    (void)hipFree(out);
}

template <int V>
void run(const char* name, const uint8_t* d, uint64_t vstride, uint32_t nblk, int waves, int hbm) {
    unsigned long long* out;
    (void)hipMalloc(&out, size_t(waves) * 32);
    hipLaunchKernelGGL(k_lone<V>, dim3(waves), dim3(64), 0, 0, d, vstride, nblk, hbm, out);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_lone<V>, dim3(waves), dim3(64), 0, 0, d, vstride, nblk, hbm, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> o(size_t(waves) * 4);
    (void)hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0, cmax = 0, ghz = 0;
    for (int w = 0; w < waves; ++w) {
        cyc += double(o[4 * w]);
        cmax = std::max(cmax, double(o[4 * w]));
        ghz += double(o[4 * w]) / (double(o[4 * w + 1]) / 100e6) / 1e9;
    }
    printf("%-28s %s waves=%4d nblk=%5u  %.3f ms  clk %.2f GHz  %.0f cycles/block (max %.0f)  %.3f us/block\n", name,
           hbm ? "HBM" : "L2 ", waves, nblk, ms, ghz / waves, cyc / waves / nblk, cmax / nblk,
           ms * 1e3 / nblk);
    (void)hipFree(out);
}

}  // namespace nkv

int main() {
    using namespace nkv;
    const uint32_t nblk = 1024;
    const uint64_t vstride = 64ull * nblk;
    const uint64_t bytes = uint64_t(2048) * 64 * vstride;
    uint8_t* d;
    if (hipMalloc(&d, bytes + 4096) != hipSuccess) return 1;
    (void)hipMemset(d, 0x5a, bytes + 4096);
    if (getenv("NKV_LONE_ILP")) {
        for (int waves : {256, 1024}) {
            run<0>("regs only, 1 msg/lane", d, vstride, nblk, waves, 0);
            run<7>("regs only, 2 msg/lane", d, vstride, nblk, waves, 0);
        }
        (void)hipFree(d);
        return 0;
    }
    if (getenv("NKV_LONE_SPLIT")) {
        for (int waves : {256, 1024}) {
            run<0>("regs only, full compress", d, vstride, nblk, waves, 0);
            run_split<8>("rounds only, W+K in LDS", nblk, waves);
            run_split<9>("rounds + schedule wave", nblk, waves);
        }
        (void)hipFree(d);
        return 0;
    }
    if (getenv("NKV_LONE_EXEC")) {
        for (int waves : {256, 1024}) {
            run<0>("regs only, 64 lanes", d, vstride, nblk, waves, 0);
            run<5>("regs only, 32 lanes", d, vstride, nblk, waves, 0);
            run<6>("regs only, 16 lanes", d, vstride, nblk, waves, 0);
        }
        (void)hipFree(d);
        return 0;
    }
    for (int hbm = 0; hbm < 2; ++hbm)
        for (int waves : {256, 512, 1024, 2048}) {
            run<0>("regs only", d, vstride, nblk, waves, hbm);
            run<2>("ring_vc<3>", d, vstride, nblk, waves, hbm);
        }
    (void)hipFree(d);
    return 0;
}
