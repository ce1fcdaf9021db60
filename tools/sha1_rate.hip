// sha1_rate.hip -- compute-only ceiling of the per-lane SHA-1 compression
// (nakevaleng_amd/csrc/sha1_dev.hpp) on the whole chip: no memory traffic,
// message words in registers.  Prints SIMD-cycles per 64-byte block per wave
// and the payload rate it would sustain (GB/s = blocks * 64 B / s).
//   hipcc --offload-arch=gfx950 -O3 -I nakevaleng_amd/csrc tools/sha1_rate.hip -o tools/sha1_rate.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#include "sha1_dev.hpp"

// LOADS: message words read from a 64 KiB L2-resident buffer (per-lane 64-byte
// rows) instead of being generated in registers.
template <int WAVES, bool LOADS = false>
__global__ __launch_bounds__(256, WAVES) void k(uint32_t* out, unsigned long long* clk, int blocks,
                                                const uint4* src = nullptr) {
    uint32_t h[5];
    nkv::sha1_init(h);
    uint32_t seed = blockIdx.x * 256 + threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int b = 0; b < blocks; ++b) {
        uint32_t w[16];
        if (LOADS) {
            const uint4* q = src + ((threadIdx.x + 64 * (b & 15)) & 1023) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint4 v = q[i];
                w[4 * i] = nkv::bswap32(v.x);
                w[4 * i + 1] = nkv::bswap32(v.y);
                w[4 * i + 2] = nkv::bswap32(v.z);
                w[4 * i + 3] = nkv::bswap32(v.w);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = nkv::bswap32(seed + i * 0x9E3779B9u + uint32_t(b));
        }
        nkv::sha1_compress(h, w);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int WAVES, bool LOADS = false>
void run(int nblk_kernel, int blocks, int reps = 1, bool random = false) {
    uint32_t* out;
    unsigned long long* clk;
    uint4* src;
    (void)hipMalloc(&out, size_t(nblk_kernel) * 256 * 4);
    (void)hipMalloc(&clk, 16);
    (void)hipMalloc(&src, 65536);
    (void)hipMemset(src, 0x5a, 65536);
    if (random) {  // splitmix64 bytes: the toggle rate of real payloads
        std::vector<uint64_t> hbuf(65536 / 8);
        uint64_t z = 0x6e616b65ull;
        for (auto& x : hbuf) {
            z += 0x9E3779B97F4A7C15ull;
            uint64_t y = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            y = (y ^ (y >> 27)) * 0x94D049BB133111EBull;
            x = y ^ (y >> 31);
        }
        (void)hipMemcpy(src, hbuf.data(), 65536, hipMemcpyHostToDevice);
    }
    hipLaunchKernelGGL((k<WAVES, LOADS>), dim3(nblk_kernel), dim3(256), 0, 0, out, clk, blocks, src);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k<WAVES, LOADS>), dim3(nblk_kernel), dim3(256), 0, 0, out, clk, blocks, src);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = double(c[0]) / (double(c[1]) / 100e6) / 1e9;
    const double waves_per_simd = double(nblk_kernel) * 4 / 1024.0;
    const double cyc = ms * 1e-3 * ghz * 1e9;
    const double per_block = cyc / (waves_per_simd * blocks);
    const double gbs = double(nblk_kernel) * 256 * blocks * 64.0 / (ms * 1e-3) / 1e9;
    printf("%s%s reps=%3d waves/SIMD=%d grid=%6d  %.3f ms  clk %.2f GHz  %.0f SIMD-cycles per block per wave  %.0f GB/s\n",
           LOADS ? "L2-loads" : "regs    ", random ? " random" : " const ", reps, WAVES, nblk_kernel, ms, ghz, per_block, gbs);
    (void)hipFree(out);
    (void)hipFree(clk);
    (void)hipFree(src);
}

int main() {
    run<8>(2048, 4096);
    run<8>(4096, 2048);
    run<4>(1024, 4096);
    run<2>(512, 4096);
    run<1>(256, 2048);
    run<8, true>(2048, 4096);
    run<8, true>(4096, 2048);
    // sustained: back-to-back launches of ~1.3 ms (the bench's regime); the
    // clock is the last launch's
    run<8>(2048, 160, 1);
    run<8>(2048, 160, 200);
    run<8, true>(2048, 160, 300, false);
    run<8, true>(2048, 160, 300, true);
    run<8, true>(4096, 80, 300, true);
    run<1>(256, 1024, 300);
    return 0;
}
