// pattern_power.hip -- does the HBM access pattern set the sustained shader
// clock of the VALU-bound leaf kernel?  The cfg2 loop (k_leaf MODE 0, LOAD 1:
// SHA-1 over blocks staged by LDS-DMA) runs with three address maps over the
// same 4 GiB, back to back like the bench:
//   P0  per-value streams: lane l of wave w hashes value 64 w + l, block b at
//       (64 w + l) * 4096 + 64 b (the product's pattern: each wave-instruction
//       touches 64 rows 4 KiB apart, every stream advances 64 B per block);
//   P1  coalesced: block b of the wave is the contiguous 4 KiB at
//       (64 w + b) * 4096, lane l takes its 64 B at + 64 l (not a SHA-1 of
//       any value -- the instruction stream is identical, only addresses move);
//   P2  no DMA: the same loop over whatever the LDS stage holds.
// Prints ms per launch, the in-kernel clock of the last launch and cycles per
// block.
//   hipcc --offload-arch=gfx950 -O3 -I nakevaleng_amd/csrc tools/pattern_power.hip -o tools/pattern_power.bin
#include "../nakevaleng_amd/csrc/kernels.hip"

#include <stdio.h>
#include <unistd.h>
#include <vector>

namespace nkv {

template <int P>
__global__ __launch_bounds__(kBlock, kLeafWavesPerSimd) void k_pat(const uint8_t* __restrict__ base, uint32_t nblk,
                                                                   uint8_t* __restrict__ nodes,
                                                                   unsigned long long* __restrict__ clk) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kBlock * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t w = uint64_t(blockIdx.x) * (kBlock / 64) + wave;
    uint8_t* wbuf = smem + 4096 * wave;
    const uint32_t q = (uint32_t(lane) & 3u) ^ ((uint32_t(lane) >> 4) & 3u);
    const uint8_t* wave_base = base + w * 64 * 4096;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t h[5];
    sha1_init(h);
    auto issue = [&](uint32_t b) {
        if constexpr (P == 0) {
            const uint32_t off0 = uint32_t(lane >> 2) * 4096u + 16u * q;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_global_load_lds(wave_base + (off0 + k * 16u * 4096u + 64u * b), wbuf + 1024 * k, 16, 0, 0);
        } else if constexpr (P == 1) {
            // the same LDS slots as P0 (value 16k + l/4, chunk q), filled from
            // the contiguous 4 KiB of block b
            const uint32_t off0 = uint32_t(lane >> 2) * 64u + 16u * q;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_global_load_lds(wave_base + (4096u * b + off0 + k * 1024u), wbuf + 1024 * k, 16, 0, 0);
        }
    };
    sha1_blocks_lds(wbuf, nblk, nblk, issue, h);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    store_digest(nodes, w * 64 + lane, h);
    if (lane == 0) {
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = r1 - r0;
    }
}

template <int P>
void run(const char* name, const uint8_t* d, uint8_t* nodes, unsigned long long* clk, int grid, int reps) {
    const uint32_t nblk = 64;
    hipLaunchKernelGGL(k_pat<P>, dim3(grid), dim3(kBlock), 0, 0, d, nblk, nodes, clk);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_pat<P>, dim3(grid), dim3(kBlock), 0, 0, d, nblk, nodes, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const int waves = grid * (kBlock / 64);
    std::vector<unsigned long long> o(size_t(waves) * 2);
    (void)hipMemcpy(o.data(), clk, o.size() * 8, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int i = 0; i < waves; ++i) ghz += double(o[2 * i]) / (double(o[2 * i + 1]) / 100e6) / 1e9;
    ghz /= waves;
    const double bytes = double(waves) * 64 * 64 * nblk;
    const double simd_cycles = ms * 1e-3 * ghz * 1e9;
    const double blocks_per_simd = double(waves) * nblk / 1024.0;
    printf("%-34s reps=%4d  %.3f ms  %.0f GB/s  clk %.2f GHz  %.0f SIMD-cycles per wave-block\n", name, reps, ms,
           bytes / (ms * 1e-3) / 1e9, ghz, simd_cycles / blocks_per_simd);
}

// clock ramp: per-launch times of n back-to-back launches (events between)
void ramp(const uint8_t* d, uint8_t* nodes, unsigned long long* clk, int grid, int n, int idle_ms) {
    std::vector<hipEvent_t> ev(n + 1);
    for (auto& e : ev) (void)hipEventCreate(&e);
    (void)hipDeviceSynchronize();
    if (idle_ms) usleep(idle_ms * 1000);
    (void)hipEventRecord(ev[0]);
    for (int r = 0; r < n; ++r) {
        hipLaunchKernelGGL(k_pat<0>, dim3(grid), dim3(kBlock), 0, 0, d, 64u, nodes, clk);
        (void)hipEventRecord(ev[r + 1]);
    }
    (void)hipEventSynchronize(ev[n]);
    printf("ramp after %d ms idle (ms per launch):", idle_ms);
    double acc = 0;
    for (int r = 0; r < n; ++r) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev[r], ev[r + 1]);
        acc += ms;
        if (r < 12 || r % 25 == 0 || r == n - 1) printf(" [%d @%.0fms] %.3f", r, acc, ms);
    }
    printf("\n");
    for (auto& e : ev) (void)hipEventDestroy(e);
}

}  // namespace nkv

int main() {
    using namespace nkv;
    const int grid = 4096;  // 16384 waves x 64 values x 4 KiB = 4 GiB
    const uint64_t bytes = uint64_t(grid) * kBlock * 4096;
    uint8_t *d, *nodes;
    unsigned long long* clk;
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    (void)hipMalloc(&nodes, uint64_t(grid) * kBlock * 20);
    (void)hipMalloc(&clk, uint64_t(grid) * 4 * 16);
    (void)hipMemset(d, 0x5a, bytes);
    printf("constant bytes (0x5a):\n");
    ramp(d, nodes, clk, grid, 400, 0);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(kBlock), 0, 0, d, bytes, 0x6e616b65ull);
    printf("splitmix64 bytes:\n");
    ramp(d, nodes, clk, grid, 400, 0);
    ramp(d, nodes, clk, grid, 400, 1000);
    for (int reps : {1, 300}) {
        run<0>("P0 per-value streams (product)", d, nodes, clk, grid, reps);
        run<1>("P1 coalesced 4 KiB per block", d, nodes, clk, grid, reps);
        run<2>("P2 no DMA", d, nodes, clk, grid, reps);
    }
    return 0;
}
