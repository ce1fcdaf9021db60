// fetch_calib.hip -- calibrate rocprofv3 FETCH_SIZE for the leaf kernel's access
// pattern (the MI355X guide: FETCH_SIZE is exact only for some access widths;
// calibrate on a known byte count in your own pattern).
//
// Reads exactly `values * vlen` bytes with the same wave-level LDS-DMA pattern as
// k_leaf<strided, LOAD=1>: per 64-byte block of 64 values, four
// global_load_lds_dwordx4, each covering 16 values x 64 contiguous bytes.  No
// hashing.  FETCH_SIZE (KB) x 1024 / bytes = the correction factor.
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ __launch_bounds__(256, 8) void k_read(const uint8_t* __restrict__ base, uint64_t n, uint32_t vlen,
                                                 uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[256 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* wbuf = smem + 4096 * wave;
    const uint64_t first = uint64_t(blockIdx.x) * 256 + 64 * uint64_t(wave);
    const uint8_t* wave_base = base + first * vlen;
    const uint32_t q = (uint32_t(lane) & 3u) ^ ((uint32_t(lane) >> 4) & 3u);
    const uint32_t off0 = uint32_t(lane >> 2) * vlen + 16u * q;
    uint32_t acc = 0;
    if (first < n) {
        for (uint32_t b = 0; b < vlen / 64; ++b) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_global_load_lds(wave_base + (off0 + k * 16u * vlen + 64u * b), wbuf + 1024 * k,
                                                 16, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= reinterpret_cast<const uint32_t*>(wbuf)[lane * 16 + (b & 15)];
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const uint64_t n = 1 << 20;
    const uint32_t vlen = 4096;
    uint8_t* d;
    uint32_t* out;
    (void)hipMalloc(&d, n * vlen);
    (void)hipMalloc(&out, n * 4);
    (void)hipMemset(d, 0x5a, n * vlen);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_read, dim3(n / 256), dim3(256), 0, 0, d, n, vlen, out);
    (void)hipDeviceSynchronize();
    printf("k_read: %llu bytes per launch (%llu values x %u B)\n", (unsigned long long)(n * vlen),
           (unsigned long long)n, vlen);
    (void)hipFree(d);
    (void)hipFree(out);
    return 0;
}
