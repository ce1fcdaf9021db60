// crc_pattern.hip -- is the record CRC kernel bound by its HBM access pattern?
// The k_crc_lanes inner loop (lane-private tables, one 128-byte line per lane
// in flight, crc_line from crc.hip) over 4 GiB, with two address maps:
//   P0  per-record streams: lane l of wave w checksums 4 KiB record 64 w + l
//       line by line (the product's pattern: each wave-instruction touches 64
//       lines 4 KiB apart);
//   P1  coalesced: step c of the wave reads the contiguous 8 KiB at
//       (wave's region) + 8 KiB c, lane l takes line l of it (not the CRC of
//       any record -- the instruction stream is identical, only addresses move);
// and the same two maps with the CRC replaced by a register XOR (P2, P3: the
// memory stream alone).  Prints ms per launch and GB/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I nakevaleng_amd/csrc tools/crc_pattern.hip -o tools/crc_pattern.bin
#include "../nakevaleng_amd/csrc/crc.hip"

#include <stdio.h>
#include <vector>

namespace nkv {

constexpr int kPatWG = 1024;
constexpr uint32_t kRecLines = 32;  // 4 KiB records

template <int P>
__global__ __launch_bounds__(kPatWG) void k_crc_pat(const uint8_t* __restrict__ base, uint64_t nrec,
                                                    uint32_t* __restrict__ out) {
    __shared__ uint32_t tab[kLaneTabWords];
    for (uint32_t i = threadIdx.x; i < kLaneTabWords; i += kPatWG) {
        const uint32_t half = i >> 14, e = (i >> 6) & 255u, k = 2u * half + ((i >> 5) & 1u);
        tab[i] = c_crc.t[k][e];
    }
    __syncthreads();
    const uint32_t la0 = (threadIdx.x & 31u) * 4u, la1 = la0 | 0x10000u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t stride = uint64_t(gridDim.x) * kPatWG;
    uint32_t acc = 0;
    for (uint64_t wb = uint64_t(blockIdx.x) * kPatWG + (threadIdx.x & ~63u); wb < nrec; wb += stride) {
        // this wave's 64 records = 256 KiB at base + 4096 wb
        const uint4* region = reinterpret_cast<const uint4*>(base + 4096ull * wb);
        auto line = [&](uint32_t c) -> const uint4* {
            if (c >= kRecLines) return g_crc_line;
            if constexpr (P == 0 || P == 2) return region + 8 * (uint64_t(lane) * kRecLines + c);
            else return region + 8 * (uint64_t(c) * 64 + lane);
        };
        crc_v4 va[8], vb[8];
        uint32_t crc = 0xFFFFFFFFu;
        crc_line_load(line(0), va);
        for (uint32_t c = 0; c < kRecLines; c += 2) {
            crc_line_load(line(c + 1), vb);
            if constexpr (P < 2) {
                crc = crc_line(crc, va, 0, 0, ~0ull, la0, la1);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) crc ^= va[i][0] ^ va[i][1] ^ va[i][2] ^ va[i][3];
            }
            crc_line_load(line(c + 2), va);
            if constexpr (P < 2) {
                crc = crc_line(crc, vb, 0, 0, ~0ull, la0, la1);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) crc ^= vb[i][0] ^ vb[i][1] ^ vb[i][2] ^ vb[i][3];
            }
        }
        acc ^= crc;
    }
    out[blockIdx.x * kPatWG + threadIdx.x] = acc;
}

}  // namespace nkv

using namespace nkv;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main() {
    const uint64_t nrec = 1ull << 20, bytes = nrec * 4096;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t* d = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 0x5A, bytes));
    CK(hipMalloc(&out, uint64_t(cus) * kPatWG * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](auto kernel, const char* name) -> int {
        for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kernel, dim3(cus), dim3(kPatWG), 0, 0, d, nrec, out);
        CK(hipEventRecord(e0));
        const int it = 20;
        for (int k = 0; k < it; ++k) hipLaunchKernelGGL(kernel, dim3(cus), dim3(kPatWG), 0, 0, d, nrec, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= it;
        printf("%s  %.4f ms  %.1f GB/s\n", name, ms, double(bytes) / (ms * 1e-3) / 1e9);
        return 0;
    };
    for (int rep = 0; rep < 2; ++rep) {
        if (run(k_crc_pat<0>, "P0 per-record streams, CRC ") ||
            run(k_crc_pat<1>, "P1 coalesced 8 KiB steps, CRC") ||
            run(k_crc_pat<2>, "P2 per-record streams, XOR ") ||
            run(k_crc_pat<3>, "P3 coalesced 8 KiB steps, XOR"))
            return 1;
    }
    CK(hipFree(d));
    CK(hipFree(out));
    return 0;
}
