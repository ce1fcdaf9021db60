// valu_rate.hip -- issue rate of the VALU forms SHA-1 uses, on the whole chip.
// Each wave runs 8 independent chains of one instruction (inline asm, so the
// exact opcode is measured); the clock is read in-kernel (s_memtime over
// s_memrealtime at 100 MHz).  Prints cycles per wave64 instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP 64
#define ITERS 2000

#define BODY8(OP)                                                                 \
    asm volatile(".rept " "64" "\n\t"                                              \
                 OP(%0) "\n\t" OP(%1) "\n\t" OP(%2) "\n\t" OP(%3) "\n\t"            \
                 OP(%4) "\n\t" OP(%5) "\n\t" OP(%6) "\n\t" OP(%7) "\n\t"            \
                 ".endr"                                                          \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(x), "v"(y) : "vcc", "v63")

#define OP_ADD(r) "v_add_u32 " #r ", " #r ", %8"
#define OP_XOR(r) "v_xor_b32 " #r ", " #r ", %8"
#define OP_ADD3(r) "v_add3_u32 " #r ", " #r ", %8, %9"
#define OP_BITOP3(r) "v_bitop3_b32 " #r ", " #r ", %8, %9 bitop3:0x96"
#define OP_ALIGNBIT(r) "v_alignbit_b32 " #r ", " #r ", " #r ", 27"
#define OP_PERM(r) "v_perm_b32 " #r ", " #r ", %8, %9"
#define OP_FMA(r) "v_fma_f32 " #r ", " #r ", %8, %9"
#define OP_LSHLOR(r) "v_lshl_or_b32 " #r ", " #r ", 5, %8"
#define OP_LSHLADD(r) "v_lshl_add_u32 " #r ", " #r ", 5, %8"
#define OP_OR3(r) "v_or3_b32 " #r ", " #r ", %8, %9"
#define OP_XAD(r) "v_xad_u32 " #r ", " #r ", %8, %9"
#define OP_SHL(r) "v_lshlrev_b32 " #r ", 5, " #r
#define OP_ADDLIT(r) "v_add_u32 " #r ", 0x5a827999, " #r
#define OP_ADD3S(r) "v_add3_u32 " #r ", " #r ", %8, s0"
#define OP_MIX1(r) "v_alignbit_b32 " #r ", " #r ", " #r ", 27\n\tv_xor_b32 " #r ", " #r ", %8"
#define OP_MIX2(r) "v_add3_u32 " #r ", " #r ", %8, %9\n\tv_bitop3_b32 " #r ", " #r ", %8, %9 bitop3:0x96"
#define OP_MIX3(r) "v_alignbit_b32 " #r ", " #r ", " #r ", 27\n\tv_xor_b32 " #r ", " #r ", %8\n\tv_xor_b32 " #r ", " #r ", %9\n\tv_bitop3_b32 " #r ", " #r ", %8, %9 bitop3:0x96"
#define CL_ALIGN(r) "v_alignbit_b32 " #r ", " #r ", " #r ", 27"
#define CL_XOR(r) "v_xor_b32 " #r ", " #r ", %8"
#define CL_BITOP(r) "v_bitop3_b32 " #r ", " #r ", %8, %9 bitop3:0x96"
#define BODYCL(OPA, OPB)                                                           \
    asm volatile(".rept " "64" "\n\t"                                              \
                 OPA(%0) "\n\t" OPA(%1) "\n\t" OPA(%2) "\n\t" OPA(%3) "\n\t"        \
                 OPA(%4) "\n\t" OPA(%5) "\n\t" OPA(%6) "\n\t" OPA(%7) "\n\t"        \
                 OPB(%0) "\n\t" OPB(%1) "\n\t" OPB(%2) "\n\t" OPB(%3) "\n\t"        \
                 OPB(%4) "\n\t" OPB(%5) "\n\t" OPB(%6) "\n\t" OPB(%7) "\n\t"        \
                 ".endr"                                                          \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(x), "v"(y))
#define OP_MADU24(r) "v_mad_u32_u24 " #r ", " #r ", %8, %9"
#define OP_ADDCO(r) "v_add_co_u32 " #r ", vcc, " #r ", %8"
#define OP_ADDC(r) "v_addc_co_u32 " #r ", vcc, " #r ", %8, vcc"
#define OP_MOV(r) "v_mov_b32 " #r ", %8"
#define OP_BFI(r) "v_bfi_b32 " #r ", " #r ", %8, %9"
#define OP_ALIGNBYTE(r) "v_alignbyte_b32 " #r ", " #r ", %8, 1"
#define OP_ROT1C(r) "v_add_co_u32 v63, vcc, " #r ", " #r "\n\tv_addc_co_u32 " #r ", vcc, " #r ", " #r ", vcc"
#define OP_SUB(r) "v_sub_u32 " #r ", " #r ", %8"
#define OP_AND(r) "v_and_b32 " #r ", " #r ", %8"
#define OP_CNDMASK(r) "v_cndmask_b32 " #r ", " #r ", %8, vcc"

template <int K>
__global__ __launch_bounds__(256) void k(uint32_t* out, unsigned long long* clk, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed * 3u + threadIdx.x, y = seed * 7u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
        if (K == 0) BODY8(OP_ADD);
        if (K == 1) BODY8(OP_XOR);
        if (K == 2) BODY8(OP_ADD3);
        if (K == 3) BODY8(OP_BITOP3);
        if (K == 4) BODY8(OP_ALIGNBIT);
        if (K == 5) BODY8(OP_PERM);
        if (K == 6) BODY8(OP_FMA);
        if (K == 7) BODY8(OP_LSHLOR);
        if (K == 8) BODY8(OP_LSHLADD);
        if (K == 9) BODY8(OP_OR3);
        if (K == 10) BODY8(OP_XAD);
        if (K == 11) BODY8(OP_SHL);
        if (K == 12) BODY8(OP_ADDLIT);
        if (K == 13) BODY8(OP_MADU24);
        if (K == 14) BODY8(OP_MIX1);
        if (K == 15) BODY8(OP_MIX2);
        if (K == 16) BODY8(OP_MIX3);
        if (K == 17) BODYCL(CL_ALIGN, CL_XOR);
        if (K == 18) BODYCL(CL_BITOP, CL_XOR);
        if (K == 19) BODYCL(CL_XOR, CL_XOR);
        if (K == 20) { if (blockIdx.x & 1) BODY8(OP_ALIGNBIT); else BODY8(OP_XOR); }
        if (K == 21) BODY8(OP_ADDCO);
        if (K == 22) BODY8(OP_ADDC);
        if (K == 23) BODY8(OP_MOV);
        if (K == 24) BODY8(OP_BFI);
        if (K == 25) BODY8(OP_ALIGNBYTE);
        if (K == 26) BODY8(OP_SUB);
        if (K == 27) BODY8(OP_AND);
        if (K == 28) BODY8(OP_CNDMASK);
        if (K == 29) { if (blockIdx.x & 1) BODY8(OP_MIX1); else BODY8(OP_XOR); }
        if (K == 30) { if ((blockIdx.x & 3) == 0) BODY8(OP_ALIGNBIT); else BODY8(OP_XOR); }
        if (K == 31) BODY8(OP_ROT1C);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int K>
void run(const char* name, int blocks) {
    uint32_t* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, size_t(blocks) * 256 * 4);
    (void)hipMalloc(&clk, 16);
    hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(256), 0, 0, out, clk, 1u);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<K>, dim3(blocks), dim3(256), 0, 0, out, clk, 2u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    double ghz = double(c[0]) / (double(c[1]) / 100e6) / 1e9;
    // wave-instructions per SIMD: blocks*4 waves / (256 CU * 4 SIMD) * ITERS * 64 * 8
    double waves_per_simd = double(blocks) * 4 / 1024.0;
    double winstr = waves_per_simd * ITERS * 64.0 * 8;
    double cyc = ms * 1e-3 * ghz * 1e9;
    printf("%-10s blocks=%6d  %.3f ms  clk %.2f GHz  %.2f cycles per wave64 instr per SIMD  (%.1f T lane-ops/s)\n",
           name, blocks, ms, ghz, cyc / winstr, double(blocks) * 256 * ITERS * 64.0 * 8 / (ms * 1e-3) / 1e12);
    (void)hipFree(out);
    (void)hipFree(clk);
}

int main() {
    for (int blocks : {2048}) {
        run<0>("v_add_u32", blocks);
        run<1>("v_xor_b32", blocks);
        run<2>("v_add3_u32", blocks);
        run<3>("v_bitop3", blocks);
        run<4>("v_alignbit", blocks);
        run<5>("v_perm_b32", blocks);
        run<6>("v_fma_f32", blocks);
        run<7>("v_lshl_or", blocks);
        run<8>("v_lshl_add", blocks);
        run<9>("v_or3_b32", blocks);
        run<10>("v_xad_u32", blocks);
        run<11>("v_lshlrev", blocks);
        run<12>("v_add_lit", blocks);
        run<13>("v_mad_u24", blocks);
        run<14>("mix alignbit+xor (2 instr)", blocks);
        run<15>("mix add3+bitop3 (2 instr)", blocks);
        run<16>("mix alignbit+3 full (4 instr)", blocks);
        run<17>("clustered 8 alignbit + 8 xor (per 2)", blocks);
        run<18>("clustered 8 bitop3 + 8 xor (per 2)", blocks);
        run<19>("16 xor (per 2)", blocks);
        run<20>("split blocks: pure alignbit | pure xor", blocks);
        run<21>("v_add_co_u32", blocks);
        run<22>("v_addc_co_u32", blocks);
        run<23>("v_mov_b32", blocks);
        run<24>("v_bfi_b32", blocks);
        run<25>("v_alignbyte", blocks);
        run<26>("v_sub_u32", blocks);
        run<27>("v_and_b32", blocks);
        run<28>("v_cndmask", blocks);
        run<29>("split blocks: mix1 (2 instr) | pure xor", blocks);
        run<30>("split 1:3 alignbit | xor", blocks);
        run<31>("rotl1 by add_co+addc (2 instr)", blocks);
    }
    return 0;
}
