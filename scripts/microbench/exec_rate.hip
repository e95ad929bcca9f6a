// exec_rate.hip -- two questions the plane kernel's roofline and drain
// design hang on (diagnostic, not product code):
//   1. issue rate of the integer VALU forms plane::pass uses (v_xor_b32,
//      v_bitop3_b32, v_lshrrev_b32, v_and_or_b32, v_add_u32, v_cndmask_b32)
//      against v_add_f32, at 1..8 waves per SIMD, 8 independent chains per
//      lane: cycles per wave64 instruction per SIMD;
//   2. cost of plane::pass when only part of the wave is active (exec mask
//      = lanes 0-31, 0-15, every other lane ...): does a SIMD-32 skip an
//      all-zero half?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-sched-strategy=iterative-ilp \
//         -o exec_rate scripts/microbench/exec_rate.hip && ./exec_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../sudoku_solver_distributed_amd/csrc/plane_solver.h"

#define ITER 128

// ---- 1: raw issue rate
#define CH8(S) S(a0, a1) S(a1, a2) S(a2, a3) S(a3, a4) S(a4, a5) S(a5, a6) S(a6, a7) S(a7, a0)
#define XOR(d, s) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(s));
#define BOP3(d, s) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x9c" : "+v"(d) : "v"(s), "v"(k));
#define LSHR(d, s) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(d) : "v"(s));
#define ANDOR(d, s) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define ADDU(d, s) asm volatile("v_add_u32 %0, %0, %1" : "+v"(d) : "v"(s));
#define ADDF(d, s) asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(s));
#define MUL24(d, s) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(d) : "v"(s));
#define OR3(d, s) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define BFE(d, s) asm volatile("v_bfe_u32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define BFI(d, s) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define SUBU(d, s) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(d) : "v"(s));
#define ORB(d, s) asm volatile("v_or_b32 %0, %0, %1" : "+v"(d) : "v"(s));
#define LSHLOR(d, s) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define ADD3(d, s) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define LSHLADD(d, s) asm volatile("v_lshl_add_u32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define LSHRE64(d, s) asm volatile("v_lshrrev_b32_e64 %0, %1, %0" : "+v"(d) : "v"(s));
#define ALIGNB(d, s) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define PERM(d, s) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define LSHLREV(d, s) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(d) : "v"(s));
#define XAD(d, s) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define OR3K(d, s) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(d) : "v"(s), "s"(ks));
#define BOP3K(d, s) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xfe" : "+v"(d) : "v"(s), "s"(ks));
#define ANDLIT(d, s) asm volatile("v_and_b32_e32 %0, 0x1ff, %0" : "+v"(d));
#define ANDSG(d, s) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(d) : "s"(ks));
#define ANDE64(d, s) asm volatile("v_and_b32_e64 %0, %0, %1" : "+v"(d) : "v"(s));
#define BOP3IC(d, s) asm volatile("v_bitop3_b32 %0, %0, %1, 7 bitop3:0xfe" : "+v"(d) : "v"(s));
#define BOP3X(d, s) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(d) : "v"(s), "v"(k));
#define NOTB(d, s) asm volatile("v_not_b32 %0, %0" : "+v"(d));
#define LSHLIC(d, s) asm volatile("v_lshlrev_b32_e32 %0, 3, %0" : "+v"(d));
#define LSHRIC(d, s) asm volatile("v_lshrrev_b32_e32 %0, 3, %0" : "+v"(d));
#define LSHLE64(d, s) asm volatile("v_lshlrev_b32_e64 %0, %1, %0" : "+v"(d) : "v"(s));
#define CNDM(d, s) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(d) : "v"(s));
#define XORE64(d, s) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(d) : "v"(s));
#define ORSG(d, s) asm volatile("v_or_b32_e32 %0, %1, %0" : "+v"(d) : "s"(ks));
#define ADDE64(d, s) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(d) : "v"(s));
#define MOVB(d, s) asm volatile("v_mov_b32 %0, %1" : "=v"(d) : "v"(s));
#define CMPEQ(d, s) asm volatile("v_cmp_eq_u32_e32 vcc, %0, %1" :: "v"(d), "v"(s) : "vcc");
#define MIX(d, s) asm volatile("v_or3_b32 %0, %0, %1, %2\n v_xor_b32 %1, %1, %0" : "+v"(d), "+v"(s) : "v"(k));
#define MIX2(d, s) asm volatile("v_or3_b32 %0, %0, %1, %2\n v_xor_b32 %3, %3, %2" : "+v"(d) : "v"(s), "v"(k), "v"(q));
#define ORLIT(d, s) asm volatile("v_or_b32_e32 %0, 0x1ff00, %0" : "+v"(d));
#define LSHL1(d, s) asm volatile("v_lshlrev_b32_e32 %0, 1, %0\n v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(s));
#define LSHR1(d, s) asm volatile("v_lshrrev_b32_e32 %0, 1, %0\n v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(s));
#define BOP3SV(d, s) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x9c" : "+v"(d) : "s"(ks), "v"(s));
#define MULLO16(d, s) asm volatile("v_mul_lo_u16 %0, %0, %1" : "+v"(d) : "v"(s));
#define PKMUL16(d, s) asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(d) : "v"(s));
#define MAD24(d, s) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(d) : "v"(s), "v"(k));
#define MULF(d, s) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(d) : "v"(s));
#define SDWA16(d, s) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0" : "+v"(d) : "v"(s));
#define LSHL16(d, s) asm volatile("v_lshlrev_b16 %0, %1, %0" : "+v"(d) : "v"(s));
#define PKLSHL(d, s) asm volatile("v_pk_lshlrev_b16 %0, %1, %0" : "+v"(d) : "v"(s));
#define DPPMOV(d, s) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(d) : "v"(s));
#define CNDM64(d, s) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(d) : "v"(s), "s"(msk));
#define CMP64(d, s) asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(msk) : "v"(d), "v"(s));
#define MULHI24(d, s) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(d) : "v"(s));
#define SUBREV(d, s) asm volatile("v_subrev_u32 %0, %1, %0" : "+v"(d) : "v"(s));
#define ADDLIT(d, s) asm volatile("v_add_u32_e32 %0, 0x3fe00, %0" : "+v"(d));
#define MAXU(d, s) asm volatile("v_max_u32 %0, %0, %1" : "+v"(d) : "v"(s));
#define ASHR(d, s) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(d) : "v"(s));
#define MULU32(d, s) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(d) : "v"(s));
#define FFBL(d, s) asm volatile("v_ffbl_b32 %0, %1" : "=v"(d) : "v"(s));
#define BCNT(d, s) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(d) : "v"(s));

template <int OP>
__global__ __launch_bounds__(256) void raw(uint32_t *sink, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, k = a0 * 3;
    const uint32_t ks = __builtin_amdgcn_readfirstlane(blockIdx.x * 3u + 0x100u);
    uint32_t q = a0 ^ 0x55u;
    uint64_t msk = __builtin_amdgcn_ballot_w64(a0 & 1);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (OP == 0) { CH8(XOR) }
            if (OP == 1) { CH8(BOP3) }
            if (OP == 2) { CH8(LSHR) }
            if (OP == 3) { CH8(ANDOR) }
            if (OP == 4) { CH8(ADDU) }
            if (OP == 5) { CH8(ADDF) }
            if (OP == 6) { CH8(MUL24) }
            if (OP == 7) { CH8(OR3) }
            if (OP == 8) { CH8(BFE) }
            if (OP == 9) { CH8(BFI) }
            if (OP == 10) { CH8(SUBU) }
            if (OP == 11) { CH8(ORB) }
            if (OP == 12) { CH8(LSHLOR) }
            if (OP == 13) { CH8(ADD3) }
            if (OP == 14) { CH8(LSHLADD) }
            if (OP == 15) { CH8(LSHRE64) }
            if (OP == 16) { CH8(ALIGNB) }
            if (OP == 17) { CH8(PERM) }
            if (OP == 18) { CH8(LSHLREV) }
            if (OP == 19) { CH8(XAD) }
            if (OP == 20) { CH8(OR3K) }
            if (OP == 21) { CH8(BOP3K) }
            if (OP == 22) { CH8(ANDLIT) }
            if (OP == 23) { CH8(ANDSG) }
            if (OP == 24) { CH8(ANDE64) }
            if (OP == 25) { CH8(BOP3IC) }
            if (OP == 26) { CH8(BOP3X) }
            if (OP == 27) { CH8(NOTB) }
            if (OP == 28) { CH8(LSHLIC) }
            if (OP == 29) { CH8(LSHRIC) }
            if (OP == 30) { CH8(LSHLE64) }
            if (OP == 31) { CH8(CNDM) }
            if (OP == 32) { CH8(XORE64) }
            if (OP == 33) { CH8(ORSG) }
            if (OP == 34) { CH8(ADDE64) }
            if (OP == 35) { CH8(MOVB) }
            if (OP == 36) { CH8(CMPEQ) }
            if (OP == 37) { CH8(MIX) }
            if (OP == 38) { CH8(MIX2) }
            if (OP == 39) { CH8(ORLIT) }
            if (OP == 40) { CH8(LSHL1) }
            if (OP == 41) { CH8(LSHR1) }
            if (OP == 42) { CH8(BOP3SV) }
            if (OP == 43) { CH8(MULLO16) }
            if (OP == 44) { CH8(PKMUL16) }
            if (OP == 45) { CH8(MAD24) }
            if (OP == 46) { CH8(MULF) }
            if (OP == 47) { CH8(SDWA16) }
            if (OP == 48) { CH8(LSHL16) }
            if (OP == 49) { CH8(PKLSHL) }
            if (OP == 50) { CH8(DPPMOV) }
            if (OP == 51) { CH8(CNDM64) }
            if (OP == 52) { CH8(CMP64) }
            if (OP == 53) { CH8(MULHI24) }
            if (OP == 54) { CH8(SUBREV) }
            if (OP == 55) { CH8(ADDLIT) }
            if (OP == 56) { CH8(MAXU) }
            if (OP == 57) { CH8(ASHR) }
            if (OP == 58) { CH8(MULU32) }
            if (OP == 59) { CH8(FFBL) }
            if (OP == 60) { CH8(BCNT) }
        }
    }
    sink[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ q ^ (uint32_t)msk;
}

// ---- 2: plane::pass under a partial exec mask
__global__ __launch_bounds__(256, 4) void pass_masked(const uint32_t *boards, uint32_t *sink, int nboards,
                                                     uint32_t mlo, uint32_t mhi)
{
    const int g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    const uint32_t m = lane < 32 ? mlo : mhi;
    if (!((m >> (lane & 31)) & 1u)) return;
    plane::Board B;
    const uint32_t *src = boards + (size_t)(g % nboards) * 27;
#pragma unroll
    for (int w = 0; w < 27; ++w) B.P[w / 3][w % 3] = src[w];
    B.Det[0] = B.Det[1] = B.Det[2] = 0;
    uint32_t acc = 0;
    for (int it = 0; it < ITER; ++it) {
        uint32_t und[3];
        acc += (uint32_t)plane::pass(B, und) + und[0] + und[1] + und[2];
    }
    sink[g] = acc;
}

typedef void (*rawk)(uint32_t *, int);

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *sink;
    hipMalloc(&sink, (size_t)cus * 16 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    enum { NOPS = 61 };
    const rawk ks[NOPS] = {raw<0>,  raw<1>,  raw<2>,  raw<3>,  raw<4>,  raw<5>,  raw<6>,  raw<7>,
                           raw<8>,  raw<9>,  raw<10>, raw<11>, raw<12>, raw<13>, raw<14>, raw<15>,
                           raw<16>, raw<17>, raw<18>, raw<19>, raw<20>, raw<21>, raw<22>, raw<23>, raw<24>, raw<25>, raw<26>, raw<27>, raw<28>, raw<29>, raw<30>, raw<31>, raw<32>, raw<33>, raw<34>, raw<35>, raw<36>, raw<37>, raw<38>, raw<39>, raw<40>, raw<41>, raw<42>, raw<43>, raw<44>, raw<45>, raw<46>, raw<47>, raw<48>, raw<49>, raw<50>, raw<51>, raw<52>, raw<53>, raw<54>, raw<55>, raw<56>, raw<57>, raw<58>, raw<59>, raw<60>};
    const char *names[NOPS] = {"v_xor_b32", "v_bitop3_b32", "v_lshrrev_b32", "v_and_or_b32", "v_add_u32",
                               "v_add_f32", "v_mul_u32_u24", "v_or3_b32", "v_bfe_u32", "v_bfi_b32",
                               "v_sub_u32", "v_or_b32", "v_lshl_or_b32", "v_add3_u32", "v_lshl_add_u32",
                               "v_lshrrev_b32_e64", "v_alignbit_b32", "v_perm_b32", "v_lshlrev_b32",
                               "v_xad_u32", "v_or3_b32_sgpr", "v_bitop3_b32_sgpr", "v_and_b32_e32_literal", "v_and_b32_e32_sgpr", "v_and_b32_e64", "v_bitop3_b32_inlineconst", "v_bitop3_b32_0x96", "v_not_b32", "v_lshlrev_b32_e32_const3", "v_lshrrev_b32_e32_const3", "v_lshlrev_b32_e64", "v_cndmask_b32_e32", "v_xor_b32_e64", "v_or_b32_e32_sgpr", "v_add_u32_e64", "v_mov_b32", "v_cmp_eq_u32_e32", "or3+dep_xor_pair", "or3+indep_xor_pair", "v_or_b32_e32_literal", "lshl1+xor_pair", "lshr1+xor_pair", "v_bitop3_b32_sgpr_src0", "v_mul_lo_u16", "v_pk_mul_lo_u16", "v_mad_u32_u24", "v_mul_f32", "v_or_b32_sdwa", "v_lshlrev_b16", "v_pk_lshlrev_b16", "v_mov_b32_dpp", "v_cndmask_b32_e64_sgprmask", "v_cmp_eq_u32_e64_sdst", "v_mul_hi_u32_u24", "v_subrev_u32", "v_add_u32_e32_literal", "v_max_u32", "v_ashrrev_i32", "v_mul_lo_u32", "v_ffbl_b32", "v_bcnt_u32_b32"};
    const int iters = 512;
    printf("{\"cus\": %d, \"raw\": {", cus);
    for (int o = 0; o < NOPS; ++o) {
        printf("%s\"%s\": {", o ? ", " : "", names[o]);
        const int wps[4] = {1, 2, 4, 8};
        for (int wi = 0; wi < 4; ++wi) {
            const int blocks = cus * wps[wi];  // 256-thread blocks: waves per SIMD = blocks per CU
            hipLaunchKernelGGL(ks[o], dim3(blocks), dim3(256), 0, 0, sink, iters);
            hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ks[o], dim3(blocks), dim3(256), 0, 0, sink, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // wave instructions per SIMD, cycles at 2.4 GHz
            const double winst = (double)wps[wi] * iters * 16 * 8 * 5;
            printf("%s\"%d\": %.3f", wi ? ", " : "", wps[wi], ms * 1e-3 * 2.4e9 / winst);
        }
        printf("}");
    }
    printf("}, \"raw_unit\": \"cycles per wave64 instruction per SIMD at 2.4 GHz\"");

    const int nb = 4096;
    uint32_t *h = (uint32_t *)malloc(nb * 27 * 4);
    srand(1);
    for (int i = 0; i < nb * 27; ++i) h[i] = (uint32_t)rand() & plane::ROWS;
    uint32_t *d;
    hipMalloc(&d, nb * 27 * 4);
    hipMemcpy(d, h, nb * 27 * 4, hipMemcpyHostToDevice);
    struct {
        const char *name;
        uint32_t lo, hi;
    } masks[] = {{"all64", ~0u, ~0u},       {"lo32", ~0u, 0u},          {"lo16", 0xFFFFu, 0u},
                 {"lo8", 0xFFu, 0u},         {"lo1", 1u, 0u},            {"even32", 0x55555555u, 0x55555555u},
                 {"q0q2", 0xFFFFu, 0xFFFFu}, {"hi32", 0u, ~0u},          {"lo1hi1", 1u, 1u}};
    printf(", \"pass_masked_us\": {");
    const int blocks = cus * 4;
    for (int mi = 0; mi < 9; ++mi) {
        hipLaunchKernelGGL(pass_masked, dim3(blocks), dim3(256), 0, 0, d, sink, nb, masks[mi].lo, masks[mi].hi);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r)
            hipLaunchKernelGGL(pass_masked, dim3(blocks), dim3(256), 0, 0, d, sink, nb, masks[mi].lo, masks[mi].hi);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%s\"%s\": %.1f", mi ? ", " : "", masks[mi].name, ms * 1e3 / 5);
    }
    printf("}, \"pass_iters\": %d, \"waves_per_simd\": 4}\n", ITER);
    return 0;
}
