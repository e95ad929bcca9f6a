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

template <int OP>
__global__ __launch_bounds__(256) void raw(uint32_t *sink, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, k = a0 * 3;
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
        }
    }
    sink[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
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
    const rawk ks[7] = {raw<0>, raw<1>, raw<2>, raw<3>, raw<4>, raw<5>, raw<6>};
    const char *names[7] = {"v_xor_b32", "v_bitop3_b32", "v_lshrrev_b32", "v_and_or_b32", "v_add_u32", "v_add_f32",
                            "v_mul_u32_u24"};
    const int iters = 512;
    printf("{\"cus\": %d, \"raw\": {", cus);
    for (int o = 0; o < 7; ++o) {
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
