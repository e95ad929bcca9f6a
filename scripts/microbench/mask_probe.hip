// mask_probe.hip -- why does plane::pass run ~1.8x SLOWER when only <= 8 lanes
// of a wave are active (profiles/r02_valu_rates.json pass_masked_us)?
// Diagnostic, not product code.  Each wave times its own loop with
// s_memtime (shader clock) from inside the divergent region, so launch and
// drain effects are out of the number:
//   * raw VALU forms (8 independent chains per lane, inline asm) and the
//     plane pass, under exec masks of 1 .. 64 lanes and different layouts;
//   * at 1 wave per SIMD (the wave's own issue and latency) and at 4 (the
//     plane kernel's occupancy).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-sched-strategy=iterative-ilp \
//         -o mask_probe scripts/microbench/mask_probe.hip && ./mask_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../sudoku_solver_distributed_amd/csrc/plane_solver.h"

#define ITER 64

#define CH8(S) S(a0, a1) S(a1, a2) S(a2, a3) S(a3, a4) S(a4, a5) S(a5, a6) S(a6, a7) S(a7, a0)
#define XOR(d, s) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(s));
#define BOP3(d, s) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x9c" : "+v"(d) : "v"(s), "v"(k));
#define MUL24(d, s) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(d) : "v"(s));
#define LSHR(d, s) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(d) : "v"(s));
// one dependent chain: the latency of one instruction
#define DEP(d, s) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a0) : "v"(a1));

template <int OP>
__global__ __launch_bounds__(256, 4) void probe(const uint32_t *boards, uint64_t *cyc, uint32_t *sink, uint32_t mlo,
                                                uint32_t mhi)
{
    const int g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    const uint32_t m = lane < 32 ? mlo : mhi;
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, k = a0 * 3;
    if (!((m >> (lane & 31)) & 1u)) return;
    plane::Board B;
    if (OP == 9) {
        const uint32_t *src = boards + (size_t)(g % 4096) * 27;
#pragma unroll
        for (int w = 0; w < 27; ++w) B.P[w / 3][w % 3] = src[w];
        B.Det[0] = B.Det[1] = B.Det[2] = 0;
    }
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
    for (int it = 0; it < ITER; ++it) {
        if (OP == 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) { CH8(XOR) }
        }
        if (OP == 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r) { CH8(BOP3) }
        }
        if (OP == 2) {
#pragma unroll
            for (int r = 0; r < 16; ++r) { CH8(MUL24) }
        }
        if (OP == 3) {
#pragma unroll
            for (int r = 0; r < 16; ++r) { CH8(LSHR) }
        }
        if (OP == 4) {
#pragma unroll
            for (int r = 0; r < 16; ++r) { CH8(DEP) }
        }
        if (OP == 9) {
            uint32_t und[3];
            acc += (uint32_t)plane::pass(B, und) + und[0] + und[1] + und[2];
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    // first active lane records the wave's cycles (a vector store)
    const uint64_t act = __builtin_amdgcn_read_exec();
    if (lane == __builtin_ctzll(act)) cyc[g >> 6] = t1 - t0;
    sink[g] = acc ^ a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*kfn)(const uint32_t *, uint64_t *, uint32_t *, uint32_t, uint32_t);

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int nb = 4096;
    uint32_t *h = (uint32_t *)malloc(nb * 27 * 4);
    srand(1);
    for (int i = 0; i < nb * 27; ++i) h[i] = (uint32_t)rand() & plane::ROWS;
    uint32_t *d, *sink;
    uint64_t *cyc;
    hipMalloc(&d, nb * 27 * 4);
    hipMemcpy(d, h, nb * 27 * 4, hipMemcpyHostToDevice);
    const size_t maxw = (size_t)cus * 4 * 4;
    hipMalloc(&sink, maxw * 64 * 4);
    hipMalloc(&cyc, maxw * 8);
    uint64_t *hc = (uint64_t *)malloc(maxw * 8);
    struct {
        const char *name;
        kfn f;
        double insts;  // wave instructions per loop iteration
    } ops[] = {{"xor8", probe<0>, 128}, {"bitop3_8", probe<1>, 128}, {"mul24_8", probe<2>, 128},
               {"lshr8", probe<3>, 128}, {"xor_dep1", probe<4>, 128}, {"pass", probe<9>, 1}};
    struct {
        const char *name;
        uint32_t lo, hi;
    } masks[] = {{"all64", ~0u, ~0u},  {"lo32", ~0u, 0u},      {"lo16", 0xFFFFu, 0u},   {"lo12", 0xFFFu, 0u},
                 {"lo9", 0x1FFu, 0u},  {"lo8", 0xFFu, 0u},      {"lo4", 0xFu, 0u},       {"lo1", 1u, 0u},
                 {"hi8", 0u, 0xFFu},   {"lo1hi1", 1u, 1u},      {"lo4hi4", 0xFu, 0xFu},  {"lo8hi8", 0xFFu, 0xFFu},
                 {"stride8", 0x01010101u, 0x01010101u},         {"even32", 0x55555555u, 0x55555555u},
                 {"b8_15", 0xFF00u, 0u}};
    const int nm = sizeof masks / sizeof masks[0], no = sizeof ops / sizeof ops[0];
    printf("{\"cus\": %d, \"unit\": \"shader cycles per wave instruction (pass: per pass): [mean, max] over waves\", "
           "\"iters\": %d, \"results\": {",
           cus, ITER);
    for (int o = 0; o < no; ++o) {
        printf("%s\"%s\": {", o ? ", " : "", ops[o].name);
        for (int wps = 1; wps <= 4; wps += 3) {
            printf("%s\"w%d\": {", wps == 1 ? "" : ", ", wps);
            const int blocks = cus * wps, waves = blocks * 4;
            for (int mi = 0; mi < nm; ++mi) {
                hipLaunchKernelGGL(ops[o].f, dim3(blocks), dim3(256), 0, 0, d, cyc, sink, masks[mi].lo, masks[mi].hi);
                hipMemset(cyc, 0, waves * 8);
                hipLaunchKernelGGL(ops[o].f, dim3(blocks), dim3(256), 0, 0, d, cyc, sink, masks[mi].lo, masks[mi].hi);
                hipMemcpy(hc, cyc, waves * 8, hipMemcpyDeviceToHost);
                double sum = 0, mx = 0;
                for (int w = 0; w < waves; ++w) {
                    sum += (double)hc[w];
                    mx = (double)hc[w] > mx ? (double)hc[w] : mx;
                }
                printf("%s\"%s\": [%.2f, %.2f]", mi ? ", " : "", masks[mi].name, sum / waves / (ITER * ops[o].insts),
                       mx / (ITER * ops[o].insts));
            }
            printf("}");
        }
        printf("}");
    }
    printf("}}\n");
    return 0;
}
