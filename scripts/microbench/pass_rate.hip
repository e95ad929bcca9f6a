// pass_rate.hip -- VALU issue ceiling of plane::pass at the plane kernel's
// occupancy: every lane runs ITER passes on a board held in registers (no
// queue, no I/O, no divergence).  Diagnostic, not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-sched-strategy=iterative-ilp \
//         -o pass_rate scripts/microbench/pass_rate.hip && ./pass_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../sudoku_solver_distributed_amd/csrc/plane_solver.h"

#ifndef WPE
#define WPE 4
#endif
#define ITER 256
#ifndef VPP
#define VPP 1463  // VALU per pass (profiles/isa_plane_pass.json)
#endif

__global__ __launch_bounds__(256, WPE) void pass_loop(const uint32_t *boards, uint32_t *sink, int nboards)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
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

int main(int argc, char **argv)
{
    // boards: random clue patterns are fine -- a pass costs the same on any board
    const int nb = 4096;
    uint32_t *h = (uint32_t *)malloc(nb * 27 * 4);
    srand(1);
    for (int i = 0; i < nb * 27; ++i) h[i] = (uint32_t)rand() & plane::ROWS;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int bpc = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, pass_loop, 256, 0);
    uint32_t *d, *sink;
    hipMalloc(&d, nb * 27 * 4);
    hipMalloc(&sink, (size_t)cus * bpc * 256 * 4);
    hipMemcpy(d, h, nb * 27 * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // argv: blocks per CU to launch (waves per SIMD = blocks per CU: 256-thread blocks)
    for (int a = 1; a <= (argc > 1 ? argc - 1 : 1); ++a) {
    const int want = argc > 1 ? atoi(argv[a]) : bpc;
    const int blocks = cus * (want < bpc ? want : bpc);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(pass_loop, dim3(blocks), dim3(256), 0, 0, d, sink, nb);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(pass_loop, dim3(blocks), dim3(256), 0, 0, d, sink, nb);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double passes = (double)blocks * 256 * ITER * reps;
    printf("{\"cus\": %d, \"max_blocks_per_cu\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"passes_per_s\": %.4g, "
           "\"valu_frac_at_%d_per_pass\": %.3f}\n",
           cus, bpc, blocks / cus, ms, passes / (ms * 1e-3), VPP, passes / (ms * 1e-3) * VPP / 78.6432e12);
    }
    return 0;
}
