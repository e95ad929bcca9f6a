// bank_probe.hip -- does a VALU instruction whose VGPR sources share a
// register bank (v mod 4) issue slower on gfx950?  v_bitop3_b32 and v_and_b32
// with sources in one bank against sources in distinct banks; no dependency
// between the instructions of a group (destinations rotate, never read).
// Diagnostic, not product code.
//   hipcc --offload-arch=gfx950 -O3 -o bank_probe scripts/microbench/bank_probe.hip && ./bank_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(X) X X X X X X X X
#define R64(X) R8(R8(X))

#define K(name, body)                                                                                   \
    __global__ __launch_bounds__(256) void name(unsigned *out, int iters)                             \
    {                                                                                                   \
        asm volatile("v_mov_b32 v20, 1\n v_mov_b32 v21, 2\n v_mov_b32 v22, 3\n v_mov_b32 v24, 5\n"     \
                     "v_mov_b32 v28, 9\n v_mov_b32 v25, 7" ::: "v20", "v21", "v22", "v24", "v25", "v28"); \
        for (int i = 0; i < iters; ++i) {                                                               \
            asm volatile(R64(body) ::: "v10", "v11", "v12", "v13");                                    \
        }                                                                                               \
        unsigned r;                                                                                     \
        asm volatile("v_mov_b32 %0, v10" : "=v"(r));                                                   \
        out[blockIdx.x * 256 + threadIdx.x] = r;                                                        \
    }

K(bop3_same, "v_bitop3_b32 v10, v20, v24, v28 bitop3:0x96\n v_bitop3_b32 v11, v20, v24, v28 bitop3:0x96\n")
K(bop3_dist, "v_bitop3_b32 v10, v20, v21, v22 bitop3:0x96\n v_bitop3_b32 v11, v20, v21, v22 bitop3:0x96\n")
K(bop3_two, "v_bitop3_b32 v10, v20, v24, v21 bitop3:0x96\n v_bitop3_b32 v11, v20, v24, v21 bitop3:0x96\n")
K(and_same, "v_and_b32 v10, v20, v24\n v_and_b32 v11, v20, v24\n")
K(and_dist, "v_and_b32 v10, v20, v21\n v_and_b32 v11, v20, v21\n")
K(mul24_dist, "v_mul_u32_u24 v10, v20, v21\n v_mul_u32_u24 v11, v20, v21\n")
K(lshr_dist, "v_lshrrev_b32 v10, 10, v20\n v_lshrrev_b32 v11, 20, v21\n")

int main()
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *out;
    (void)hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct { const char *n; void (*k)(unsigned *, int); } ks[] = {
        {"bop3_same_bank3", bop3_same}, {"bop3_distinct", bop3_dist}, {"bop3_two_same", bop3_two},
        {"and_same_bank", and_same},    {"and_distinct", and_dist},   {"mul24", mul24_dist}, {"lshr", lshr_dist}};
    const int iters = 2000;
    for (int w = 4; w <= 8; w += 4)
        for (auto &k : ks) {
            const int blocks = cus * w;  // 256-thread blocks: w waves per SIMD
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 10);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            // wave64 instructions per SIMD: blocks * 4 waves / (cus * 4 SIMDs) * iters * 128
            const double per_simd = (double)blocks * 4 / (cus * 4.0) * iters * 128;
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst\": %.3f}\n", k.n, w,
                   ms * 1e-3 * 2.4e9 / per_simd);
        }
    return 0;
}
