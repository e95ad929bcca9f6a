// lat_probe.hip -- dependent-chain latency and independent-chain issue cost of
// a few VALU forms on gfx950, at 1 and 4 waves per SIMD.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -o lat_probe scripts/microbench/lat_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N 256
#define OP_MUL24(x) asm volatile("v_mul_u32_u24 %0, %0, %0" : "+v"(x))
#define OP_MUL16(x) asm volatile("v_mul_lo_u16 %0, 7, %0" : "+v"(x))
#define OP_XOR(x) asm volatile("v_xor_b32 %0, 0x55, %0" : "+v"(x))
#define OP_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 10, %0" : "+v"(x))
#define OP_LSHL(x) asm volatile("v_lshlrev_b32 %0, 10, %0" : "+v"(x))
#define OP_LSHR(x) asm volatile("v_lshrrev_b32 %0, 10, %0" : "+v"(x))
#define OP_BOP3(x) asm volatile("v_bitop3_b32 %0, %0, %0, %0 bitop3:0x96" : "+v"(x))
#define OP_MAD24(x) asm volatile("v_mad_u32_u24 %0, %0, %0, %0" : "+v"(x))

#define KERN(name, OP)                                                                     \
    __global__ void dep_##name(uint32_t *o, uint32_t s)                                    \
    {                                                                                      \
        uint32_t x = s + threadIdx.x;                                                      \
        for (int i = 0; i < N; ++i) {                                                      \
            OP(x); OP(x); OP(x); OP(x); OP(x); OP(x); OP(x); OP(x);                        \
        }                                                                                  \
        o[blockIdx.x * blockDim.x + threadIdx.x] = x;                                      \
    }                                                                                      \
    __global__ void ind_##name(uint32_t *o, uint32_t s)                                    \
    {                                                                                      \
        uint32_t a = s + threadIdx.x, b = a + 1, c = a + 2, d = a + 3;                     \
        uint32_t e = a + 4, f = a + 5, g = a + 6, h = a + 7;                               \
        for (int i = 0; i < N; ++i) {                                                      \
            OP(a); OP(b); OP(c); OP(d); OP(e); OP(f); OP(g); OP(h);                        \
        }                                                                                  \
        o[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;          \
    }

KERN(mul24, OP_MUL24)
KERN(mul16, OP_MUL16)
KERN(xor, OP_XOR)
KERN(lshlor, OP_LSHLOR)
KERN(lshl, OP_LSHL)
KERN(lshr, OP_LSHR)
KERN(bop3, OP_BOP3)
KERN(mad24, OP_MAD24)

typedef void (*K)(uint32_t *, uint32_t);

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *o;
    hipMalloc(&o, (size_t)cus * 16 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"mul24", "mul16", "xor", "lshlor", "lshl", "lshr", "bop3", "mad24"};
    K dep[] = {dep_mul24, dep_mul16, dep_xor, dep_lshlor, dep_lshl, dep_lshr, dep_bop3, dep_mad24};
    K ind[] = {ind_mul24, ind_mul16, ind_xor, ind_lshlor, ind_lshl, ind_lshr, ind_bop3, ind_mad24};
    printf("{\"clock_ghz_assumed\": 2.4, \"insts_per_wave\": %d, \"runs\": [", 8 * N);
    bool first = true;
    for (int k = 0; k < 8; ++k)
        for (int kind = 0; kind < 2; ++kind)
            for (int wps = 1; wps <= 4; wps *= 4) {
                const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD each
                K f = kind ? ind[k] : dep[k];
                for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, o, 1u);
                hipEventRecord(e0);
                const int reps = 20;
                for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, o, 1u);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                // cycles per instruction per wave (a dependent chain: its latency) and per SIMD
                const double cyc = ms * 1e-3 / reps * 2.4e9;
                const double per_wave = cyc / (8.0 * N);
                printf("%s{\"op\": \"%s\", \"chain\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_wave\": %.3f, "
                       "\"cycles_per_inst_per_simd\": %.3f}",
                       first ? "" : ", ", names[k], kind ? "8 independent" : "dependent", wps, per_wave,
                       per_wave / wps);
                first = false;
            }
    printf("]}\n");
    return 0;
}
