// Probe of gfx950's row-exchange VALU ops (v_permlane16_swap_b32,
// v_permlane32_swap_b32) and DPP row_ror: what each lane receives, for the
// wave-wide tail solver's cross-band sums (plane_wide.h).  Prints, per op,
// the source lane each lane of the two results reads.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(unsigned *out)
{
    const unsigned l = __lane_id();
    const unsigned a = l, b = 100u + l;
    auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    out[l] = r16[0];
    out[64 + l] = r16[1];
    out[128 + l] = r32[0];
    out[192 + l] = r32[1];
    out[256 + l] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)a, 0x121, 0xF, 0xF, false);  // row_ror:1
}

int main()
{
    unsigned *d, h[320];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *name[5] = {"permlane16_swap.first", "permlane16_swap.second", "permlane32_swap.first",
                           "permlane32_swap.second", "dpp row_ror:1"};
    for (int k = 0; k < 5; ++k) {
        printf("%s:", name[k]);
        for (int l = 0; l < 64; ++l) printf(" %u", h[64 * k + l]);
        printf("\n");
    }
    return 0;
}
