// plane_kernels.hip -- translation unit of the lane-per-board digit-plane
// solve kernel (plane_kernel.h).  Built on its own (build.py) with
// -mllvm -amdgpu-sched-strategy=iterative-minreg: the default scheduler
// interleaves the nine digits of a pass for ILP and needs ~136 VGPRs, the
// min-register strategy ~103, so four waves fit per SIMD without spills
// (one wave alone issues VALU every 4 cycles, two saturate the SIMD).
#include "common.h"
#include "plane_kernel.h"

hipError_t sdk_launch_plane(const uint8_t *puzzles, uint8_t *sols, int32_t *status, int64_t n,
                            unsigned long long *ws, uint32_t *stack, int ordered, int order, int64_t threads,
                            hipStream_t st)
{
    const int64_t blocks = (threads + PLANE_THREADS - 1) / PLANE_THREADS;
    hipLaunchKernelGGL(plane_kernel, dim3((unsigned)blocks), dim3(PLANE_THREADS), 0, st, puzzles, sols, status, n, ws,
                       stack, ordered, order);
    return hipGetLastError();
}

int sdk_plane_blocks_per_cu()
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, plane_kernel, PLANE_THREADS, 0) != hipSuccess || nb <= 0)
        nb = 4;
    return nb > 8 ? 8 : nb;
}
