// plane_kernels.hip -- translation unit of the lane-per-board digit-plane
// solve kernel (plane_kernel.h), built on its own by build.py with LLVM's
// iterative-ilp machine scheduler (+1.4 % over the default, same registers;
// $SDK_PLANE_SCHED selects another strategy for A/B builds).  The pass pins its board between digits (plane_solver.h PS_PIN),
// which keeps the kernel at ~120 VGPRs: four waves per SIMD, no spills (forcing
// five or six waves spills and measured 4 % / 13 % slower).
#include <stdlib.h>

#include <atomic>

#include "common.h"
#include "plane_kernel.h"

// runtime tuning knobs (A/B without a rebuild): $SDK_PLANE_REFILL idle lanes
// before a wave refills, $SDK_PLANE_TAIL active lanes at or below which a
// drained wave hands its last boards to the tail solver (0: off; at most
// PLANE_TAIL_MAX), $SDK_PLANE_TAIL_MODE where the wave-wide solver continues
// them (2: through the XCD's tail pool, 1: on the wave itself),
// $SDK_PLANE_CHUNK most boards a wave claims from the queue at once (0: one
// claim per refill), $SDK_PLANE_MRV passes on a board before its search
// switches to the completion count (plane::search_step; 0: never).
// Pipelined launches (SDK_GRID_PIPELINED: another launch is queued behind)
// take $SDK_PLANE_PIPE_TAIL / $SDK_PLANE_PIPE_TAIL_MODE instead: their
// drained waves exit after their own tails, the next launch wants the slots
// (pool on a pipelined launch: -5 % at 100 steps in flight; off the pipeline
// +16 % on the N = 8 rank's runs).  sdk_set_plane_tuning's
// tail / tail mode apply to both.
static int env_int(const char *name, int dflt)
{
    const char *e = getenv(name);
    return e && e[0] ? atoi(e) : dflt;
}

// sdk_set_plane_tuning / sdk_set_plane_search overrides (-1: the
// environment's / built-in default)
static std::atomic<int> g_refill{-1}, g_tail{-1}, g_tail_mode{-1}, g_chunk{-1}, g_mrv{-1};

int sdk_set_plane_tuning(int refill, int tail, int tail_mode, int chunk)
{
    if (refill > 64 || tail > PLANE_TAIL_MAX || tail_mode == 0 || tail_mode > 2 || refill == 0 ||
        chunk > PLANE_CHUNK_MAX)
        return -1;
    if (refill < 0 && tail < 0 && tail_mode < 0 && chunk < 0) {
        g_refill = g_tail = g_tail_mode = g_chunk = -1;
        return 0;
    }
    if (refill >= 0) g_refill = refill;
    if (tail >= 0) g_tail = tail;
    if (tail_mode >= 0) g_tail_mode = tail_mode;
    if (chunk >= 0) g_chunk = chunk;
    return 0;
}

struct PlaneKnobs {
    int refill, tail, tail_mode, chunk;
    uint32_t mrv_after, pool_polls;
};

static PlaneKnobs plane_knobs(int pipelined)
{
    static const int refill_env = env_int("SDK_PLANE_REFILL", SDK_PLANE_REFILL);
    static const int tail_env = env_int("SDK_PLANE_TAIL", SDK_PLANE_TAIL);
    static const int tail_mode_env = env_int("SDK_PLANE_TAIL_MODE", SDK_PLANE_TAIL_MODE);
    static const int chunk_env = env_int("SDK_PLANE_CHUNK", SDK_PLANE_CHUNK);
    static const int mrv_env = env_int("SDK_PLANE_MRV", SDK_PLANE_MRV);
    static const int pipe_tail_env = env_int("SDK_PLANE_PIPE_TAIL", SDK_PLANE_PIPE_TAIL);
    static const int pipe_tail_mode_env = env_int("SDK_PLANE_PIPE_TAIL_MODE", SDK_PLANE_PIPE_TAIL_MODE);
    const int refill = g_refill >= 0 ? g_refill.load() : refill_env;
    int tail = g_tail >= 0 ? g_tail.load() : pipelined ? pipe_tail_env : tail_env;
    tail = tail > PLANE_TAIL_MAX ? PLANE_TAIL_MAX : tail;
    int tail_mode = g_tail_mode >= 0 ? g_tail_mode.load() : pipelined ? pipe_tail_mode_env : tail_mode_env;
    tail_mode = tail_mode < 1 ? 1 : tail_mode > 2 ? 2 : tail_mode;  // ($SDK_PLANE_*TAIL_MODE is not range-checked)
    int chunk = g_chunk >= 0 ? g_chunk.load() : chunk_env;
    chunk = chunk > PLANE_CHUNK_MAX ? PLANE_CHUNK_MAX : chunk;  // ($SDK_PLANE_CHUNK is not range-checked)
    int mrv = g_mrv >= 0 ? g_mrv.load() : mrv_env;
    mrv = mrv < 0 ? 0 : mrv > (int)plane::MST_PASSES ? (int)plane::MST_PASSES : mrv;
    // flag polls before a pool consumer gives up (~1 s; read at every launch:
    // tests/test_gpu_full_size.py forces 0 to see the host raise, then
    // recovers on the same workspace)
    const uint32_t polls = (uint32_t)env_int("SDK_PLANE_POOL_POLLS", 1 << 23);
    return {refill, tail, tail_mode, chunk, (uint32_t)mrv, polls};
}

int sdk_set_plane_search(int mrv_after)
{
    if (mrv_after > (int)plane::MST_PASSES) return -2;
    const int prev = (int)plane_knobs(0).mrv_after;  // the setting in effect, default or not
    g_mrv = mrv_after < 0 ? -1 : mrv_after;
    return prev;
}

hipError_t sdk_launch_plane(const uint8_t *puzzles, uint8_t *sols, int32_t *status, int64_t n,
                            unsigned long long *ws, uint32_t *stack, int64_t *defer_list, int ordered, int order,
                            int64_t threads, int pipelined, hipStream_t st)
{
    const PlaneKnobs k = plane_knobs(pipelined);
    const int64_t blocks = (threads + PLANE_THREADS - 1) / PLANE_THREADS;
    hipLaunchKernelGGL(plane_kernel, dim3((unsigned)blocks), dim3(PLANE_THREADS), 0, st, puzzles, sols, status, n, ws,
                       stack, defer_list, ordered, order, k.refill, k.tail, k.tail_mode, k.chunk, k.mrv_after, k.pool_polls);
    return hipGetLastError();
}

hipError_t sdk_launch_plane_multi(const PlaneBatches &bs, unsigned long long *ws, uint32_t *stack,
                                  int64_t *defer_list, int order, int64_t threads, int pipelined, hipStream_t st)
{
    const PlaneKnobs k = plane_knobs(pipelined);
    const int64_t blocks = (threads + PLANE_THREADS - 1) / PLANE_THREADS;
    hipLaunchKernelGGL(plane_kernel_multi, dim3((unsigned)blocks), dim3(PLANE_THREADS), 0, st, bs, ws, stack,
                       defer_list, order, k.refill, k.tail, k.tail_mode, k.chunk, k.mrv_after, k.pool_polls);
    return hipGetLastError();
}

int sdk_plane_blocks_per_cu()
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, plane_kernel, PLANE_THREADS, 0) != hipSuccess || nb <= 0)
        nb = 4;
    const int cap = 32 * 64 / PLANE_THREADS;  // 32 waves per CU
    return nb > cap ? cap : nb;
}
