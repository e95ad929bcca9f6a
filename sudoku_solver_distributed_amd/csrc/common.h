// common.h -- definitions shared by the two translation units
// (sudoku_kernels.hip: wave-per-board kernel, check / task / frontier kernels
// and the C ABI; plane_kernels.hip: the lane-per-board digit-plane kernel).
#ifndef SDK_COMMON_H
#define SDK_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sudoku_hip.h"

#define WAVES_PER_BLOCK 4
// internal status of a board the plane kernel leaves to the packed kernel
// (never visible to callers: the deferred pass overwrites it)
#define SDK_DEFERRED 0x7FFF0001
#define BLOCK_THREADS (64 * WAVES_PER_BLOCK)

// ---------------------------------------------------------------- workspace
// word layout of the device workspace (uint64 words)
enum {
    WS_QUEUE = 0,        // chunked board queue head (re-armed every call)
    WS_BEST = 1,         // ordered mode: lowest solved index (re-armed to INT64_MAX)
    WS_DEFER_COUNT = 2,  // boards the plane kernel handed back (list entries, re-armed)
    WS_DEFER_OVER = 3,   // 1: the list overflowed, every deferred board is found by status (re-armed)
    WS_ARM_WORDS = 4,    // words re-armed per call
    WS_GEN = 4,          // launch generation (low 32 bits, never 0): arm_kernel adds one per call; the
                         // tail pool's ready flags hold it, so a flag left by an earlier launch never reads as set
    WS_ERR_SLOT = 5,     // diagnostic: the pool slot of the last flag-wait timeout
    WS_STACK_BYTE = 256, // the plane kernel's per-lane stacks start here, then the deferred list
    WS_FINISHED = 8,   // statistics (accumulate until sdk_read_stats(reset))
    WS_SOLVED = 9,
    WS_GUESSES = 10,
    WS_SWEEPS = 11,
    WS_DEFERRED = 12,  // boards the plane kernel left to the packed kernel
    WS_ASSIGNED = 13,  // boards handed to the solve kernels (each launch adds its n): == WS_FINISHED once done
    WS_ERROR = 14,     // SDK_ERR_* bits, sticky until sdk_verify_workspace reports them
    WS_RESERVED = 15,  // always 0 (sdk_read_stats / sdk_verify_workspace out[3])
    WS_WORDS = 16
};
// WS_ERROR bits
#define SDK_ERR_POOL_WAIT 1u  // a pool consumer gave up waiting on a claimed record: that board was not solved

__device__ __forceinline__ uint32_t lowbit(uint32_t x) { return x & (0u - x); }

// Orders this wave's LDS accesses (a single wave's DS ops execute in order;
// this keeps the compiler from moving them and drains returns).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}

// wave-uniform "any lane": the ballot's SGPR pair, no VGPR round trip
__device__ __forceinline__ bool wany(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

__device__ __forceinline__ void cell_units(int cell, int &r, int &c, int &b)
{
    r = cell / 9;
    c = cell - r * 9;
    b = (r / 3) * 3 + c / 3;
}

// The walk's next cell among the empty cells {eb0 (cells 0..63), eb1 (64..80)},
// not both zero.  Scalar bit work only.
__device__ __forceinline__ int order_cell(uint64_t eb0, uint64_t eb1, int order)
{
    if (order == SDK_ORDER_NODE)  // node.py:63-65: row-major first
        return eb0 ? __builtin_ctzll(eb0) : 64 + __builtin_ctzll(eb1);
    // gen.py:11-15: last row holding an empty cell, its first empty column
    const int hi = eb1 ? 64 + 63 - __builtin_clzll(eb1) : 63 - __builtin_clzll(eb0);
    const int start = (hi / 9) * 9;
    if (start >= 64) return start + __builtin_ctzll(eb1 >> (start - 64));
    const uint64_t m = eb0 & (~0ull << start);
    return m ? __builtin_ctzll(m) : 64 + __builtin_ctzll(eb1);
}

// Several batches in one plane launch (sdk_solve_batches): the queue hands
// out virtual indices over the batches laid end to end; a lane's board id is
// batch j << PLANE_BATCH_SHIFT | index in batch j (deferred-list entries too).
// Passed by value as a kernel argument (1032 bytes at 32 batches).
struct PlaneBatches {
    int64_t end[SDK_MAX_BATCHES];  // virtual index one past batch j (cumulative, ascending)
    const uint8_t *in[SDK_MAX_BATCHES];
    uint8_t *out[SDK_MAX_BATCHES];
    int32_t *status[SDK_MAX_BATCHES];
    int count;
};
#define PLANE_BATCH_SHIFT 40
#define PLANE_LOCAL_MASK ((1ll << PLANE_BATCH_SHIFT) - 1)

// Launch the plane kernel (plane_kernels.hip) and report its occupancy.
hipError_t sdk_launch_plane(const uint8_t *puzzles, uint8_t *sols, int32_t *status, int64_t n,
                            unsigned long long *ws, uint32_t *stack, int64_t *defer_list, int ordered, int order,
                            int64_t threads, int pipelined, hipStream_t st);
// the same over several batches (unordered only)
hipError_t sdk_launch_plane_multi(const PlaneBatches &bs, unsigned long long *ws, uint32_t *stack,
                                  int64_t *defer_list, int order, int64_t threads, int pipelined, hipStream_t st);
int sdk_plane_blocks_per_cu();
#define PLANE_MAX_DEPTH 32
// plane kernel workgroup: ONE wave.  Its waves share nothing (each has its
// own LDS areas), and a one-wave workgroup frees its LDS the moment its wave
// exits, so during a launch's drain the next launch in flight starts wave by
// wave instead of block by block (+3 %; 256 = the former 4-wave block)
#ifndef SDK_PLANE_BLOCK
#define SDK_PLANE_BLOCK 64
#endif
#define PLANE_THREADS SDK_PLANE_BLOCK
#define PLANE_STACK_WORDS 32  // per level: 27 planes + branch entry, padded to one 128-byte line
// board indices the plane kernel hands to the wave kernel (int64 each; more
// than this and the wave kernel finds them by scanning the statuses)
#define PLANE_DEFER_CAP (1 << 20)
// The drained waves' tail pool (plane_kernel.h, tail mode 2), after the
// deferred list: per XCD, one 128-byte control line (slots reserved, records
// published, slots taken; re-armed every call), PLANE_POOL_CAP records of
// PLANE_POOL_REC dwords, then one ready flag (uint32) per record.  A ready
// flag holds the launch generation (WS_GEN) of the record it publishes, so
// flags need no clearing: one left by an earlier launch (or set after its
// consumer gave up) never matches a later launch's generation.
#define PLANE_POOL_XCDS 8
#define PLANE_POOL_CAP 16384
#define PLANE_POOL_REC 36
#define PLANE_POOL_CTL 32       // one 128-byte line
#define PLANE_POOL_ARM_WORDS 4  // its words 0..3
#define PLANE_POOL_STRIDE (PLANE_POOL_CTL + PLANE_POOL_CAP * (PLANE_POOL_REC + 1))  // dwords per XCD
#define PLANE_POOL_BYTES ((size_t)PLANE_POOL_XCDS * PLANE_POOL_STRIDE * 4)

#endif  // SDK_COMMON_H
