// sudoku_kernels.hip -- MI355X (gfx950, CDNA4) Sudoku solver kernels + C ABI.
//
// Hot path: batch solving of 9x9 boards, bit-identical to the reference's
// backtracking walks.  Both fill one cell at a time with digits 1..9
// ascending; they differ in which empty cell they pick:
//   SDK_ORDER_GEN  gen.py:6-28 solve_sudoku -- its scan (gen.py:11-15) breaks
//                  only the column loop, so it takes the first empty cell of
//                  the LAST row that has one (rows 8..0, columns 0..8);
//   SDK_ORDER_NODE node.py:62-74 solve_sudoku_recursive -- first empty cell
//                  in row-major order.
// Either way the cell sequence is a fixed order of the empty cells, so the
// walk's first solution is the lexicographically smallest completion in that
// order.  We reach the same board with far fewer nodes by interleaving sound
// propagation (naked singles, hidden singles, conflict detection) with
// branching on the same first-in-order empty cell and the same digit order:
// propagation only removes completions, never reorders them, so the first
// completion found is still the smallest one.
//
// Execution model:
//   * one 64-lane wavefront owns one board; lane l owns cell l (slot 0) and,
//     for l < 17, cell 64+l (slot 1);
//   * the 27 unit masks (rows 0-8, columns 9-17, boxes 18-26; bit d-1 = digit
//     d used) are rebuilt every sweep in the wave's LDS slice with ds_or
//     atomics, which also detect two placements of one digit in one unit;
//   * hidden singles come from per-unit "seen once" / "seen twice" masks built
//     with returning ds_or atomics (old & cand = second sighting);
//   * backtracking is a trail: every cell remembers the depth at which it was
//     filled, so undoing a guess is one compare per lane; the DFS stack (cell,
//     untried digits) is 16 bits per level, kept one level per lane in two
//     VGPRs and read/written with readlane / lane-select;
//   * waves are persistent and pull boards from a chunked global queue.
// No MFMA: this is branchy 9-bit mask work, VALU + LDS bound.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <atomic>
#include <mutex>
#include <stdlib.h>

#include "../../include/sudoku_hip.h"
#include "lane_solver.h"

#include "common.h"

#ifndef SDK_PLANE_MIN_BATCH
#define SDK_PLANE_MIN_BATCH 8192
#endif


// Per-lane view of its two cells, plus the lane's unit role (lanes 0..26).
struct Cells {
    uint32_t v0, v1;    // digit 0..9 (0 = empty)
    uint32_t lv0, lv1;  // depth at which the cell was filled (givens: 0)
    bool g0, g1;        // given
    bool nw0, nw1;      // placed since the last sweep: not yet in the unit masks
    int r0, c0, b0, r1, c1, b1;
    bool has1;
    // unit gather: lane u < 27 reads the cells ub + k*us1 + (k/3)*us2, k = 0..8
    int ub, us1, us2;
};

__device__ __forceinline__ void cell_units(int cell, int &r, int &c, int &b)
{
    r = cell / 9;
    c = cell - r * 9;
    b = (r / 3) * 3 + c / 3;
}

__device__ __forceinline__ void init_lane(Cells &s, int lane)
{
    cell_units(lane, s.r0, s.c0, s.b0);
    cell_units(lane < 17 ? 64 + lane : 80, s.r1, s.c1, s.b1);
    if (lane < 9) { s.ub = 9 * lane; s.us1 = 1; s.us2 = 0; }                      // row
    else if (lane < 18) { s.ub = lane - 9; s.us1 = 9; s.us2 = 0; }                // column
    else { const int b = lane < 27 ? lane - 18 : 0;                               // box
           s.ub = (b / 3) * 27 + (b % 3) * 3; s.us1 = 1; s.us2 = 6; }
}

// Load one board (81 bytes) into the wave.  Returns false (wave-uniform) if
// any byte is > 9.
__device__ __forceinline__ bool load_board(const uint8_t *__restrict__ src, int lane, Cells &s)
{
    s.has1 = lane < 17;
    uint32_t a = src[lane];
    uint32_t b = s.has1 ? (uint32_t)src[64 + lane] : 0u;
    s.v0 = a;
    s.v1 = b;
    s.g0 = a != 0;
    s.g1 = s.has1 && b != 0;
    s.lv0 = 0;
    s.lv1 = 0;
    s.nw0 = false;
    s.nw1 = false;
    return !wany(a > 9 || b > 9);
}

// Build the givens' unit masks (returned in lanes 0..26; W.M holds them on
// return) and the bad-unit mask.
__device__ __forceinline__ uint32_t build_given_masks(WaveLds &W, int lane, const Cells &s, uint32_t &bad)
{
    if (lane < 28) W.M[lane] = 0;
    if (lane == 0) W.bad = 0;
    wave_lds_order();
    if (s.g0) {
        uint32_t bit = 1u << (s.v0 - 1);
        uint32_t d = 0;
        if (atomicOr(&W.M[s.r0], bit) & bit) d |= 1u << s.r0;
        if (atomicOr(&W.M[9 + s.c0], bit) & bit) d |= 1u << (9 + s.c0);
        if (atomicOr(&W.M[18 + s.b0], bit) & bit) d |= 1u << (18 + s.b0);
        if (d) atomicOr(&W.bad, d);
    }
    if (s.g1) {
        uint32_t bit = 1u << (s.v1 - 1);
        uint32_t d = 0;
        if (atomicOr(&W.M[s.r1], bit) & bit) d |= 1u << s.r1;
        if (atomicOr(&W.M[9 + s.c1], bit) & bit) d |= 1u << (9 + s.c1);
        if (atomicOr(&W.M[18 + s.b1], bit) & bit) d |= 1u << (18 + s.b1);
        if (d) atomicOr(&W.bad, d);
    }
    wave_lds_order();
    bad = __builtin_amdgcn_readfirstlane(W.bad);
    return lane < 27 ? W.M[lane] : 0u;
}

enum { PROP_OPEN = 0, PROP_DEAD = 1, PROP_SOLVED = 2 };

// One propagation sweep.  Returns PROP_DEAD on a contradiction, PROP_SOLVED
// when no cell is empty, otherwise PROP_OPEN and sets `placed` if any single
// was placed (then call again).  When it returns PROP_OPEN with !placed the
// state is a fixpoint and cand0/cand1 hold every empty cell's candidates.
//
// Unit masks live in W.M across sweeps: normally only the cells placed since
// the last sweep are OR-ed in (their returning atomics also catch two
// placements of one digit in one unit); after a backtrack (`rebuild`) the
// masks are rebuilt from the givens and every filled cell.
__device__ __forceinline__ int sweep(WaveLds &W, int lane, Cells &s, uint32_t gmask, uint32_t bad,
                                     uint32_t depth, bool &rebuild, uint32_t &cand0, uint32_t &cand1,
                                     bool &placed)
{
    placed = false;
    // ---- phase A: bring the unit masks up to date; clash detection
    bool f0, f1;
    if (rebuild) {
        if (lane < 27) W.M[lane] = gmask;
        f0 = s.v0 != 0 && !s.g0;
        f1 = s.has1 && s.v1 != 0 && !s.g1;
    } else {
        f0 = s.nw0;
        f1 = s.nw1;
    }
    s.nw0 = false;
    s.nw1 = false;
    uint32_t clash = 0;
    if (rebuild || wany(f0 || f1)) {
        wave_lds_order();
        if (f0) {
            uint32_t bit = 1u << (s.v0 - 1);
            clash |= (atomicOr(&W.M[s.r0], bit) | atomicOr(&W.M[9 + s.c0], bit) |
                      atomicOr(&W.M[18 + s.b0], bit)) & bit;
        }
        if (f1) {
            uint32_t bit = 1u << (s.v1 - 1);
            clash |= (atomicOr(&W.M[s.r1], bit) | atomicOr(&W.M[9 + s.c1], bit) |
                      atomicOr(&W.M[18 + s.b1], bit)) & bit;
        }
        wave_lds_order();
    }
    rebuild = false;
    const bool e0 = s.v0 == 0;
    const bool e1 = s.has1 && s.v1 == 0;
    // unconditional reads + selects (lanes >= 17 address cell 80's units):
    // no exec-mask branches around the loads
    const uint32_t m0 = W.M[s.r0] | W.M[9 + s.c0] | W.M[18 + s.b0];
    const uint32_t m1 = W.M[s.r1] | W.M[9 + s.c1] | W.M[18 + s.b1];
    cand0 = e0 ? (~m0 & 0x1FFu) : 0u;
    cand1 = e1 ? (~m1 & 0x1FFu) : 0u;
    const bool dead = clash != 0 || (e0 && cand0 == 0) || (e1 && cand1 == 0);
    if (wany(dead)) return PROP_DEAD;
    if (!wany(e0 || e1)) return PROP_SOLVED;

    // ---- naked singles
    const bool n0 = e0 && (cand0 & (cand0 - 1)) == 0;
    const bool n1 = e1 && (cand1 & (cand1 - 1)) == 0;
    if (wany(n0 || n1)) {
        s.v0 = n0 ? __builtin_ctz(cand0) + 1 : s.v0;
        s.lv0 = n0 ? depth : s.lv0;
        s.v1 = n1 ? __builtin_ctz(cand1) + 1 : s.v1;
        s.lv1 = n1 ? depth : s.lv1;
        s.nw0 = n0;
        s.nw1 = n1;
        placed = true;
        return PROP_OPEN;
    }

    // ---- phase B: hidden singles and digits with no place in a unit.
    // Cells publish their candidates; lanes 0..26 each gather one unit's nine
    // cells (conflict-light plain reads) and fold "seen once / seen twice".
    // A unit whose givens clash publishes T = all digits, which switches the
    // hidden-single rule off there without any test on the cell side.
    W.C[lane] = cand0;
    W.C[64 + lane] = cand1;  // lanes >= 17 land in padding
    wave_lds_order();
    bool udead = false;
    if (lane < 27) {
        uint32_t once = 0, twice = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t x = W.C[s.ub + k * s.us1 + (k / 3) * s.us2];
            twice |= once & x;
            once |= x;
        }
        const bool ok = !((bad >> lane) & 1u);
        W.T[lane] = ok ? twice : 0x1FFu;
        udead = ok && (once | W.M[lane]) != 0x1FFu;
    }
    wave_lds_order();
    const uint32_t h0 = cand0 & ~(W.T[s.r0] & W.T[9 + s.c0] & W.T[18 + s.b0]);
    const uint32_t h1 = cand1 & ~(W.T[s.r1] & W.T[9 + s.c1] & W.T[18 + s.b1]);
    const bool dead2 = udead || (h0 & (h0 - 1)) != 0 || (h1 & (h1 - 1)) != 0;
    if (wany(dead2)) return PROP_DEAD;
    if (wany(h0 != 0 || h1 != 0)) {
        s.v0 = h0 ? __builtin_ctz(h0) + 1 : s.v0;
        s.lv0 = h0 ? depth : s.lv0;
        s.v1 = h1 ? __builtin_ctz(h1) + 1 : s.v1;
        s.lv1 = h1 ? depth : s.lv1;
        s.nw0 = h0 != 0;
        s.nw1 = h1 != 0;
        placed = true;
    }
    return PROP_OPEN;
}

__device__ __forceinline__ int propagate(WaveLds &W, int lane, Cells &s, uint32_t gmask, uint32_t bad,
                                         uint32_t depth, bool &rebuild, uint32_t &cand0, uint32_t &cand1,
                                         uint32_t &sweeps)
{
    for (;;) {
        bool placed;
        int st = sweep(W, lane, s, gmask, bad, depth, rebuild, cand0, cand1, placed);
        sweeps++;
        if (st != PROP_OPEN || !placed) return st;
    }
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

// the walk's branch cell and its candidates; requires a fixpoint state
__device__ __forceinline__ void first_empty(const Cells &s, uint32_t cand0, uint32_t cand1, int order, int &cell,
                                            uint32_t &cand)
{
    const uint64_t eb0 = __ballot(s.v0 == 0);
    const uint64_t eb1 = __ballot(s.has1 && s.v1 == 0);
    cell = order_cell(eb0, eb1, order);
    cand = cell < 64 ? rdlane(cand0, cell) : rdlane(cand1, cell - 64);
}

__device__ __forceinline__ void place(Cells &s, int lane, int cell, uint32_t dbit, uint32_t level)
{
    const uint32_t v = __builtin_ctz(dbit) + 1;
    if (cell < 64) {
        if (lane == cell) { s.v0 = v; s.lv0 = level; s.nw0 = true; }
    } else {
        if (lane == cell - 64) { s.v1 = v; s.lv1 = level; s.nw1 = true; }
    }
}

__device__ __forceinline__ void store_board(uint8_t *__restrict__ dst, int lane, const Cells &s, bool original)
{
    uint32_t a = original ? (s.g0 ? s.v0 : 0u) : s.v0;
    uint32_t b = original ? (s.g1 ? s.v1 : 0u) : s.v1;
    dst[lane] = (uint8_t)a;
    if (s.has1) dst[64 + lane] = (uint8_t)b;
}

// Full search of one board.  Returns SDK_SOLVED / SDK_UNSOLVABLE /
// SDK_CANCELLED; on SOLVED the cells hold the walk's first solution.
__device__ __forceinline__ int search(WaveLds &W, int lane, Cells &s, int64_t idx, int order,
                                      const int64_t *best, uint32_t &guesses, uint32_t &sweeps)
{
    uint32_t bad;
    const uint32_t gmask = build_given_masks(W, lane, s, bad);
    bool rebuild = false;  // W.M already holds exactly the givens
    uint32_t depth = 0;
    uint32_t stk0 = 0, stk1 = 0;  // DFS stack: level k lives in lane k&63 of stk(k>>6)
    uint32_t cand0, cand1;
    for (;;) {
        int st = propagate(W, lane, s, gmask, bad, depth, rebuild, cand0, cand1, sweeps);
        if (st == PROP_SOLVED) return SDK_SOLVED;
        if (st == PROP_OPEN) {
            // branch on the walk's next cell, smallest digit first
            int cell;
            uint32_t cand;
            first_empty(s, cand0, cand1, order, cell, cand);
            if (cand == 0) return SDK_FAULT;  // unreachable: a fixpoint has no empty cell without candidates
            const uint32_t d = lowbit(cand);
            const uint32_t entry = ((uint32_t)cell << 9) | (cand ^ d);
            if (depth < 64) { if (lane == (int)depth) stk0 = entry; }
            else if (lane == (int)depth - 64) stk1 = entry;
            depth++;
            place(s, lane, cell, d, depth);
            guesses++;
            if (best && (guesses & 63u) == 0) {
                const int64_t b = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__builtin_amdgcn_readfirstlane((int)(b < idx))) return SDK_CANCELLED;
            }
            continue;
        }
        // dead: backtrack to the deepest level with an untried digit
        rebuild = true;
        s.nw0 = false;
        s.nw1 = false;
        for (;;) {
            if (depth == 0) return SDK_UNSOLVABLE;
            const uint32_t top = depth - 1;
            const uint32_t entry = top < 64 ? rdlane(stk0, top) : rdlane(stk1, top - 64);
            if (s.lv0 >= depth) s.v0 = 0;  // undo everything filled at this depth
            if (s.lv1 >= depth) s.v1 = 0;
            depth = top;
            const uint32_t rem = entry & 0x1FFu;
            if (rem == 0) continue;
            const int cell = (int)(entry >> 9);
            const uint32_t d = lowbit(rem);
            const uint32_t ne = ((uint32_t)cell << 9) | (rem ^ d);
            if (depth < 64) { if (lane == (int)depth) stk0 = ne; }
            else if (lane == (int)depth - 64) stk1 = ne;
            depth++;
            place(s, lane, cell, d, depth);
            guesses++;
            break;
        }
    }
}

// ------------------------------------------------------------- solve kernel
// re-arm the per-call workspace words on the stream (graph-capturable)
__global__ void arm_kernel(unsigned long long *ws)
{
    if (threadIdx.x == WS_QUEUE) ws[WS_QUEUE] = 0ull;
    if (threadIdx.x == WS_BEST) ws[WS_BEST] = (unsigned long long)INT64_MAX;
}

#ifndef SDK_SOLVE_WAVES_PER_EU
#define SDK_SOLVE_WAVES_PER_EU 1
#endif
__global__ __launch_bounds__(BLOCK_THREADS, SDK_SOLVE_WAVES_PER_EU) void solve_kernel(
    const uint8_t *__restrict__ puzzles, uint8_t *__restrict__ sols, int32_t *__restrict__ status,
    int64_t n, unsigned long long *__restrict__ ws, int64_t chunk, int ordered, int order)
{
    __shared__ WaveLds lds[WAVES_PER_BLOCK];
    const int lane = threadIdx.x & 63;
    WaveLds &W = lds[threadIdx.x >> 6];
    const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    const int64_t gw = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    const int64_t *best = ordered ? (const int64_t *)&ws[WS_BEST] : nullptr;

    uint32_t fin = 0, solved = 0, guesses = 0, sweeps = 0;
    // first chunk statically, the rest from the queue
    int64_t base = gw * chunk;
    const int64_t static_end = nwaves * chunk;
    while (base < n) {
        const int64_t end = base + chunk < n ? base + chunk : n;
        for (int64_t p = base; p < end; ++p) {
            Cells s;
            init_lane(s, lane);
            const uint8_t *src = puzzles + p * 81;
            uint8_t *dst = sols + p * 81;
            int st;
            if (!load_board(src, lane, s)) {
                st = SDK_INVALID;
                store_board(dst, lane, s, false);  // raw input back
            } else if (best && __builtin_amdgcn_readfirstlane((int)(
                           __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p))) {
                st = SDK_CANCELLED;
                store_board(dst, lane, s, true);
            } else {
                st = search(W, lane, s, p, order, best, guesses, sweeps);
                store_board(dst, lane, s, st != SDK_SOLVED);
                if (st == SDK_SOLVED) {
                    solved++;
                    if (best && lane == 0)
                        __hip_atomic_fetch_min((int64_t *)&ws[WS_BEST], p, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (lane == 0) status[p] = st;
            fin++;
        }
        unsigned long long t = 0;
        if (lane == 0) t = atomicAdd(&ws[WS_QUEUE], 1ull);
        t = __shfl(t, 0);
        base = static_end + (int64_t)t * chunk;
    }
    if (lane == 0 && fin) {
        atomicAdd(&ws[WS_FINISHED], (unsigned long long)fin);
        atomicAdd(&ws[WS_SOLVED], (unsigned long long)solved);
        atomicAdd(&ws[WS_GUESSES], (unsigned long long)guesses);
        atomicAdd(&ws[WS_SWEEPS], (unsigned long long)sweeps);
    }
}

// ====================================================== v4: packed cell pairs
#include "packed_solver.h"

// ====================================================== v3: two boards / wave
// Half h = lane >> 5 of the wavefront owns one board; lane q = lane & 31 owns
// cells q, 32+q and (q < 17) 64+q, and lanes q < 27 are that board's unit
// lanes (row / column / box q) for the hidden-single gather.  Every VALU,
// SALU and LDS instruction -- and every LDS round trip -- then serves two
// boards, and 81 of the 96 cell slots are live (v2: 81 of 128).  Each half
// keeps its own LDS slice, trail, stack (three VGPRs, level k at lane
// 32h + (k & 31) of register k >> 5) and board cursor; per-half decisions
// come from the two 32-bit halves of each ballot.  Same walk, same
// propagation rules as v2, so the same first completion.

struct __attribute__((aligned(16))) HalfLds {
    uint32_t M[28];  // unit masks of filled cells
    uint32_t T[28];  // per unit: digits that are candidates of >= 2 empty cells
    uint32_t C[96];  // per cell slot: candidates published for the gather
    uint32_t bad;    // units whose givens clash
    uint32_t pad[3];
};

enum { H_STUCK = 0, H_DEAD = 1, H_SOLVED = 2, H_PLACED = 3, H_NEEDB = 4, H_IDLE = 5 };

struct Lane3 {
    uint32_t v[3], lv[3];
    uint32_t gbits;   // bit s: slot s holds a given
    uint32_t nwbits;  // bit s: slot s placed since the last sweep
    int ur[3], uc[3], ub[3];
    int ga[9];        // unit lanes: cells gathered for unit q
    int q, h;
    bool has2;        // slot 2 exists (q < 17)
};

struct HalfState {
    uint32_t p, end;  // current board, end of the current chunk (n < 2^32 - chunk, checked on the host)
    int act;          // a board is loaded
    int rebuild;
    uint32_t depth, bad;
    uint32_t nguess;  // guesses on the current board (cancellation polling)
};

__device__ __forceinline__ void init_lane3(Lane3 &s, int lane)
{
    s.h = lane >> 5;
    s.q = lane & 31;
    s.has2 = s.q < 17;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int cell = (k < 2 || s.has2) ? 32 * k + s.q : 80;
        int r, c, b;
        cell_units(cell, r, c, b);
        s.ur[k] = r;
        s.uc[k] = 9 + c;
        s.ub[k] = 18 + b;
    }
    const int u = s.q < 27 ? s.q : 0;
    int base, s1, s2;
    if (u < 9) { base = 9 * u; s1 = 1; s2 = 0; }
    else if (u < 18) { base = u - 9; s1 = 9; s2 = 0; }
    else { const int b = u - 18; base = (b / 3) * 27 + (b % 3) * 3; s1 = 1; s2 = 6; }
#pragma unroll
    for (int k = 0; k < 9; ++k) s.ga[k] = base + k * s1 + (k / 3) * s2;
    s.gbits = 0;
    s.nwbits = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) { s.v[k] = 0; s.lv[k] = 0; }
}

__device__ __forceinline__ bool slot_ok(const Lane3 &s, int k) { return k < 2 || s.has2; }

// Load board `p` into half X.  Returns false if a byte is > 9 (then the
// half's cells hold the raw bytes for the write-back).
template <int X>
__device__ __forceinline__ bool load_half(const uint8_t *__restrict__ src, Lane3 &s)
{
    bool bad = false;
    if (s.h == X) {
        s.gbits = 0;
        s.nwbits = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t x = slot_ok(s, k) ? (uint32_t)src[32 * k + s.q] : 0u;
            s.v[k] = x;
            s.lv[k] = 0;
            if (x) s.gbits |= 1u << k;
            bad |= x > 9;
        }
    }
    const uint64_t b = __ballot(bad);
    return (X == 0 ? (uint32_t)b : (uint32_t)(b >> 32)) == 0;
}

// Givens' unit masks of half X into L.M (and the lanes' gmask), clash mask.
template <int X>
__device__ __forceinline__ uint32_t build_half_masks(HalfLds &L, const Lane3 &s, uint32_t &gmask)
{
    if (s.h == X) {
        if (s.q < 28) L.M[s.q] = 0;
        if (s.q == 0) L.bad = 0;
    }
    wave_lds_sync();
    if (s.h == X) {
        uint32_t d = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if ((s.gbits >> k) & 1u) {
                const uint32_t bit = 1u << (s.v[k] - 1);
                if (atomicOr(&L.M[s.ur[k]], bit) & bit) d |= 1u << s.ur[k];
                if (atomicOr(&L.M[s.uc[k]], bit) & bit) d |= 1u << s.uc[k];
                if (atomicOr(&L.M[s.ub[k]], bit) & bit) d |= 1u << s.ub[k];
            }
        }
        if (d) atomicOr(&L.bad, d);
    }
    wave_lds_sync();
    if (s.h == X && s.q < 27) gmask = L.M[s.q];
    return (uint32_t)__builtin_amdgcn_readlane((int)L.bad, 32 * X);
}

__device__ __forceinline__ int half_status(uint32_t dead, uint32_t empty, uint32_t naked, int act)
{
    return !act ? H_IDLE : dead ? H_DEAD : !empty ? H_SOLVED : naked ? H_PLACED : H_NEEDB;
}

// One sweep of both halves.  lane-level inputs: gmask, the lane's half's
// bad units, depth and rebuild flag; outputs per-half statuses.
__device__ __forceinline__ void sweep3(HalfLds &L, Lane3 &s, uint32_t gmask, int act0, int act1, int rb0, int rb1,
                                       uint32_t bad0, uint32_t bad1, uint32_t depth0, uint32_t depth1,
                                       uint32_t (&cand)[3], int &st0, int &st1)
{
    // per-lane views of the two halves' uniform state (values, never a
    // pointer select: that would push the state to scratch)
    const bool mine0 = s.h == 0;
    const bool act = mine0 ? act0 != 0 : act1 != 0;
    const bool rb = mine0 ? rb0 != 0 : rb1 != 0;
    const uint32_t bad = mine0 ? bad0 : bad1;
    const uint32_t depth = mine0 ? depth0 : depth1;
    const bool any_rb = rb0 || rb1;

    // ---- phase A: unit masks up to date, clash detection
    if (any_rb && rb && s.q < 27) L.M[s.q] = gmask;
    uint32_t f = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool filled_nongiven = slot_ok(s, k) && s.v[k] != 0 && !((s.gbits >> k) & 1u);
        const bool fk = act && (rb ? filled_nongiven : ((s.nwbits >> k) & 1u));
        f |= (uint32_t)fk << k;
    }
    s.nwbits = 0;
    uint32_t clash = 0;
    if (any_rb || __any(f != 0)) {
        wave_lds_sync();
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if ((f >> k) & 1u) {
                const uint32_t bit = 1u << (s.v[k] - 1);
                clash |= (atomicOr(&L.M[s.ur[k]], bit) | atomicOr(&L.M[s.uc[k]], bit) |
                          atomicOr(&L.M[s.ub[k]], bit)) & bit;
            }
        }
    }
    wave_lds_sync();
    bool dead = clash != 0, anyempty = false, naked = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool e = act && slot_ok(s, k) && s.v[k] == 0;
        cand[k] = e ? (~(L.M[s.ur[k]] | L.M[s.uc[k]] | L.M[s.ub[k]]) & 0x1FFu) : 0u;
        dead |= e && cand[k] == 0;
        anyempty |= e;
        naked |= e && (cand[k] & (cand[k] - 1)) == 0;
    }
    const uint64_t bd = __ballot(dead), be = __ballot(anyempty), bn = __ballot(naked);
    st0 = half_status((uint32_t)bd, (uint32_t)be, (uint32_t)bn, act0);
    st1 = half_status((uint32_t)(bd >> 32), (uint32_t)(be >> 32), (uint32_t)(bn >> 32), act1);
    const int mst = mine0 ? st0 : st1;
    if (mst == H_PLACED) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (cand[k] != 0 && (cand[k] & (cand[k] - 1)) == 0) {
                s.v[k] = __builtin_ctz(cand[k]) + 1;
                s.lv[k] = depth;
                s.nwbits |= 1u << k;
            }
        }
    }
    if (st0 != H_NEEDB && st1 != H_NEEDB) return;

    // ---- phase B: hidden singles (halves in H_NEEDB only)
    const bool needb = mst == H_NEEDB;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (slot_ok(s, k)) L.C[32 * k + s.q] = cand[k];
    wave_lds_sync();
    bool udead = false;
    if (needb && s.q < 27) {
        uint32_t once = 0, twice = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t x = L.C[s.ga[k]];
            twice |= once & x;
            once |= x;
        }
        L.T[s.q] = twice;
        if (!((bad >> s.q) & 1u)) udead = (once | L.M[s.q]) != 0x1FFu;
    }
    wave_lds_sync();
    bool dead2 = udead, hid = false;
    uint32_t hm[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        uint32_t x = 0;
        if (needb && cand[k] != 0) {
            if (!((bad >> s.ur[k]) & 1u)) x |= cand[k] & ~L.T[s.ur[k]];
            if (!((bad >> s.uc[k]) & 1u)) x |= cand[k] & ~L.T[s.uc[k]];
            if (!((bad >> s.ub[k]) & 1u)) x |= cand[k] & ~L.T[s.ub[k]];
        }
        hm[k] = x;
        dead2 |= (x & (x - 1)) != 0;
        hid |= x != 0;
    }
    const uint64_t bd2 = __ballot(dead2), bh = __ballot(hid);
    if (st0 == H_NEEDB) st0 = (uint32_t)bd2 ? H_DEAD : (uint32_t)bh ? H_PLACED : H_STUCK;
    if (st1 == H_NEEDB) st1 = (uint32_t)(bd2 >> 32) ? H_DEAD : (uint32_t)(bh >> 32) ? H_PLACED : H_STUCK;
    if (needb && (mine0 ? st0 : st1) == H_PLACED) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (hm[k]) {
                s.v[k] = __builtin_ctz(hm[k]) + 1;
                s.lv[k] = depth;
                s.nwbits |= 1u << k;
            }
        }
    }
}

template <int X>
__device__ __forceinline__ uint32_t rd_half(uint32_t v, int q) { return rdlane(v, 32 * X + q); }

// place digit bit d at `cell` of half X with fill level `level`
template <int X>
__device__ __forceinline__ void place3(Lane3 &s, int cell, uint32_t dbit, uint32_t level)
{
    const bool hit = s.h == X && s.q == (cell & 31);
    const int k = cell >> 5;
    const uint32_t v = __builtin_ctz(dbit) + 1;
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // static slot index: keeps the cells in VGPRs
        if (hit && k == j) {
            s.v[j] = v;
            s.lv[j] = level;
            s.nwbits |= 1u << j;
        }
    }
}

// Three named VGPRs, never an array: a select between array elements turns
// into a dynamic index and pushes the array to scratch.
struct Reg3 {
    uint32_t a, b, c;
};

template <int X>
__device__ __forceinline__ void stk_write(Reg3 &stk, const Lane3 &s, uint32_t level, uint32_t val)
{
    const bool me = s.h == X && s.q == (int)(level & 31);
    if (level < 32) { if (me) stk.a = val; }
    else if (level < 64) { if (me) stk.b = val; }
    else { if (me) stk.c = val; }
}

template <int X>
__device__ __forceinline__ uint32_t reg3_read(const Reg3 &r, uint32_t idx)
{
    if (idx < 32) return rd_half<X>(r.a, (int)idx);
    if (idx < 64) return rd_half<X>(r.b, (int)(idx - 32));
    return rd_half<X>(r.c, (int)(idx - 64));
}

template <int X>
__device__ __forceinline__ uint32_t stk_read(const Reg3 &stk, uint32_t level) { return reg3_read<X>(stk, level); }

// Branch half X on the walk's next cell (state is a fixpoint).
template <int X>
__device__ __forceinline__ bool guess3(Lane3 &s, Reg3 &stk, HalfState &H, const Reg3 &cand, int order)
{
    const bool me = s.h == X;
    const uint64_t e0 = __ballot(me && s.v[0] == 0), e1 = __ballot(me && s.v[1] == 0),
                   e2 = __ballot(me && s.has2 && s.v[2] == 0);
    const uint32_t E0 = X ? (uint32_t)(e0 >> 32) : (uint32_t)e0;
    const uint32_t E1 = X ? (uint32_t)(e1 >> 32) : (uint32_t)e1;
    const uint32_t E2 = X ? (uint32_t)(e2 >> 32) : (uint32_t)e2;
    const int cell = order_cell((uint64_t)E0 | ((uint64_t)E1 << 32), (uint64_t)E2, order);
    const uint32_t c = reg3_read<X>(cand, (uint32_t)cell);
    if (c == 0) return false;  // unreachable at a fixpoint
    const uint32_t d = lowbit(c);
    stk_write<X>(stk, s, H.depth, ((uint32_t)cell << 9) | (c ^ d));
    H.depth++;
    place3<X>(s, cell, d, H.depth);
    H.nguess++;
    return true;
}

// Backtrack half X; returns false when the tree is exhausted (unsolvable).
template <int X>
__device__ __forceinline__ bool backtrack3(Lane3 &s, Reg3 &stk, HalfState &H)
{
    H.rebuild = 1;
    if (s.h == X) s.nwbits = 0;
    for (;;) {
        if (H.depth == 0) return false;
        const uint32_t top = H.depth - 1;
        const uint32_t entry = stk_read<X>(stk, top);
        if (s.h == X) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (s.lv[k] >= H.depth) s.v[k] = 0;
        }
        H.depth = top;
        const uint32_t rem = entry & 0x1FFu;
        if (rem == 0) continue;
        const int cell = (int)(entry >> 9);
        const uint32_t d = lowbit(rem);
        stk_write<X>(stk, s, H.depth, ((uint32_t)cell << 9) | (rem ^ d));
        H.depth++;
        place3<X>(s, cell, d, H.depth);
        H.nguess++;
        return true;
    }
}

template <int X>
__device__ __forceinline__ void store_half(uint8_t *__restrict__ dst, const Lane3 &s, bool original)
{
    if (s.h == X) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (!slot_ok(s, k)) continue;
            const uint32_t x = original ? (((s.gbits >> k) & 1u) ? s.v[k] : 0u) : s.v[k];
            dst[32 * k + s.q] = (uint8_t)x;
        }
    }
}

struct Solve3Ctx {
    const uint8_t *puzzles;
    uint8_t *sols;
    int32_t *status;
    int64_t n, chunk, static_end;
    unsigned long long *ws;
    const int64_t *best;
    int order;
    uint32_t fin, solved, guesses, sweeps;
};

// Advance half X to its next board (chunk cursor, then the global queue) and
// load it; sets H.act = 0 when the queue is drained.
template <int X>
__device__ __forceinline__ void next_board(HalfLds &L, Lane3 &s, HalfState &H, uint32_t &gmask, Solve3Ctx &c)
{
    int act = 0;
    for (;;) {
        H.p++;
        if (H.p >= H.end) {
            uint32_t t = 0;
            if (s.h == X && s.q == 0) t = atomicAdd((unsigned int *)&c.ws[WS_QUEUE], 1u);
            const uint64_t base = c.static_end + (uint64_t)rd_half<X>(t, 0) * c.chunk;
            const uint64_t end = base + c.chunk < c.n ? base + c.chunk : c.n;
            H.p = base < c.n ? (uint32_t)base : (uint32_t)c.n;
            H.end = (uint32_t)end;
        }
        if (H.p >= c.n) break;
        const uint8_t *src = c.puzzles + (uint64_t)H.p * 81;
        uint8_t *dst = c.sols + (uint64_t)H.p * 81;
        if (!load_half<X>(src, s)) {  // byte > 9: raw input back
            store_half<X>(dst, s, false);
            if (s.h == X && s.q == 0) c.status[H.p] = SDK_INVALID;
            c.fin++;
            continue;
        }
        if (c.best && __hip_atomic_load(c.best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (int64_t)H.p) {
            store_half<X>(dst, s, true);
            if (s.h == X && s.q == 0) c.status[H.p] = SDK_CANCELLED;
            c.fin++;
            continue;
        }
        H.bad = build_half_masks<X>(L, s, gmask);
        act = 1;
        break;
    }
    // one assignment point per field: stores of equal constants to different
    // fields on two paths get merged behind a pointer phi, which pins the
    // state to scratch
    H.act = act;
    H.rebuild = 0;
    H.depth = 0;
    H.nguess = 0;
}

template <int X>
__device__ __forceinline__ void finish_board(HalfLds &L, Lane3 &s, HalfState &H, uint32_t &gmask, Solve3Ctx &c,
                                             int st)
{
    uint8_t *dst = c.sols + (uint64_t)H.p * 81;
    store_half<X>(dst, s, st != SDK_SOLVED);
    if (s.h == X && s.q == 0) c.status[H.p] = st;
    if (st == SDK_SOLVED) {
        c.solved++;
        if (c.best && s.h == X && s.q == 0)
            __hip_atomic_fetch_min((int64_t *)&c.ws[WS_BEST], (int64_t)H.p, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    c.fin++;
    c.guesses += H.nguess;
    next_board<X>(L, s, H, gmask, c);
}

template <int X>
__device__ __forceinline__ void step_half(HalfLds &L, Lane3 &s, Reg3 &stk, HalfState &H, uint32_t &gmask,
                                          const Reg3 &cand, Solve3Ctx &c, int st)
{
    if (st == H_SOLVED) {
        finish_board<X>(L, s, H, gmask, c, SDK_SOLVED);
    } else if (st == H_DEAD) {
        if (!backtrack3<X>(s, stk, H)) finish_board<X>(L, s, H, gmask, c, SDK_UNSOLVABLE);
    } else if (st == H_STUCK) {
        if (!guess3<X>(s, stk, H, cand, c.order)) {
            finish_board<X>(L, s, H, gmask, c, SDK_FAULT);
        } else if (c.best && (H.nguess & 63u) == 0 &&
                   __hip_atomic_load(c.best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (int64_t)H.p) {
            finish_board<X>(L, s, H, gmask, c, SDK_CANCELLED);
        }
    }
}

__global__ __launch_bounds__(BLOCK_THREADS) void solve2_kernel(
    const uint8_t *__restrict__ puzzles, uint8_t *__restrict__ sols, int32_t *__restrict__ status,
    int64_t n, unsigned long long *__restrict__ ws, int64_t chunk, int ordered, int order)
{
    __shared__ HalfLds lds[WAVES_PER_BLOCK][2];
    const int lane = threadIdx.x & 63;
    Lane3 s;
    init_lane3(s, lane);
    HalfLds &L = lds[threadIdx.x >> 6][s.h];
    const int64_t slots = (int64_t)gridDim.x * WAVES_PER_BLOCK * 2;
    const int64_t gw = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);

    Solve3Ctx c;
    c.puzzles = puzzles; c.sols = sols; c.status = status; c.n = n; c.chunk = chunk;
    c.static_end = slots * chunk; c.ws = ws; c.order = order;
    c.best = ordered ? (const int64_t *)&ws[WS_BEST] : nullptr;
    c.fin = c.solved = c.guesses = c.sweeps = 0;

    HalfState H0, H1;
    uint32_t gmask = 0;
    Reg3 stk = {0u, 0u, 0u};
    // static first chunk of each half (the cursor starts one before it)
    {
        const int64_t b0 = (2 * gw) * chunk, b1 = (2 * gw + 1) * chunk;
        H0.p = (uint32_t)(b0 < n ? b0 : n) - 1u;  // the cursor starts one before its chunk
        H1.p = (uint32_t)(b1 < n ? b1 : n) - 1u;
        H0.end = (uint32_t)(b0 + chunk < n ? b0 + chunk : n);
        H1.end = (uint32_t)(b1 + chunk < n ? b1 + chunk : n);
    }
    H0.act = H1.act = 0;
    next_board<0>(L, s, H0, gmask, c);
    next_board<1>(L, s, H1, gmask, c);

    uint32_t cand[3];
    while (H0.act || H1.act) {
        int st0, st1;
        sweep3(L, s, gmask, H0.act, H1.act, H0.rebuild, H1.rebuild, H0.bad, H1.bad, H0.depth, H1.depth, cand,
               st0, st1);
        const Reg3 cr = {cand[0], cand[1], cand[2]};
        c.sweeps += (uint32_t)H0.act + (uint32_t)H1.act;
        H0.rebuild = 0;
        H1.rebuild = 0;
        step_half<0>(L, s, stk, H0, gmask, cr, c, st0);
        step_half<1>(L, s, stk, H1, gmask, cr, c, st1);
    }
    if (lane == 0 && c.fin) {
        atomicAdd(&ws[WS_FINISHED], (unsigned long long)c.fin);
        atomicAdd(&ws[WS_SOLVED], (unsigned long long)c.solved);
        atomicAdd(&ws[WS_GUESSES], (unsigned long long)c.guesses);
        atomicAdd(&ws[WS_SWEEPS], (unsigned long long)c.sweeps);
    }
}

// ====================================================== lane-per-board kernel
// Each LANE owns one board (lane_solver.h: unit masks in registers, fully
// unrolled Gauss-Seidel passes, DFS stack in per-lane scratch).  The loop is
// a per-lane state machine -- every iteration runs one naked pass, a hidden
// pass for the lanes whose naked pass stalled, then each lane's own guess /
// backtrack / finish -- and a lane that finishes pulls its next board from
// the queue in the same iteration, so lanes of a wave never wait for a
// slower board.

struct ScratchStack {
    uint32_t w[lane::MAX_DEPTH * lane::STACK_WORDS];
    __device__ __forceinline__ void put(uint32_t d, int k, uint32_t v) { w[d * lane::STACK_WORDS + k] = v; }
    __device__ __forceinline__ uint32_t get(uint32_t d, int k) const { return w[d * lane::STACK_WORDS + k]; }
};

__global__ __launch_bounds__(BLOCK_THREADS) void lane_kernel(
    const uint8_t *__restrict__ puzzles, uint8_t *__restrict__ sols, int32_t *__restrict__ status,
    int64_t n, unsigned long long *__restrict__ ws, int ordered, int order)
{
    ScratchStack stk;
    lane::Board b;
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // first board: static
    const int64_t *best = ordered ? (const int64_t *)&ws[WS_BEST] : nullptr;
    const int node_order = order == SDK_ORDER_NODE;
    uint32_t depth = 0, nguess = 0;
    uint32_t fin = 0, solved = 0, guesses = 0, passes = 0;
    bool have = false;

    for (;;) {
        // ---- refill: lanes without a board take the next one
        while (!have) {
            if (p >= n) break;
            const uint8_t *src = puzzles + p * 81;
            const bool valid = lane::load_dw(b, src);
            if (!valid) {
                for (int i = 0; i < 81; ++i) sols[p * 81 + i] = src[i];
                status[p] = SDK_INVALID;
                fin++;
            } else if (best && __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p) {
                for (int i = 0; i < 81; ++i) sols[p * 81 + i] = src[i];
                status[p] = SDK_CANCELLED;
                fin++;
            } else {
                depth = 0;
                nguess = 0;
                have = true;
                break;
            }
            p = nthreads + (int64_t)atomicAdd(&ws[WS_QUEUE], 1ull);
        }
        if (!__any(have)) break;
        if (!have) continue;

        // ---- one propagation step
        uint32_t dead = 0, placed = 0;
        lane::NakedPass<0>::run(b, dead, placed);
        passes++;
        const bool empty = (b.E[0] | b.E[1] | b.E[2]) != 0;
        if (!dead && !placed && empty) {
            lane::HiddenPass<0>::run(b, dead, placed);
            passes++;
        }
        int done = -1;  // board status when it finishes in this step
        if (!dead) {
            if (!(b.E[0] | b.E[1] | b.E[2])) {
                done = SDK_SOLVED;
            } else if (!placed) {
                // branch on the walk's next cell, smallest digit first
                const int cell = lane::order_cell((uint64_t)b.E[0] | ((uint64_t)b.E[1] << 32),
                                                  (uint64_t)b.E[2], node_order);
                const uint32_t cand = lane::cand_at(b, cell);
                const uint32_t d = cand & (0u - cand);
#pragma unroll
                for (int w = 0; w < 11; ++w) stk.put(depth, w, b.V[w]);
#pragma unroll
                for (int w = 0; w < 3; ++w) stk.put(depth, 11 + w, b.E[w]);
                stk.put(depth, lane::STACK_ENTRY, ((uint32_t)cell << 9) | (cand ^ d));
                depth++;
                nguess++;
                lane::place_at(b, cell, d);
                if (best && (nguess & 63u) == 0 &&
                    __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p)
                    done = SDK_CANCELLED;
            }
        } else {
            // back to the deepest level with an untried digit
            done = SDK_UNSOLVABLE;
            while (depth > 0) {
                depth--;
                const uint32_t entry = stk.get(depth, lane::STACK_ENTRY);
                const uint32_t rem = entry & 0x1FFu;
                if (!rem) continue;
                const int cell = (int)(entry >> 9);
                const uint32_t d = rem & (0u - rem);
#pragma unroll
                for (int w = 0; w < 11; ++w) b.V[w] = stk.get(depth, w);
#pragma unroll
                for (int w = 0; w < 3; ++w) b.E[w] = stk.get(depth, 11 + w);
                lane::rebuild_units(b);
                stk.put(depth, lane::STACK_ENTRY, ((uint32_t)cell << 9) | (rem ^ d));
                depth++;
                nguess++;
                lane::place_at(b, cell, d);
                done = -1;
                break;
            }
        }
        if (done >= -2 && done != -1) {
            uint8_t *dst = sols + p * 81;
            if (done == SDK_SOLVED) {
                lane::store(b, dst);
                solved++;
                if (best)
                    __hip_atomic_fetch_min((int64_t *)&ws[WS_BEST], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const uint8_t *src = puzzles + p * 81;
                for (int i = 0; i < 81; ++i) dst[i] = src[i];
            }
            status[p] = done;
            fin++;
            guesses += nguess;
            have = false;
            p = nthreads + (int64_t)atomicAdd(&ws[WS_QUEUE], 1ull);
        }
    }
    // per-wave statistics
    unsigned long long f = fin, sv = solved, g = guesses, ps = passes;
    for (int o = 32; o > 0; o >>= 1) {
        f += __shfl_xor(f, o);
        sv += __shfl_xor(sv, o);
        g += __shfl_xor(g, o);
        ps += __shfl_xor(ps, o);
    }
    if ((threadIdx.x & 63) == 0 && f) {
        atomicAdd(&ws[WS_FINISHED], f);
        atomicAdd(&ws[WS_SOLVED], sv);
        atomicAdd(&ws[WS_GUESSES], g);
        atomicAdd(&ws[WS_SWEEPS], ps);
    }
}

// ------------------------------------------------------------ check kernel
// One thread per grid; the block stages its 64 grids (5184 B) through LDS
// with coalesced dword loads.
#define CHECK_GRIDS 64
__global__ __launch_bounds__(64) void check_kernel(const uint8_t *__restrict__ grids, int32_t *__restrict__ ok,
                                                   int64_t n, int mode)
{
    __shared__ __attribute__((aligned(16))) uint8_t tile[CHECK_GRIDS * 81 + 16];
    const int64_t g0 = (int64_t)blockIdx.x * CHECK_GRIDS;
    const int64_t cnt = n - g0 < CHECK_GRIDS ? n - g0 : CHECK_GRIDS;
    const uint8_t *src = grids + g0 * 81;
    const int64_t bytes = cnt * 81;
    for (int64_t i = threadIdx.x; i < bytes; i += 64) tile[i] = src[i];
    __syncthreads();
    if (threadIdx.x >= cnt) return;
    const uint8_t *g = tile + threadIdx.x * 81;
    bool good = true;
    // units: rows, columns, boxes (sudoku.py:125-138 order; result is order-free)
    for (int u = 0; u < 27 && good; ++u) {
        int idx[9];
        if (u < 9) {
            for (int k = 0; k < 9; ++k) idx[k] = u * 9 + k;
        } else if (u < 18) {
            for (int k = 0; k < 9; ++k) idx[k] = k * 9 + (u - 9);
        } else {
            const int br = ((u - 18) / 3) * 3, bc = ((u - 18) % 3) * 3;
            for (int k = 0; k < 9; ++k) idx[k] = (br + k / 3) * 9 + bc + k % 3;
        }
        uint32_t sum = 0;
        for (int k = 0; k < 9; ++k) sum += g[idx[k]];
        if (sum != 45) { good = false; break; }
        if (mode == 0) {
            // len(set(unit)) == 9: all nine bytes pairwise distinct
            bool distinct = true;
            for (int a = 0; a < 9; ++a)
                for (int b = a + 1; b < 9; ++b) distinct &= g[idx[a]] != g[idx[b]];
            good = distinct;
        }
    }
    ok[g0 + threadIdx.x] = good ? 1 : 0;
}

// ----------------------------------------------------- first-candidate kernel
// node.py:76-80 with node.py:42-60's is_valid_move (check() short-circuit).
__global__ __launch_bounds__(256) void first_candidate_kernel(const uint8_t *__restrict__ grids,
                                                              const int32_t *__restrict__ cells,
                                                              int32_t *__restrict__ num, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *g = grids + i * 81;
    const int cell = cells[i];
    if (cell < 0 || cell >= 81) { num[i] = -1; return; }
    // node.py:82-116 sums check
    bool sums = true;
    for (int u = 0; u < 27 && sums; ++u) {
        uint32_t sum = 0;
        for (int k = 0; k < 9; ++k) {
            int idx = u < 9 ? u * 9 + k
                    : u < 18 ? k * 9 + (u - 9)
                             : (((u - 18) / 3) * 3 + k / 3) * 9 + ((u - 18) % 3) * 3 + k % 3;
            sum += g[idx];
        }
        sums = sum == 45;
    }
    if (sums) { num[i] = 1; return; }
    const int r = cell / 9, c = cell % 9, br = (r / 3) * 3, bc = (c / 3) * 3;
    uint32_t used = 0;
    for (int k = 0; k < 9; ++k) {
        uint32_t a = g[r * 9 + k], b = g[k * 9 + c], x = g[(br + k / 3) * 9 + bc + k % 3];
        if (a >= 1 && a <= 9) used |= 1u << (a - 1);
        if (b >= 1 && b <= 9) used |= 1u << (b - 1);
        if (x >= 1 && x <= 9) used |= 1u << (x - 1);
    }
    const uint32_t free_ = ~used & 0x1FFu;
    num[i] = free_ ? (int32_t)__builtin_ctz(free_) + 1 : 0;
}

// ------------------------------------------------------ frontier expansion
// pass 1: propagate each node (one wave each), keep the propagated grid and
// the number of children it will produce.
__global__ __launch_bounds__(BLOCK_THREADS) void expand_count_kernel(const uint8_t *__restrict__ nodes, int64_t n,
                                                                     uint8_t *__restrict__ tmp,
                                                                     int64_t *__restrict__ counts, int order)
{
    __shared__ WaveLds lds[WAVES_PER_BLOCK];
    const int lane = threadIdx.x & 63;
    WaveLds &W = lds[threadIdx.x >> 6];
    const int64_t p = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    if (p >= n) return;
    Cells s;
    init_lane(s, lane);
    uint8_t *dst = tmp + p * 81;
    int64_t cnt = 0;
    if (load_board(nodes + p * 81, lane, s)) {
        uint32_t bad;
        const uint32_t gmask = build_given_masks(W, lane, s, bad);
        uint32_t cand0, cand1, sweeps = 0;
        bool rebuild = false;
        const int st = propagate(W, lane, s, gmask, bad, 0, rebuild, cand0, cand1, sweeps);
        if (st == PROP_SOLVED) {
            cnt = 1;
        } else if (st == PROP_OPEN) {
            int cell;
            uint32_t cand;
            first_empty(s, cand0, cand1, order, cell, cand);
            cnt = __builtin_popcount(cand);
        }
    }
    store_board(dst, lane, s, false);
    if (lane == 0) counts[p] = cnt;
}

// exclusive scan of counts -> offsets (n+1 entries), one block
__global__ __launch_bounds__(1024) void scan_kernel(const int64_t *__restrict__ counts, int64_t *__restrict__ offsets,
                                                    int64_t n)
{
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t per = (n + 1023) / 1024;
    const int64_t lo = t * per, hi = lo + per < n ? lo + per : n;
    int64_t s = 0;
    for (int64_t i = lo; i < hi; ++i) s += counts[i];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        int64_t run = 0;
        for (int k = 0; k < 1024; ++k) { int64_t v = part[k]; part[k] = run; run += v; }
        offsets[n] = run;
    }
    __syncthreads();
    int64_t run = part[t];
    for (int64_t i = lo; i < hi; ++i) {  // in place: read the count before overwriting it
        const int64_t c = counts[i];
        offsets[i] = run;
        run += c;
    }
}

// pass 2: write children (one wave per node) in digit order
__global__ __launch_bounds__(BLOCK_THREADS) void expand_write_kernel(const uint8_t *__restrict__ tmp, int64_t n,
                                                                     const int64_t *__restrict__ offsets,
                                                                     uint8_t *__restrict__ children, int64_t cap,
                                                                     int order)
{
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    if (p >= n) return;
    const int64_t off = offsets[p], cnt = offsets[p + 1] - off;
    if (cnt == 0) return;
    const uint8_t *g = tmp + p * 81;
    const uint32_t a = g[lane];
    const uint32_t b = lane < 17 ? g[64 + lane] : 1u;
    // candidates of the first empty cell recomputed from the grid itself
    const uint64_t eb0 = __ballot(a == 0);
    const uint64_t eb1 = __ballot(lane < 17 && b == 0);
    const int cell = (eb0 | eb1) ? order_cell(eb0, eb1, order) : -1;
    uint32_t used = 0;
    if (cell >= 0) {
        const int r = cell / 9, c = cell % 9, br = (r / 3) * 3, bc = (c / 3) * 3;
        // lanes 0..8 read row / column / box members, OR-reduce
        uint32_t m = 0;
        if (lane < 9) {
            uint32_t x = g[r * 9 + lane], y = g[lane * 9 + c], z = g[(br + lane / 3) * 9 + bc + lane % 3];
            if (x) m |= 1u << (x - 1);
            if (y) m |= 1u << (y - 1);
            if (z) m |= 1u << (z - 1);
        }
        for (int sh = 1; sh < 16; sh <<= 1) m |= __shfl_xor(m, sh);
        used = rdlane(m, 0);
    }
    uint32_t cand = cell >= 0 ? (~used & 0x1FFu) : 0u;
    for (int64_t k = 0; k < cnt; ++k) {
        const int64_t o = off + k;
        if (o >= cap) break;
        uint8_t *dst = children + o * 81;
        uint32_t va = a, vb = b;
        if (cell >= 0) {
            const uint32_t d = __builtin_ctz(cand) + 1;
            cand &= cand - 1;
            if (cell < 64) { if (lane == cell) va = d; }
            else if (lane == cell - 64) vb = d;
        }
        dst[lane] = (uint8_t)va;
        if (lane < 17) dst[64 + lane] = (uint8_t)vb;
    }
}

// ==================================================================== C ABI
static thread_local char g_err[512];
static std::mutex g_mu;
static int g_cu_count[64];

static int set_err(const char *what, hipError_t e)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -1;
}

static int cu_count()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_cu_count[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        g_cu_count[dev] = v;
    }
    return g_cu_count[dev];
}

template <typename K>
static int blocks_per_cu(K kernel, std::atomic<int> &cached)
{
    int v = cached.load();
    if (v) return v;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, BLOCK_THREADS, 0) != hipSuccess || nb <= 0)
        nb = 4;
    if (nb > 8) nb = 8;
    cached.store(nb);
    return nb;
}
static std::atomic<int> g_bpc_v2{0}, g_bpc_v3{0}, g_bpc_lane{0}, g_bpc_v4{0}, g_bpc_plane{0};

// lanes of a full plane-kernel grid on the current device, and the bytes of
// their stacks (the workspace holds them after WS_STACK_BYTE)
#ifndef SDK_PLANE_BOARDS_PER_LANE
#define SDK_PLANE_BOARDS_PER_LANE 0
#endif
// SDK_PLANE_BPL overrides the default (A/B runs)
static int64_t plane_boards_per_lane()
{
    static const int64_t v = [] {
        const char *e = getenv("SDK_PLANE_BPL");
        return e && e[0] ? (int64_t)atoll(e) : (int64_t)SDK_PLANE_BOARDS_PER_LANE;
    }();
    return v;
}

static int64_t plane_max_threads()
{
    if (!g_bpc_plane.load()) g_bpc_plane.store(sdk_plane_blocks_per_cu());
    return (int64_t)cu_count() * g_bpc_plane.load() * PLANE_THREADS;
}
static size_t plane_stack_bytes(int64_t threads)
{
    return (size_t)threads * PLANE_MAX_DEPTH * PLANE_STACK_WORDS * sizeof(uint32_t);
}

// kernel variant: 1 = auto (default): 6 for batches of at least
// SDK_PLANE_MIN_BATCH boards, 5 below (a lone board on one lane is slower
// than on a whole wave, and a small batch does not fill the lanes);
// 6 = one board per lane on digit planes (SDK_SOLVE_KERNEL=plane);
// 5 = one board per wave, packed cell pairs (SDK_SOLVE_KERNEL=p);
// 2 = one board per wave, one register set per cell slot (=2);
// 3 = two boards per wave (=3), 4 = one board per lane, nibble cells (=l).
// All give identical results; DESIGN.md has the measurements.
static std::atomic<int> g_variant{0};

static int env_variant()
{
    const char *e = getenv("SDK_SOLVE_KERNEL");
    if (!e || !e[0] || e[0] == 'a') return SDK_KERNEL_AUTO;
    if (e[0] == '3') return SDK_KERNEL_PAIR;
    if (e[0] == 'l') return SDK_KERNEL_LANE;
    if (e[0] == '2' || e[0] == 'w') return SDK_KERNEL_WAVE;
    if (e[0] == 'p' && e[1] != 'l') return SDK_KERNEL_PACKED;
    return SDK_KERNEL_PLANE;
}

static int solve_variant()
{
    int x = g_variant.load();
    if (!x) {
        x = env_variant();
        g_variant.store(x);
    }
    return x;
}

extern "C" {

const char *sdk_last_error(void) { return g_err; }
const char *sdk_version(void)
{
    const int v = solve_variant();
    return v == SDK_KERNEL_AUTO ? "sudoku_hip 0.5 gfx950 auto: lane-per-board digit-planes (large batches), wave-per-board packed-pairs (small) walk-order"
         : v == SDK_KERNEL_PLANE ? "sudoku_hip 0.5 gfx950 lane-per-board digit-planes walk-order"
         : v == SDK_KERNEL_LANE ? "sudoku_hip 0.3 gfx950 lane-per-board walk-order"
         : v == SDK_KERNEL_PACKED ? "sudoku_hip 0.4 gfx950 wave-per-board packed-pairs walk-order"
         : v == SDK_KERNEL_PAIR ? "sudoku_hip 0.3 gfx950 board-pair-per-wave walk-order"
                  : "sudoku_hip 0.3 gfx950 wave-per-board walk-order";
}
int sdk_device_cu_count(void) { return cu_count(); }
int sdk_set_solve_kernel(int kernel)
{
    if (kernel != 0 && kernel != SDK_KERNEL_WAVE && kernel != SDK_KERNEL_PAIR && kernel != SDK_KERNEL_LANE &&
        kernel != SDK_KERNEL_PACKED && kernel != SDK_KERNEL_PLANE && kernel != SDK_KERNEL_AUTO)
        return -1;
    const int prev = solve_variant();
    g_variant.store(kernel ? kernel : env_variant());
    return prev;
}
size_t sdk_workspace_bytes(void) { return WS_STACK_BYTE + plane_stack_bytes(plane_max_threads()); }

int sdk_solve_batch(const uint8_t *d_puzzles, uint8_t *d_solutions, int32_t *d_status, int64_t n,
                    void *d_workspace, int order, int ordered, void *stream)
{
    if (n < 0 || (n > 0 && (!d_puzzles || !d_solutions || !d_status || !d_workspace)) ||
        (order != SDK_ORDER_GEN && order != SDK_ORDER_NODE)) {
        snprintf(g_err, sizeof g_err, "sdk_solve_batch: bad arguments (n=%lld)", (long long)n);
        return -2;
    }
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    unsigned long long *ws = (unsigned long long *)d_workspace;
    hipLaunchKernelGGL(arm_kernel, dim3(1), dim3(64), 0, st, ws);
    hipError_t e;
    int variant = solve_variant();
    if (variant == SDK_KERNEL_AUTO) variant = n >= SDK_PLANE_MIN_BATCH ? SDK_KERNEL_PLANE : SDK_KERNEL_PACKED;
    if (variant == SDK_KERNEL_LANE) {
        // lane per board: one persistent thread per resident lane
        const int64_t max_threads = (int64_t)cu_count() * blocks_per_cu(lane_kernel, g_bpc_lane) * BLOCK_THREADS;
        const int64_t threads = n < max_threads ? n : max_threads;
        const int64_t blocks = (threads + BLOCK_THREADS - 1) / BLOCK_THREADS;
        hipLaunchKernelGGL(lane_kernel, dim3((unsigned)blocks), dim3(BLOCK_THREADS), 0, st, d_puzzles, d_solutions,
                           d_status, n, ws, ordered, order);
    } else if (variant == SDK_KERNEL_PAIR) {
        if (n > (int64_t)0xFFFF0000u) {
            snprintf(g_err, sizeof g_err, "sdk_solve_batch: n=%lld exceeds 2^32-2^16 boards per call", (long long)n);
            return -2;
        }
        // persistent grid of exactly the resident waves, two board slots each
        const int64_t max_slots = (int64_t)cu_count() * blocks_per_cu(solve2_kernel, g_bpc_v3) * WAVES_PER_BLOCK * 2;
        const int64_t slots = n < max_slots ? n : max_slots;
        int64_t chunk = n / (slots * 16);
        if (chunk < 1) chunk = 1;
        if (chunk > 16) chunk = 16;
        const int64_t blocks = (slots + 2 * WAVES_PER_BLOCK - 1) / (2 * WAVES_PER_BLOCK);
        hipLaunchKernelGGL(solve2_kernel, dim3((unsigned)blocks), dim3(BLOCK_THREADS), 0, st, d_puzzles, d_solutions,
                           d_status, n, ws, chunk, ordered, order);
    } else if (variant == SDK_KERNEL_PACKED) {
        const int64_t max_waves = (int64_t)cu_count() * blocks_per_cu(solvep_kernel, g_bpc_v4) * WAVES_PER_BLOCK;
        const int64_t waves = n < max_waves ? n : max_waves;
        int64_t chunk = n / (waves * 16);
        if (chunk < 1) chunk = 1;
        if (chunk > 16) chunk = 16;
        const int64_t blocks = (waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
        hipLaunchKernelGGL(solvep_kernel, dim3((unsigned)blocks), dim3(BLOCK_THREADS), 0, st, d_puzzles, d_solutions,
                           d_status, n, ws, chunk, ordered, order);
    } else if (variant == SDK_KERNEL_PLANE) {
        // lanes: one per board up to a full grid; the stacks sit in the workspace
        const int64_t max_threads = plane_max_threads();
        int64_t threads = n < max_threads ? n : max_threads;
        // at least plane_boards_per_lane() boards per lane: with too few, the
        // drain at the end of the batch (lanes idle while their wave's last
        // boards finish) dominates the launch
        const int64_t bpl = plane_boards_per_lane();
        if (bpl > 1 && threads > n / bpl) {
            threads = n / bpl;
            threads = threads < PLANE_THREADS ? PLANE_THREADS : (threads + PLANE_THREADS - 1) / PLANE_THREADS * PLANE_THREADS;
            if (threads > max_threads) threads = max_threads;
        }
        uint32_t *stack = (uint32_t *)((char *)d_workspace + WS_STACK_BYTE);
        e = sdk_launch_plane(d_puzzles, d_solutions, d_status, n, ws, stack, ordered, order, threads, st);
        if (e != hipSuccess) return set_err("sdk_solve_batch: plane launch", e);
        // the boards it left (clashing givens, deep searches): wave per board
        const int64_t max_waves = (int64_t)cu_count() * blocks_per_cu(solvep_deferred_kernel, g_bpc_v4) * WAVES_PER_BLOCK;
        const int64_t groups = (n + 63) / 64;
        const int64_t waves = groups < max_waves ? groups : max_waves;
        hipLaunchKernelGGL(solvep_deferred_kernel, dim3((unsigned)((waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK)),
                           dim3(BLOCK_THREADS), 0, st, d_puzzles, d_solutions, d_status, n, ws, ordered, order);
    } else {
        const int64_t max_waves = (int64_t)cu_count() * blocks_per_cu(solve_kernel, g_bpc_v2) * WAVES_PER_BLOCK;
        const int64_t waves = n < max_waves ? n : max_waves;
        int64_t chunk = n / (waves * 16);
        if (chunk < 1) chunk = 1;
        if (chunk > 16) chunk = 16;
        const int64_t blocks = (waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
        hipLaunchKernelGGL(solve_kernel, dim3((unsigned)blocks), dim3(BLOCK_THREADS), 0, st, d_puzzles, d_solutions,
                           d_status, n, ws, chunk, ordered, order);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return set_err("sdk_solve_batch: launch", e);
    return 0;
}

int sdk_check_batch(const uint8_t *d_grids, int32_t *d_ok, int64_t n, int mode, void *stream)
{
    if (n < 0 || (n > 0 && (!d_grids || !d_ok)) || (mode != 0 && mode != 1)) {
        snprintf(g_err, sizeof g_err, "sdk_check_batch: bad arguments");
        return -2;
    }
    if (n == 0) return 0;
    const int64_t blocks = (n + CHECK_GRIDS - 1) / CHECK_GRIDS;
    hipLaunchKernelGGL(check_kernel, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream, d_grids, d_ok, n, mode);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("sdk_check_batch: launch", e);
}

int sdk_first_candidate_batch(const uint8_t *d_grids, const int32_t *d_cells, int32_t *d_num, int64_t n,
                              void *stream)
{
    if (n < 0 || (n > 0 && (!d_grids || !d_cells || !d_num))) {
        snprintf(g_err, sizeof g_err, "sdk_first_candidate_batch: bad arguments");
        return -2;
    }
    if (n == 0) return 0;
    hipLaunchKernelGGL(first_candidate_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_grids, d_cells, d_num, n);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("sdk_first_candidate_batch: launch", e);
}

int sdk_expand_frontier(const uint8_t *d_nodes, int64_t n, uint8_t *d_tmp, int64_t *d_offsets,
                        uint8_t *d_children, int64_t cap, int order, void *stream)
{
    if (n < 0 || cap < 0 || (n > 0 && (!d_nodes || !d_tmp || !d_offsets || (cap > 0 && !d_children))) ||
        (order != SDK_ORDER_GEN && order != SDK_ORDER_NODE)) {
        snprintf(g_err, sizeof g_err, "sdk_expand_frontier: bad arguments");
        return -2;
    }
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_offsets, 0, sizeof(int64_t), st);
        return e == hipSuccess ? 0 : set_err("sdk_expand_frontier: memset", e);
    }
    const unsigned blocks = (unsigned)((n + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    // per-node child counts are written into d_offsets[0..n) and scanned in place
    hipLaunchKernelGGL(expand_count_kernel, dim3(blocks), dim3(BLOCK_THREADS), 0, st, d_nodes, n, d_tmp, d_offsets,
                       order);
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, d_offsets, d_offsets, n);
    hipLaunchKernelGGL(expand_write_kernel, dim3(blocks), dim3(BLOCK_THREADS), 0, st, d_tmp, n, d_offsets,
                       d_children, cap, order);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("sdk_expand_frontier: launch", e);
}

int sdk_read_stats(void *d_workspace, int64_t out[6], int reset, void *stream)
{
    if (!d_workspace || !out) {
        snprintf(g_err, sizeof g_err, "sdk_read_stats: bad arguments");
        return -2;
    }
    hipStream_t st = (hipStream_t)stream;
    unsigned long long h[WS_WORDS];
    hipError_t e = hipMemcpyAsync(h, d_workspace, sizeof h, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return set_err("sdk_read_stats", e);
    out[0] = (int64_t)h[WS_FINISHED];
    out[1] = (int64_t)h[WS_SOLVED];
    out[2] = (int64_t)h[WS_GUESSES];
    out[3] = (int64_t)h[WS_SWEEPS];
    out[4] = (int64_t)h[WS_BEST];
    out[5] = (int64_t)h[WS_DEFERRED];
    if (reset) {
        e = hipMemsetAsync((unsigned long long *)d_workspace + WS_FINISHED, 0, 5 * sizeof(unsigned long long), st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return set_err("sdk_read_stats: reset", e);
    }
    return 0;
}

}  // extern "C"
