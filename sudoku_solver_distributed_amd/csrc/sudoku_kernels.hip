// sudoku_kernels.hip -- MI355X (gfx950, CDNA4) Sudoku kernels + C ABI.
//
// Hot path: batch solving of 9x9 boards, bit-identical to the reference's
// backtracking walks.  Both fill one cell at a time with digits 1..9
// ascending; they differ in which empty cell they pick:
//   SDK_ORDER_GEN  gen.py:6-28 solve_sudoku -- its scan (gen.py:11-15) breaks
//                  only the column loop, so it takes the first empty cell of
//                  the LAST row that has one (rows 8..0, columns 0..8);
//   SDK_ORDER_NODE node.py:62-74 solve_sudoku_recursive -- first empty cell
//                  in row-major order, digits tested with is_valid_move
//                  (node.py:42-60, including its sums-45 short-circuit).
// Either way the cell sequence is a fixed order of the empty cells, so the
// walk's first solution is the lexicographically smallest completion in that
// order.  We reach the same board with far fewer nodes by interleaving sound
// propagation (naked singles, hidden singles, conflict detection) with
// branching on the same first-in-order empty cell and the same digit order:
// propagation only removes completions, never reorders them, so the first
// completion found is still the smallest one.
//
// Kernels:
//   plane_kernel        (plane_kernel.h, own translation unit) one board per
//                       LANE on digit-plane bitboards: the batch hot path;
//   solvep_kernel       (packed_solver.h) one board per WAVEFRONT: small
//                       batches, and the boards the plane kernel hands back;
//   check_kernel, first_candidate_kernel, expand_* (below).
// No MFMA: this is branchy 9-bit mask work, VALU bound.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <atomic>
#include <mutex>
#include <stdlib.h>

#include "../../include/sudoku_hip.h"

#include "common.h"

#ifndef SDK_PLANE_MIN_BATCH
#define SDK_PLANE_MIN_BATCH 8192
#endif

// ------------------------------------------------------------- solve kernel
// re-arm the per-call workspace words on the stream (graph-capturable)
// pool: the plane kernel's tail pool (common.h), or null
__global__ void arm_kernel(unsigned long long *ws, uint32_t *pool)
{
    static_assert(PLANE_POOL_XCDS * PLANE_POOL_ARM_WORDS <= 64, "arm_kernel: one thread per pool word");
    if (pool && threadIdx.x < PLANE_POOL_XCDS * PLANE_POOL_ARM_WORDS) {
        const uint32_t k = threadIdx.x % PLANE_POOL_ARM_WORDS;  // the control words (plane_kernel.h POOL_*)
        pool[(threadIdx.x / PLANE_POOL_ARM_WORDS) * PLANE_POOL_STRIDE + k] = 0u;
    }
    if (threadIdx.x == WS_QUEUE) ws[WS_QUEUE] = 0ull;
    if (threadIdx.x == WS_BEST) ws[WS_BEST] = (unsigned long long)INT64_MAX;
    if (threadIdx.x == WS_DEFER_COUNT) ws[WS_DEFER_COUNT] = 0ull;
    if (threadIdx.x == WS_DEFER_OVER) ws[WS_DEFER_OVER] = 0ull;
    if (threadIdx.x == WS_GEN) {
        // the next generation; its low 32 bits (the pool's flag value) never 0
        unsigned long long g = ws[WS_GEN] + 1ull;
        if ((uint32_t)g == 0u) g++;
        ws[WS_GEN] = g;
    }
}

#include "packed_solver.h"

#ifndef SDK_PACKED_WAVES_PER_EU
#define SDK_PACKED_WAVES_PER_EU 1
#endif
__global__ __launch_bounds__(BLOCK_THREADS, SDK_PACKED_WAVES_PER_EU) void solvep_kernel(
    const uint8_t *__restrict__ puzzles, uint8_t *__restrict__ sols, int32_t *__restrict__ status,
    int64_t n, unsigned long long *__restrict__ ws, int64_t chunk, int ordered, int order)
{
    __shared__ PackLds lds[WAVES_PER_BLOCK];
    const int lane = threadIdx.x & 63;
    PackLds &W = lds[threadIdx.x >> 6];
    const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    const int64_t gw = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    const int64_t *best = ordered ? (const int64_t *)&ws[WS_BEST] : nullptr;

    if (gw == 0 && lane == 0) atomicAdd(&ws[WS_ASSIGNED], (unsigned long long)n);  // sdk_verify_workspace
    PCells s;
    pinit_lane(s, lane);
    uint32_t fin = 0, solved = 0, guesses = 0, sweeps = 0;
    // first chunk statically, the rest from the queue
    int64_t base = gw * chunk;
    const int64_t static_end = nwaves * chunk;
    while (base < n) {
        const int64_t end = base + chunk < n ? base + chunk : n;
        for (int64_t p = base; p < end; ++p) {
            psolve_board(W, lane, s, puzzles, sols, status, p, ws, best, order, solved, guesses, sweeps);
            fin++;
        }
        unsigned long long t = 0;
        if (lane == 0) t = atomicAdd(&ws[WS_QUEUE], 1ull);
        t = __shfl(t, 0);
        base = static_end + (int64_t)t * chunk;
    }
    pflush_stats(lane, ws, fin, solved, guesses, sweeps);
}

// Second pass behind the plane kernel: solve exactly the boards it left
// (status SDK_DEFERRED): the deferred list's entries, one board per wave,
// grid-stride; if the list overflowed, every wave scans 64 statuses per load
// instead and runs the deferred ones among them.
__global__ __launch_bounds__(BLOCK_THREADS, SDK_PACKED_WAVES_PER_EU) void solvep_deferred_kernel(
    const uint8_t *__restrict__ puzzles, uint8_t *__restrict__ sols, int32_t *__restrict__ status,
    int64_t n, unsigned long long *__restrict__ ws, const int64_t *__restrict__ list, int ordered, int order)
{
    __shared__ PackLds lds[WAVES_PER_BLOCK];
    const int lane = threadIdx.x & 63;
    PackLds &W = lds[threadIdx.x >> 6];
    const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    const int64_t gw = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    const int64_t *best = ordered ? (const int64_t *)&ws[WS_BEST] : nullptr;
    // both words were last written by the plane kernel (an earlier launch)
    const int64_t cnt = (int64_t)ws[WS_DEFER_COUNT];
    const bool over = ws[WS_DEFER_OVER] != 0;
    if (cnt == 0 || (!over && gw >= cnt)) return;

    PCells s;
    pinit_lane(s, lane);
    uint32_t fin = 0, solved = 0, guesses = 0, sweeps = 0;
    if (!over) {
        for (int64_t k = gw; k < cnt; k += nwaves) {
            const int64_t p = list[k];
            psolve_board(W, lane, s, puzzles, sols, status, p, ws, best, order, solved, guesses, sweeps);
            fin++;
        }
    } else {
        for (int64_t base = gw * 64; base < n; base += nwaves * 64) {
            const int32_t sv = base + lane < n ? status[base + lane] : 0;
            uint64_t m = __builtin_amdgcn_ballot_w64(sv == SDK_DEFERRED);
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                psolve_board(W, lane, s, puzzles, sols, status, base + j, ws, best, order, solved, guesses, sweeps);
                fin++;
            }
        }
    }
    pflush_stats(lane, ws, fin, solved, guesses, sweeps);
}

// The same for a plane_kernel_multi launch: list entries are board ids
// (batch j << PLANE_BATCH_SHIFT | index), the overflow scan runs batch by batch.
__global__ __launch_bounds__(BLOCK_THREADS, SDK_PACKED_WAVES_PER_EU) void solvep_deferred_multi_kernel(
    const PlaneBatches bs, unsigned long long *__restrict__ ws, const int64_t *__restrict__ list, int order)
{
    __shared__ PackLds lds[WAVES_PER_BLOCK];
    const int lane = threadIdx.x & 63;
    PackLds &W = lds[threadIdx.x >> 6];
    const int64_t nwaves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    const int64_t gw = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    const int64_t cnt = (int64_t)ws[WS_DEFER_COUNT];
    const bool over = ws[WS_DEFER_OVER] != 0;
    if (cnt == 0 || (!over && gw >= cnt)) return;

    PCells s;
    pinit_lane(s, lane);
    uint32_t fin = 0, solved = 0, guesses = 0, sweeps = 0;
    if (!over) {
        for (int64_t k = gw; k < cnt; k += nwaves) {
            const int64_t p = list[k];
            const int j = (int)(p >> PLANE_BATCH_SHIFT);
            psolve_board(W, lane, s, bs.in[j], bs.out[j], bs.status[j], p & PLANE_LOCAL_MASK, ws, nullptr, order,
                         solved, guesses, sweeps);
            fin++;
        }
    } else {
        for (int j = 0; j < bs.count; ++j) {
            const int64_t n = bs.end[j] - (j ? bs.end[j - 1] : 0);
            for (int64_t base = gw * 64; base < n; base += nwaves * 64) {
                const int32_t sv = base + lane < n ? bs.status[j][base + lane] : 0;
                uint64_t m = __builtin_amdgcn_ballot_w64(sv == SDK_DEFERRED);
                while (m) {
                    const int i = __builtin_ctzll(m);
                    m &= m - 1;
                    psolve_board(W, lane, s, bs.in[j], bs.out[j], bs.status[j], base + i, ws, nullptr, order, solved,
                                 guesses, sweeps);
                    fin++;
                }
            }
        }
    }
    pflush_stats(lane, ws, fin, solved, guesses, sweeps);
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

// ------------------------------------------------- reference /solve (greedy)
// node.py:534-557 P2PNode.peer_sudoku_solve, one thread per board
// (peer_greedy.h; its ~1.9 KB of state lives in scratch: a cold serving path).
#include "peer_greedy.h"

__global__ __launch_bounds__(64) void peer_solve_kernel(const uint8_t *__restrict__ boards, uint8_t *__restrict__ out,
                                                        int32_t *__restrict__ status,
                                                        int32_t *__restrict__ validations, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const uint8_t *src = boards + i * 81;
    uint8_t *dst = out + i * 81;
    peer::State s;
    bool bad = false;
    for (int k = 0; k < 81; ++k) {
        s.sudoku[k] = src[k];
        bad |= s.sudoku[k] > 9;
    }
    if (bad) {
        for (int k = 0; k < 81; ++k) dst[k] = s.sudoku[k];
        status[i] = SDK_INVALID;
        validations[i] = 0;
        return;
    }
    int checks = 0;
    peer::clear_node(s.node);  // a fresh node per board
    const int r = peer::run(s, checks);
    for (int k = 0; k < 81; ++k) dst[k] = s.sudoku[k];
    status[i] = r == peer::PG_CHECKED ? SDK_SOLVED : r == peer::PG_CHECK_FAILED ? SDK_UNSOLVABLE : SDK_NO_RETURN;
    validations[i] = checks;
}

// ONE node serving n requests in order (sdk_peer_solve_seq): a single lane
// walks them, the node's partial_solution / tried sets carried from each
// request to the next through `node` (device memory, in and out)
__global__ __launch_bounds__(64) void peer_seq_kernel(const uint8_t *__restrict__ boards, uint8_t *__restrict__ out,
                                                      int32_t *__restrict__ status,
                                                      int32_t *__restrict__ validations, int64_t n,
                                                      peer::NodeState *__restrict__ node)
{
    if (threadIdx.x != 0) return;
    peer::State s;
    s.node = *node;
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t *src = boards + i * 81;
        uint8_t *dst = out + i * 81;
        bool bad = false;
        for (int k = 0; k < 81; ++k) {
            s.sudoku[k] = src[k];
            bad |= s.sudoku[k] > 9;
        }
        int checks = 0, r = -1;
        if (!bad) r = peer::run(s, checks);  // a rejected request leaves the node as it was
        for (int k = 0; k < 81; ++k) dst[k] = s.sudoku[k];
        status[i] = bad ? SDK_INVALID
                        : r == peer::PG_CHECKED ? SDK_SOLVED : r == peer::PG_CHECK_FAILED ? SDK_UNSOLVABLE : SDK_NO_RETURN;
        validations[i] = checks;
    }
    *node = s.node;
}

// ------------------------------------------------------ frontier expansion
// pass 1: propagate each node (one wave each), keep the propagated grid and
// the number of children it will produce.  In node order a node from which
// node.py's short-circuit is reachable (packed_solver.h, literal mode) is not
// propagated: its children are the literal walk's.
__global__ __launch_bounds__(BLOCK_THREADS) void expand_count_kernel(const uint8_t *__restrict__ nodes, int64_t n,
                                                                     uint8_t *__restrict__ tmp,
                                                                     int64_t *__restrict__ counts, int order)
{
    __shared__ PackLds lds[WAVES_PER_BLOCK];
    const int lane = threadIdx.x & 63;
    PackLds &W = lds[threadIdx.x >> 6];
    const int64_t p = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    if (p >= n) return;
    PCells s;
    pinit_lane(s, lane);
    uint8_t *dst = tmp + p * 81;
    int64_t cnt = 0;
    uint32_t a, b;
    if (!pload_board(nodes + p * 81, lane, s, a, b)) {
        dst[lane] = (uint8_t)a;  // raw bytes back, no child
        if (lane < 17) dst[64 + lane] = (uint8_t)b;
    } else {
        uint32_t bad;
        uint32_t gmask = pbuild_given_masks(W, lane, s, bad);
        bool literal = false;
        if (order == SDK_ORDER_NODE && bad) {
            const LitEval e = lit_eval(W, lane, s);
            if (e.R) {
                literal = true;
                const uint64_t eb0 = __builtin_amdgcn_ballot_w64((s.EK & 0x8000u) != 0);
                const uint64_t eb1 = __builtin_amdgcn_ballot_w64((s.EK & 0x80000000u) != 0);
                const int cell = order_cell(eb0, eb1, SDK_ORDER_NODE);
                const uint32_t cand = e.s45 ? 0x1FFu
                                    : cell < 64 ? rdlane(e.cand, cell) & 0x1FFu : rdlane(e.cand, cell - 64) >> 16;
                cnt = __builtin_popcount(cand);
            } else {
                s.GS = s.D;  // already equal: no cell placed yet
            }
        }
        if (!literal) {
            uint32_t c9, sweeps = 0;
            bool rebuild = false;
            const int st = ppropagate(W, lane, s, gmask, bad, 0, rebuild, c9, sweeps);
            if (st == PROP_SOLVED) {
                cnt = 1;
            } else if (st == PROP_OPEN) {
                const uint64_t eb0 = __builtin_amdgcn_ballot_w64((s.EK & 0x8000u) != 0);
                const uint64_t eb1 = __builtin_amdgcn_ballot_w64((s.EK & 0x80000000u) != 0);
                const int cell = order_cell(eb0, eb1, order);
                const uint32_t cand = cell < 64 ? rdlane(c9, cell) & 0x1FFu : rdlane(c9, cell - 64) >> 16;
                cnt = __builtin_popcount(cand);
            }
        }
        pstore_board(dst, lane, s, false);
    }
    if (lane == 0) counts[p] = cnt;
}

// exclusive scan of counts -> offsets (n+1 entries), one block; counts and
// offsets may be the same buffer (in-place scan, hence no __restrict__)
__global__ __launch_bounds__(1024) void scan_kernel(const int64_t *counts, int64_t *offsets, int64_t n)
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
    bool s45 = false;
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
        if (order == SDK_ORDER_NODE) {
            // node.py:44-45: every unit sums to 45 -> is_valid_move accepts 1..9
            bool is45 = true;
            if (lane < 27) {
                uint32_t sum = 0;
                for (int k = 0; k < 9; ++k) {
                    const int idx = lane < 9 ? lane * 9 + k
                                  : lane < 18 ? k * 9 + (lane - 9)
                                              : (((lane - 18) / 3) * 3 + k / 3) * 9 + ((lane - 18) % 3) * 3 + k % 3;
                    sum += g[idx];
                }
                is45 = sum == 45u;
            }
            s45 = !wany(!is45);
        }
    }
    uint32_t cand = cell >= 0 ? (s45 ? 0x1FFu : (~used & 0x1FFu)) : 0u;
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
static std::atomic<int> g_bpc_packed{0}, g_bpc_plane{0};

// waves of the deferred-board kernels after a plane launch: one workgroup
// (4 waves) per CU.  The count of deferred boards is known only on the
// device; the waves past it exit at once, and a full grid of them only
// queues for the slots the next launches in flight want (8.8 % of the
// traced kernel time), while a batch that is mostly deferred
// (clashing givens) still gets a wave per SIMD.
static int64_t deferred_waves() { return (int64_t)cu_count() * WAVES_PER_BLOCK; }

// lanes of a full plane-kernel grid on the current device, and the bytes of
// their stacks (the workspace holds them after WS_STACK_BYTE)
static int64_t plane_max_threads()
{
    if (!g_bpc_plane.load()) g_bpc_plane.store(sdk_plane_blocks_per_cu());
    return (int64_t)cu_count() * g_bpc_plane.load() * PLANE_THREADS;
}
static size_t plane_stack_bytes(int64_t threads)
{
    return (size_t)threads * PLANE_MAX_DEPTH * PLANE_STACK_WORDS * sizeof(uint32_t);
}

// Solve-kernel selection: SDK_KERNEL_AUTO (default) runs the plane kernel
// for batches of at least SDK_PLANE_MIN_BATCH boards and the packed kernel
// below (a lone board on one lane is slower than on a whole wave, and a
// small batch does not fill the lanes).  $SDK_SOLVE_KERNEL = auto | plane |
// packed picks the process default.  Both give identical results.
static std::atomic<int> g_variant{0};

static int env_variant()
{
    const char *e = getenv("SDK_SOLVE_KERNEL");
    if (!e || !e[0] || e[0] == 'a') return SDK_KERNEL_AUTO;
    if (!strcmp(e, "packed") || !strcmp(e, "p")) return SDK_KERNEL_PACKED;
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

// Launches that share a workspace must not interleave: sdk_solve_batch
// re-arms the workspace's queue head before its kernels, so two callers'
// arm / solve pairs are enqueued under this lock (and must share a stream,
// include/sudoku_hip.h).
static std::mutex g_launch_mu;

extern "C" {

const char *sdk_last_error(void) { return g_err; }
const char *sdk_version(void)
{
    const int v = solve_variant();
    return v == SDK_KERNEL_AUTO ? "sudoku_hip 0.6 gfx950 auto: lane-per-board digit-planes (large batches), wave-per-board packed-pairs (small) walk-order"
         : v == SDK_KERNEL_PLANE ? "sudoku_hip 0.6 gfx950 lane-per-board digit-planes walk-order"
                                 : "sudoku_hip 0.6 gfx950 wave-per-board packed-pairs walk-order";
}
int sdk_device_cu_count(void) { return cu_count(); }
int sdk_set_solve_kernel(int kernel)
{
    if (kernel != 0 && kernel != SDK_KERNEL_PACKED && kernel != SDK_KERNEL_PLANE && kernel != SDK_KERNEL_AUTO)
        return -1;
    const int prev = solve_variant();
    g_variant.store(kernel ? kernel : env_variant());
    return prev;
}
// the tail pool: after the stacks and the deferred list
static uint32_t *plane_pool_base(void *d_workspace, int64_t max_threads)
{
    return (uint32_t *)((char *)d_workspace + WS_STACK_BYTE + plane_stack_bytes(max_threads) +
                        (size_t)PLANE_DEFER_CAP * sizeof(int64_t));
}

size_t sdk_workspace_bytes(void)
{
    return WS_STACK_BYTE + plane_stack_bytes(plane_max_threads()) + (size_t)PLANE_DEFER_CAP * sizeof(int64_t) +
           PLANE_POOL_BYTES;
}

int sdk_solve_batch(const uint8_t *d_puzzles, uint8_t *d_solutions, int32_t *d_status, int64_t n,
                    void *d_workspace, int order, int ordered, void *stream)
{
    return sdk_solve_batch_grid(d_puzzles, d_solutions, d_status, n, d_workspace, order, ordered, stream, 0);
}

int sdk_solve_batch_grid(const uint8_t *d_puzzles, uint8_t *d_solutions, int32_t *d_status, int64_t n,
                         void *d_workspace, int order, int ordered, void *stream, int grid_waves)
{
    if (n < 0 || (n > 0 && (!d_puzzles || !d_solutions || !d_status || !d_workspace)) ||
        (order != SDK_ORDER_GEN && order != SDK_ORDER_NODE) || grid_waves < 0) {
        snprintf(g_err, sizeof g_err, "sdk_solve_batch: bad arguments (n=%lld)", (long long)n);
        return -2;
    }
    if (n == 0) return 0;
    const int pipelined = (grid_waves & SDK_GRID_PIPELINED) != 0;
    grid_waves &= ~SDK_GRID_PIPELINED;
    hipStream_t st = (hipStream_t)stream;
    unsigned long long *ws = (unsigned long long *)d_workspace;
    int variant = solve_variant();
    if (variant == SDK_KERNEL_AUTO) variant = n >= SDK_PLANE_MIN_BATCH ? SDK_KERNEL_PLANE : SDK_KERNEL_PACKED;
    std::lock_guard<std::mutex> lk(g_launch_mu);
    hipError_t e;
    if (variant == SDK_KERNEL_PACKED) {
        const int64_t max_waves = (int64_t)cu_count() * blocks_per_cu(solvep_kernel, g_bpc_packed) * WAVES_PER_BLOCK;
        // A batch the static hand-out covers (one board per wave) never uses
        // the queue head's value, and an unordered one not the best word:
        // no re-arm launch then (a single board's latency: -1 launch)
        if (ordered || n > max_waves) hipLaunchKernelGGL(arm_kernel, dim3(1), dim3(64), 0, st, ws, (uint32_t *)nullptr);
        const int64_t waves = n < max_waves ? n : max_waves;
        int64_t chunk = n / (waves * 16);
        if (chunk < 1) chunk = 1;
        if (chunk > 16) chunk = 16;
        const int64_t blocks = (waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
        hipLaunchKernelGGL(solvep_kernel, dim3((unsigned)blocks), dim3(BLOCK_THREADS), 0, st, d_puzzles, d_solutions,
                           d_status, n, ws, chunk, ordered, order);
    } else {
        // lanes: one per board up to a full grid; the stacks sit in the workspace
        const int64_t max_threads = plane_max_threads();
        hipLaunchKernelGGL(arm_kernel, dim3(1), dim3(64), 0, st, ws, plane_pool_base(d_workspace, max_threads));
        // grid_waves > 0: at most that many waves per SIMD (4 SIMDs per CU) in
        // this launch's grid, so launches in flight on other streams are
        // co-resident with it instead of queueing behind its drain
        const int64_t grid_cap = (int64_t)cu_count() * 4 * grid_waves * 64;
        const int64_t lane_cap = grid_waves > 0 && grid_cap < max_threads ? grid_cap : max_threads;
        const int64_t threads = n < lane_cap ? n : lane_cap;
        uint32_t *stack = (uint32_t *)((char *)d_workspace + WS_STACK_BYTE);
        int64_t *list = (int64_t *)((char *)d_workspace + WS_STACK_BYTE + plane_stack_bytes(max_threads));
        e = sdk_launch_plane(d_puzzles, d_solutions, d_status, n, ws, stack, list, ordered, order, threads, pipelined,
                             st);
        if (e != hipSuccess) return set_err("sdk_solve_batch: plane launch", e);
        // the boards it left (clashing givens, deep searches): wave per board,
        // one workgroup per CU (deferred_waves)
        const int64_t max_waves = deferred_waves();
        const int64_t groups = (n + 63) / 64;
        const int64_t waves = groups < max_waves ? groups : max_waves;
        hipLaunchKernelGGL(solvep_deferred_kernel, dim3((unsigned)((waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK)),
                           dim3(BLOCK_THREADS), 0, st, d_puzzles, d_solutions, d_status, n, ws,
                           (const int64_t *)list, ordered, order);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return set_err("sdk_solve_batch: launch", e);
    return 0;
}

int sdk_solve_batches(const uint8_t *const *d_puzzles, uint8_t *const *d_solutions, int32_t *const *d_status,
                      const int64_t *n, int count, void *d_workspace, int order, void *stream, int grid_waves)
{
    if (count < 1 || count > SDK_MAX_BATCHES || !d_puzzles || !d_solutions || !d_status || !n || !d_workspace ||
        (order != SDK_ORDER_GEN && order != SDK_ORDER_NODE) || grid_waves < 0) {
        snprintf(g_err, sizeof g_err, "sdk_solve_batches: bad arguments (count=%d)", count);
        return -2;
    }
    PlaneBatches bs = {};
    int64_t total = 0;
    for (int i = 0; i < count; ++i) {
        if (n[i] < 0 || n[i] > PLANE_LOCAL_MASK || (n[i] > 0 && (!d_puzzles[i] || !d_solutions[i] || !d_status[i]))) {
            snprintf(g_err, sizeof g_err, "sdk_solve_batches: bad batch %d (n=%lld)", i, (long long)n[i]);
            return -2;
        }
        if (n[i] == 0) continue;  // empty batches take no slot
        bs.in[bs.count] = d_puzzles[i];
        bs.out[bs.count] = d_solutions[i];
        bs.status[bs.count] = d_status[i];
        total += n[i];
        bs.end[bs.count] = total;
        bs.count++;
    }
    if (bs.count == 0) return 0;
    int variant = solve_variant();
    if (variant == SDK_KERNEL_AUTO) variant = total >= SDK_PLANE_MIN_BATCH ? SDK_KERNEL_PLANE : SDK_KERNEL_PACKED;
    if (bs.count == 1 || variant == SDK_KERNEL_PACKED) {
        // one batch, or the wave-per-board kernel: the batches one after the other
        for (int i = 0; i < bs.count; ++i) {
            const int rc = sdk_solve_batch_grid(bs.in[i], bs.out[i], bs.status[i], bs.end[i] - (i ? bs.end[i - 1] : 0),
                                                d_workspace, order, 0, stream, grid_waves);
            if (rc) return rc;
        }
        return 0;
    }
    const int pipelined = (grid_waves & SDK_GRID_PIPELINED) != 0;
    grid_waves &= ~SDK_GRID_PIPELINED;
    hipStream_t st = (hipStream_t)stream;
    unsigned long long *ws = (unsigned long long *)d_workspace;
    std::lock_guard<std::mutex> lk(g_launch_mu);
    const int64_t max_threads = plane_max_threads();
    hipLaunchKernelGGL(arm_kernel, dim3(1), dim3(64), 0, st, ws, plane_pool_base(d_workspace, max_threads));
    const int64_t grid_cap = (int64_t)cu_count() * 4 * grid_waves * 64;
    const int64_t lane_cap = grid_waves > 0 && grid_cap < max_threads ? grid_cap : max_threads;
    const int64_t threads = total < lane_cap ? total : lane_cap;
    uint32_t *stack = (uint32_t *)((char *)d_workspace + WS_STACK_BYTE);
    int64_t *list = (int64_t *)((char *)d_workspace + WS_STACK_BYTE + plane_stack_bytes(max_threads));
    hipError_t e = sdk_launch_plane_multi(bs, ws, stack, list, order, threads, pipelined, st);
    if (e != hipSuccess) return set_err("sdk_solve_batches: plane launch", e);
    const int64_t max_waves = deferred_waves();
    const int64_t groups = (total + 63) / 64;
    const int64_t waves = groups < max_waves ? groups : max_waves;
    hipLaunchKernelGGL(solvep_deferred_multi_kernel, dim3((unsigned)((waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK)),
                       dim3(BLOCK_THREADS), 0, st, bs, ws, (const int64_t *)list, order);
    e = hipGetLastError();
    if (e != hipSuccess) return set_err("sdk_solve_batches: launch", e);
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
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, (const int64_t *)d_offsets, d_offsets, n);
    hipLaunchKernelGGL(expand_write_kernel, dim3(blocks), dim3(BLOCK_THREADS), 0, st, d_tmp, n, d_offsets,
                       d_children, cap, order);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("sdk_expand_frontier: launch", e);
}

int sdk_peer_solve_batch(const uint8_t *d_boards, uint8_t *d_out, int32_t *d_status, int32_t *d_validations, int64_t n,
                         void *stream)
{
    if (n < 0 || (n > 0 && (!d_boards || !d_out || !d_status || !d_validations))) {
        snprintf(g_err, sizeof g_err, "sdk_peer_solve_batch: bad arguments");
        return -2;
    }
    if (n == 0) return 0;
    hipLaunchKernelGGL(peer_solve_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream, d_boards,
                       d_out, d_status, d_validations, n);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("sdk_peer_solve_batch: launch", e);
}

int sdk_peer_solve_seq(const uint8_t *d_boards, uint8_t *d_out, int32_t *d_status, int32_t *d_validations, int64_t n,
                       void *d_node_state, void *stream)
{
    static_assert(sizeof(peer::NodeState) == SDK_PEER_STATE_BYTES, "node state record");
    if (n < 0 || !d_node_state || (n > 0 && (!d_boards || !d_out || !d_status || !d_validations))) {
        snprintf(g_err, sizeof g_err, "sdk_peer_solve_seq: bad arguments");
        return -2;
    }
    if (n == 0) return 0;
    hipLaunchKernelGGL(peer_seq_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_boards, d_out, d_status,
                       d_validations, n, (peer::NodeState *)d_node_state);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("sdk_peer_solve_seq: launch", e);
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
        // the counters and the assigned-boards word (never the error word:
        // only sdk_verify_workspace clears it, once it has reported it)
        static_assert(WS_ASSIGNED == WS_FINISHED + 5, "counter words");
        e = hipMemsetAsync((unsigned long long *)d_workspace + WS_FINISHED, 0, 6 * sizeof(unsigned long long), st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return set_err("sdk_read_stats: reset", e);
    }
    return 0;
}

int sdk_verify_workspace(void *d_workspace, int64_t out[4], void *stream)
{
    if (!d_workspace) {
        snprintf(g_err, sizeof g_err, "sdk_verify_workspace: bad arguments");
        return -2;
    }
    hipStream_t st = (hipStream_t)stream;
    unsigned long long h[WS_WORDS];
    hipError_t e = hipMemcpyAsync(h, d_workspace, sizeof h, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return set_err("sdk_verify_workspace", e);
    if (out) {
        out[0] = (int64_t)h[WS_ASSIGNED];
        out[1] = (int64_t)h[WS_FINISHED];
        out[2] = (int64_t)h[WS_ERROR];
        out[3] = 0;  // reserved
    }
    if (h[WS_ASSIGNED] == h[WS_FINISHED] && h[WS_ERROR] == 0) return 0;
    snprintf(g_err, sizeof g_err,
             "sdk_verify_workspace: %lld boards handed to the solve kernels, %lld answered; error bits 0x%llx%s "
             "(pool slot %llu)",
             (long long)h[WS_ASSIGNED], (long long)h[WS_FINISHED], h[WS_ERROR],
             (h[WS_ERROR] & SDK_ERR_POOL_WAIT) ? ": a tail-pool record was never published" : "",
             h[WS_ERR_SLOT]);
    // reported once: the next check starts from a consistent workspace
    unsigned long long fix[2] = {h[WS_FINISHED], 0ull};
    static_assert(WS_ERROR == WS_ASSIGNED + 1, "assigned / error words");
    e = hipMemcpyAsync((unsigned long long *)d_workspace + WS_ASSIGNED, fix, sizeof fix, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return set_err("sdk_verify_workspace: clear", e);
    return -3;
}

__global__ void snapshot_stats_kernel(const unsigned long long *__restrict__ ws, int64_t *__restrict__ out)
{
    const int i = threadIdx.x;
    const int word[6] = {WS_FINISHED, WS_SOLVED, WS_GUESSES, WS_SWEEPS, WS_BEST, WS_DEFERRED};
    if (i < 6) out[i] = (int64_t)ws[word[i]];
}

int sdk_snapshot_stats(const void *d_workspace, int64_t *d_out, void *stream)
{
    if (!d_workspace || !d_out) {
        snprintf(g_err, sizeof g_err, "sdk_snapshot_stats: bad arguments");
        return -2;
    }
    hipLaunchKernelGGL(snapshot_stats_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                       (const unsigned long long *)d_workspace, d_out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_err("sdk_snapshot_stats: launch", e);
}

}  // extern "C"
