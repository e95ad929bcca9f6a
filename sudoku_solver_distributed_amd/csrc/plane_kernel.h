// plane_kernel.h -- the hot solve kernel: one board per LANE on digit planes
// (plane_solver.h), built in its own translation unit (plane_kernels.hip).
//
// Why a lane per board: on digit planes one lane runs a whole propagation
// pass over its board (naked AND hidden singles for every cell and unit) in
// ~1300 issue slots, i.e. ~20 wave instructions per board-pass, where a
// wave-per-board solver spends ~57 per sweep on masks for 81 cells spread
// over 64 lanes, LDS round trips and wave-uniform control.
//
// Execution: persistent lanes.  Each lane holds one board (27 plane words +
// 3 bookkeeping words in VGPRs) and steps it one pass per loop iteration;
// guesses push the 27 words + the branch entry to the lane's stack lines in
// the workspace (PlaneStack).  Finished lanes wait until at least
// SDK_PLANE_REFILL lanes of the wave are free, then stores and refills run
// once for all of them: solved boards go to the wave's LDS outbox (written
// out 64 at a time, a board per lane, as dwords), new boards come from the
// wave's chunk records in LDS (each claimed chunk staged as one span and
// converted lane-parallel to value bit-slices once; a refilled lane reads
// its record and builds its planes).  Boards come from a static first
// hand-out and then chunked claims on one queue head.  A workgroup is one
// wave: the waves share nothing, and a finished wave frees its LDS at once
// for the next launch in flight (BatchSolver.solve_inflight).
//
// Once the queue is empty, a wave down to SDK_PLANE_TAIL boards hands them to
// the wave-wide solver (plane_wide.h): each board in turn is spread over the
// whole wave and its search continues from the lane's state and stack.
//
// Boards the planes cannot take -- givens that repeat a digit in a unit
// (rules B/C are unsound there, plane_solver.h; tested only once a board's
// search ends without a completion, since a completion proves the givens
// clean) or a search deeper than PLANE_MAX_DEPTH -- get status SDK_DEFERRED
// and an entry in the deferred list; solvep_deferred_kernel solves exactly
// those afterwards.  Results are identical either way.
#ifndef SDK_PLANE_KERNEL_H
#define SDK_PLANE_KERNEL_H

#include "plane_solver.h"
#include "plane_wide.h"

// defaults of the runtime knobs (plane_kernels.hip: $SDK_PLANE_REFILL,
// $SDK_PLANE_TAIL, $SDK_PLANE_TAIL_MODE, $SDK_PLANE_CHUNK)
#ifndef SDK_PLANE_REFILL
#define SDK_PLANE_REFILL 3
#endif
#ifndef SDK_PLANE_TAIL
#define SDK_PLANE_TAIL 6  // 12 until rule D and the open-root count shortened the heavy boards
#endif
// 2: continue through the XCD's tail pool on the wave-wide solver, 1: the
// wave-wide solver on the wave's own boards only.  1 since round 6: with
// ~15 passes per board a wave's last boards end soon enough that sharing
// them through the pool (claims, flags) costs more than it evens out
// (+2.7 % on an 8-GPU rank, +1 % on a 4-GPU one, +2 % search-heavy)
#ifndef SDK_PLANE_TAIL_MODE
#define SDK_PLANE_TAIL_MODE 1
#endif
// a pipelined launch's (SDK_GRID_PIPELINED)
#ifndef SDK_PLANE_PIPE_TAIL
#define SDK_PLANE_PIPE_TAIL 8
#endif
#ifndef SDK_PLANE_PIPE_TAIL_MODE
#define SDK_PLANE_PIPE_TAIL_MODE 1
#endif
#ifndef SDK_PLANE_CHUNK
#define SDK_PLANE_CHUNK 64
#endif
// passes on a board before its search switches from the walk's branch order
// to the completion count (plane::search_step; 0: never).  128 since round 6
// (box -> row pointing on): the metric's boards are unchanged, the
// search-heavy set +6 %, an 8-GPU rank +3 % against 64
#ifndef SDK_PLANE_MRV
#define SDK_PLANE_MRV 128
#endif
// guided claims: a wave takes (boards left, as of its own last claim) /
// (SDK_PLANE_GUIDE x waves), at least its idle lanes, at most `chunk`
#ifndef SDK_PLANE_GUIDE
#define SDK_PLANE_GUIDE 3
#endif
#ifndef SDK_PLANE_PUSH_PAD
#define SDK_PLANE_PUSH_PAD 1
#endif
// diagnostic builds only (build.py --tag stamps -DSDK_PLANE_STAMPS=1): per
// wave, s_memrealtime (100 MHz) at start, when the queue drained and at exit,
// plus the loop iterations after the drain, into the second half of the
// deferred-list area (scripts/plane_timeline.py reads them)
#ifndef SDK_PLANE_STAMPS
#define SDK_PLANE_STAMPS 0
#endif
#ifndef SDK_PLANE_LDS_PAD
#define SDK_PLANE_LDS_PAD 0
#endif
static_assert(plane::STACK_ENTRY == 27, "stack layout");
typedef uint32_t sdk_v4u __attribute__((ext_vector_type(4)));

// Per-lane DFS stack in the workspace: level L of lane g is one 128-byte
// line at byte (g * PLANE_MAX_DEPTH + L) * 128, words 0..26 = the 27 planes
// (word 3d+b = P[d][b]), word 27 = the branch entry, 28..31 unused.  A push
// or pop is 7 buffer dwordx4 accesses to ONE line (guesses are lane-
// divergent: a lane-interleaved layout made every push touch 28 lines).
struct PlaneStack {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t lane_off;  // g * PLANE_MAX_DEPTH * 128
    __device__ __forceinline__ uint32_t voff(uint32_t level) const { return lane_off + level * 128u; }
    // a value the optimizer cannot trace back to the board's memory layout:
    // four consecutive board words gathered into a vector are otherwise
    // turned into one vector load, which keeps the whole board in scratch
    static __device__ __forceinline__ uint32_t opaque(uint32_t x)
    {
        asm("" : "+v"(x));
        return x;
    }
    __device__ __forceinline__ void push(uint32_t level, plane::Board &B, uint32_t entry) const
    {
        const int v = (int)voff(level);
        plane::pin_board(B);
#define PQ(a, b, c, d) (sdk_v4u){B.P[a / 3][a % 3], B.P[b / 3][b % 3], B.P[c / 3][c % 3], B.P[d / 3][d % 3]}
        const sdk_v4u q0 = PQ(0, 1, 2, 3), q1 = PQ(4, 5, 6, 7), q2 = PQ(8, 9, 10, 11), q3 = PQ(12, 13, 14, 15),
                      q4 = PQ(16, 17, 18, 19), q5 = PQ(20, 21, 22, 23),
                      q6 = (sdk_v4u){B.P[8][0], B.P[8][1], B.P[8][2], entry};
#undef PQ
        __builtin_amdgcn_raw_buffer_store_b128(q0, rsrc, v, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(q1, rsrc, v, 16, 0);
        __builtin_amdgcn_raw_buffer_store_b128(q2, rsrc, v, 32, 0);
        __builtin_amdgcn_raw_buffer_store_b128(q3, rsrc, v, 48, 0);
        __builtin_amdgcn_raw_buffer_store_b128(q4, rsrc, v, 64, 0);
        __builtin_amdgcn_raw_buffer_store_b128(q5, rsrc, v, 80, 0);
        __builtin_amdgcn_raw_buffer_store_b128(q6, rsrc, v, 96, 0);
#if SDK_PLANE_PUSH_PAD
        // a dwordx4 store reads its data registers after issue; hipcc pads a
        // following VALU write of them only when soffset is an inline constant,
        // and with a register soffset (offsets past 64) it has reused them at
        // once.  Keeping all seven quads live through a 2-state pad makes
        // every store read its data before any of them is overwritten.
        asm volatile("s_nop 1" ::"v"(q0), "v"(q1), "v"(q2), "v"(q3), "v"(q4), "v"(q5), "v"(q6));
#endif
    }
    // the last quad: planes 24..26 and the branch entry
    __device__ __forceinline__ sdk_v4u top(uint32_t level) const
    {
        return __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)voff(level), 96, 0);
    }
    // the whole line in one round trip: the entry (last quad) decides whether
    // the level still has a digit; if not (rare), the planes go unused
    __device__ __forceinline__ uint32_t pop(uint32_t level, plane::Board &B) const { return pop_line(level, B)[3]; }
    __device__ __forceinline__ sdk_v4u pop_line(uint32_t level, plane::Board &B) const
    {
        const int v = (int)voff(level);
        const sdk_v4u q0 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 0, 0);
        const sdk_v4u q1 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 16, 0);
        const sdk_v4u q2 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 32, 0);
        const sdk_v4u q3 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 48, 0);
        const sdk_v4u q4 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 64, 0);
        const sdk_v4u q5 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 80, 0);
        const sdk_v4u t = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 96, 0);
        B.P[0][0] = q0.x; B.P[0][1] = q0.y; B.P[0][2] = q0.z; B.P[1][0] = q0.w;
        B.P[1][1] = q1.x; B.P[1][2] = q1.y; B.P[2][0] = q1.z; B.P[2][1] = q1.w;
        B.P[2][2] = q2.x; B.P[3][0] = q2.y; B.P[3][1] = q2.z; B.P[3][2] = q2.w;
        B.P[4][0] = q3.x; B.P[4][1] = q3.y; B.P[4][2] = q3.z; B.P[5][0] = q3.w;
        B.P[5][1] = q4.x; B.P[5][2] = q4.y; B.P[6][0] = q4.z; B.P[6][1] = q4.w;
        B.P[6][2] = q5.x; B.P[7][0] = q5.y; B.P[7][1] = q5.z; B.P[7][2] = q5.w;
        B.P[8][0] = t.x; B.P[8][1] = t.y; B.P[8][2] = t.z;
        // all seven loads issued before the caller's branch on the entry
        plane::pin_board(B);
        return t;
    }
    __device__ __forceinline__ void restore(uint32_t level, plane::Board &B, const sdk_v4u &t) const
    {
        const int v = (int)voff(level);
        const sdk_v4u q0 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 0, 0);
        const sdk_v4u q1 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 16, 0);
        const sdk_v4u q2 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 32, 0);
        const sdk_v4u q3 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 48, 0);
        const sdk_v4u q4 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 64, 0);
        const sdk_v4u q5 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 80, 0);
        B.P[0][0] = q0.x; B.P[0][1] = q0.y; B.P[0][2] = q0.z; B.P[1][0] = q0.w;
        B.P[1][1] = q1.x; B.P[1][2] = q1.y; B.P[2][0] = q1.z; B.P[2][1] = q1.w;
        B.P[2][2] = q2.x; B.P[3][0] = q2.y; B.P[3][1] = q2.z; B.P[3][2] = q2.w;
        B.P[4][0] = q3.x; B.P[4][1] = q3.y; B.P[4][2] = q3.z; B.P[5][0] = q3.w;
        B.P[5][1] = q4.x; B.P[5][2] = q4.y; B.P[6][0] = q4.z; B.P[6][1] = q4.w;
        B.P[6][2] = q5.x; B.P[7][0] = q5.y; B.P[7][1] = q5.z; B.P[7][2] = q5.w;
        B.P[8][0] = t.x; B.P[8][1] = t.y; B.P[8][2] = t.z;
    }
    __device__ __forceinline__ void put_entry(uint32_t level, uint32_t entry) const
    {
        __builtin_amdgcn_raw_buffer_store_b32(entry, rsrc, (int)voff(level), 108, 0);
    }
};

// Cooperative board I/O.  Loads and stores run for one board at a time over
// the whole wave, in the band-word layout: lane l's slot 0 is bit (l & 31)
// of band l >> 5 and its slot 1 bit l of band 2, so one ballot per digit and
// slot yields that digit's band words directly (bits 9, 19, 29 and 30-31 of
// a band word are no cell: those slots hold none).
__device__ __forceinline__ int plane_slot_cell(int lane, int slot)
{
    const int band = slot ? 2 : (lane >> 5), pos = lane & 31;
    if ((slot && lane >= 32) || pos >= 30 || pos % 10 == 9) return -1;
    return 27 * band + 9 * (pos / 10) + pos % 10;
}

// copy board q's 81 bytes from src to dst (lanes l and 64 + l)
__device__ __forceinline__ void plane_copy_board(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, int lane)
{
    dst[lane] = src[lane];
    if (lane < 17) dst[64 + lane] = src[64 + lane];
}

// Do board src's givens repeat a digit in a unit?  Wave-cooperative (the
// ballots make its planes wave-uniform); run only for boards the planes
// found unsolvable, which is rare.
__device__ __forceinline__ bool plane_givens_clash(const uint8_t *__restrict__ src, int c0, int c1)
{
    const uint32_t a0 = c0 >= 0 ? src[c0] : 0x100u, a1 = c1 >= 0 ? src[c1] : 0x100u;
    plane::Board G;
    uint32_t given[3];
    const uint64_t e0 = __builtin_amdgcn_ballot_w64(a0 == 0u);
    const uint32_t E[3] = {(uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)__builtin_amdgcn_ballot_w64(a1 == 0u)};
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        const uint64_t m0 = __builtin_amdgcn_ballot_w64(a0 == (uint32_t)(d + 1));
        G.P[d][0] = (uint32_t)m0;
        G.P[d][1] = (uint32_t)(m0 >> 32);
        G.P[d][2] = (uint32_t)__builtin_amdgcn_ballot_w64(a1 == (uint32_t)(d + 1));
    }
#pragma unroll
    for (int b = 0; b < 3; ++b) given[b] = plane::ROWS & ~E[b];
    return plane::givens_clash(G, given);
}

// Hand board p (status word st) to the wave kernel (status SDK_DEFERRED + an
// entry in the deferred list; past PLANE_DEFER_CAP entries the wave kernel
// scans statuses).
__device__ __forceinline__ void plane_defer(int32_t *st, int64_t p, unsigned long long *__restrict__ ws,
                                            int64_t *__restrict__ list)
{
    *st = SDK_DEFERRED;
    const unsigned long long k = atomicAdd(&ws[WS_DEFER_COUNT], 1ull);
    if (k < (unsigned long long)PLANE_DEFER_CAP) list[k] = p;
    else atomicOr(&ws[WS_DEFER_OVER], 1ull);
}

// ---- board I/O of one launch.  The queue hands out VIRTUAL indices v over
// the launch's boards; a claimed range is staged one batch segment at a time
// (seg_*), and a lane keeps its board's id p (src / dst / stat).  One batch
// (PlaneIO1, sdk_solve_batch): p = v = the board's index.  Several batches
// (PlaneIOn, sdk_solve_batches): p = j << PLANE_BATCH_SHIFT | index in batch
// j, and v runs over the batches laid end to end.
struct PlaneIO1 {
    static constexpr bool multi = false;
    const uint8_t *in;
    uint8_t *out;
    int32_t *st;
    int64_t n;
    __device__ __forceinline__ int64_t total() const { return n; }
    __device__ __forceinline__ const uint8_t *src(int64_t p) const { return in + p * 81; }
    __device__ __forceinline__ uint8_t *dst(int64_t p) const { return out + p * 81; }
    __device__ __forceinline__ int32_t *stat(int64_t p) const { return st + p; }
    // board p's batch, as (input, output, status, index) for the wave solver
    __device__ __forceinline__ const uint8_t *b_in(int64_t) const { return in; }
    __device__ __forceinline__ uint8_t *b_out(int64_t) const { return out; }
    __device__ __forceinline__ int32_t *b_st(int64_t) const { return st; }
    __device__ __forceinline__ int64_t local(int64_t p) const { return p; }
    // the segment from virtual v: its end (at most hi), v's id, the batch's
    // input, its size and v's index in it
    __device__ __forceinline__ int64_t seg_end(int64_t, int64_t hi) const { return hi; }
    __device__ __forceinline__ int64_t id(int64_t v) const { return v; }
    __device__ __forceinline__ const uint8_t *seg_in(int64_t) const { return in; }
    __device__ __forceinline__ int64_t seg_n(int64_t) const { return n; }
    __device__ __forceinline__ int64_t seg_local(int64_t v) const { return v; }
};

struct PlaneIOn {
    static constexpr bool multi = true;
    const PlaneBatches &b;
    __device__ __forceinline__ int64_t total() const { return b.end[b.count - 1]; }
    // batch of virtual v (wave-uniform: a scalar loop over at most 31 bounds)
    __device__ __forceinline__ int batch(int64_t v) const
    {
        int j = 0;
        for (int k = 0; k + 1 < b.count; ++k) j += v >= b.end[k];
        return j;
    }
    __device__ __forceinline__ int64_t start(int j) const { return j ? b.end[j - 1] : 0; }
    __device__ __forceinline__ const uint8_t *b_in(int64_t p) const { return b.in[p >> PLANE_BATCH_SHIFT]; }
    __device__ __forceinline__ uint8_t *b_out(int64_t p) const { return b.out[p >> PLANE_BATCH_SHIFT]; }
    __device__ __forceinline__ int32_t *b_st(int64_t p) const { return b.status[p >> PLANE_BATCH_SHIFT]; }
    __device__ __forceinline__ int64_t local(int64_t p) const { return p & PLANE_LOCAL_MASK; }
    __device__ __forceinline__ const uint8_t *src(int64_t p) const { return b_in(p) + local(p) * 81; }
    __device__ __forceinline__ uint8_t *dst(int64_t p) const { return b_out(p) + local(p) * 81; }
    __device__ __forceinline__ int32_t *stat(int64_t p) const { return b_st(p) + local(p); }
    __device__ __forceinline__ int64_t seg_end(int64_t v, int64_t hi) const
    {
        const int64_t e = b.end[batch(v)];
        return e < hi ? e : hi;
    }
    __device__ __forceinline__ int64_t id(int64_t v) const
    {
        const int j = batch(v);
        return ((int64_t)j << PLANE_BATCH_SHIFT) | (v - start(j));
    }
    __device__ __forceinline__ const uint8_t *seg_in(int64_t v) const { return b.in[batch(v)]; }
    __device__ __forceinline__ int64_t seg_n(int64_t v) const
    {
        const int j = batch(v);
        return b.end[j] - start(j);
    }
    __device__ __forceinline__ int64_t seg_local(int64_t v) const { return v - start(batch(v)); }
};

// ---- cooperative span loads through LDS
// A refill (and the start-up) takes k <= 64 CONSECUTIVE boards from the
// queue, i.e. one contiguous byte span of the batch.  It lands in the wave's
// LDS staging area by buffer_load_dword ... lds (one wave instruction per 64
// dwords, all in flight together, no VGPRs), so a refill costs one HBM round
// trip instead of one per board; the per-board ballots then read bytes from
// LDS.  Bytes past the batch read as 0 (buffer range check).
// >= (3 + 64*81 + 3) / 4 rounded up to 64 (the span DMA writes whole 64-dword
// rows), plus one dword the DMA never writes: a zero byte for the refill's
// cell-less slots (byte offset PLANE_STAGE_ZERO, zeroed at kernel start)
// (a five-waves-per-SIMD budget, <= 8 KB of LDS per wave with 48-board
// claims, a 56-board outbox and two start-up spans, measured -4 % / -9 % at
// N = 1 / 8: the 96-VGPR limit spills 30 registers in the lane loop)
enum {
    PLANE_STAGE_DWORDS = 1348, PLANE_STAGE_ZERO = 4 * (PLANE_STAGE_DWORDS - 1),
    PLANE_START_SPAN = 64  // boards per staged span at start-up
};

typedef __attribute__((address_space(3))) void lds_void_t;
// s_waitcnt immediates (gfx9: vmcnt bits 3:0 + 15:14, expcnt 6:4, lgkmcnt 11:8)
enum { SDK_WAIT_VM0 = 0x0F70, SDK_WAIT_LGKM0 = 0xC07F, SDK_WAIT_VM0_LGKM0 = 0x0070 };

__device__ __forceinline__ uint32_t plane_stage_span(const uint8_t *__restrict__ puzzles, int64_t n, int64_t q0, int k,
                                                     uint32_t *stage, int lane)
{
    const uint64_t start = (uint64_t)q0 * 81u, a0 = start & ~3ull, total = (uint64_t)n * 81u;
    const uint32_t shift = (uint32_t)(start - a0);
    const uint64_t avail = total - a0;
    const uint32_t nrec = avail > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)avail;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(puzzles + a0), 0, (int)nrec, 0x00020000);
    const uint32_t nd = (shift + 81u * (uint32_t)k + 3u) / 4u;
    // the DMA writes LDS through the memory path, unordered with this wave's
    // earlier ds_writes to the same area (the store path's bit-slices):
    // those must have landed first
    __builtin_amdgcn_s_waitcnt(SDK_WAIT_LGKM0);
    for (uint32_t i = 0; i < nd; i += 64)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t *)(stage + i), 4, (int)((i + lane) * 4u), 0, 0, 0);
    // (the builtin, not inline asm: the compiler's wait tracking sees it, so
    // later LDS reads do not wait on every outstanding store "in case" they
    // alias the DMA -- with asm here the store loop drained vmcnt per board)
    __builtin_amdgcn_s_waitcnt(SDK_WAIT_VM0);
    // the batch's last dword may be partial: the range check zeroes all of
    // it, so its bytes come in one by one
    const uint64_t tail = total & ~3ull;
    if ((total & 3u) && tail >= a0 && tail < a0 + 4ull * nd) {
        uint8_t *sb = (uint8_t *)stage;
        if ((uint64_t)lane < (total & 3u)) sb[tail - a0 + lane] = puzzles[tail + lane];
        __builtin_amdgcn_s_waitcnt(SDK_WAIT_VM0_LGKM0);
    }
    return shift;
}

// lanes of `mask` below this lane
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// The 21 words of the board at byte offset o of the staging area (22 aligned
// dword reads, funnel-shifted into place)
__device__ __forceinline__ void plane_stage_words(const uint32_t *stage, uint32_t o, uint32_t (&x)[21])
{
    const uint32_t *d = stage + (o >> 2);
    const uint32_t r = (o & 3u) * 8u;
    uint32_t lo = d[0];
#pragma unroll
    for (int k = 0; k < 21; ++k) {
        const uint32_t hi = d[k + 1];
        x[k] = r ? __builtin_amdgcn_alignbit(hi, lo, r) : lo;
        lo = hi;
    }
}

// ---- chunk records
// A claimed chunk (<= 64 consecutive boards) is staged once and converted
// lane-parallel, a board per lane, into records of its value bit-slices:
// V[s][b] at word 3s + b, word 12 = nonzero if a byte is > 9 (stride 13, odd:
// 64 lanes writing / reading one word each hit 64 different banks).  A
// refill then hands record i to the idle lane of rank i: every loaded lane
// reads its own record at once, no per-board serial work.
enum { PLANE_REC = 13, PLANE_CHUNK_MAX = 64 };
static_assert(PLANE_CHUNK_MAX * PLANE_REC + 1 < PLANE_STAGE_DWORDS, "chunk records");
static_assert((3 + 81 * PLANE_CHUNK_MAX + 3 + 255) / 256 * 64 < PLANE_STAGE_DWORDS, "a claimed chunk's span");
static_assert((3 + 81 * PLANE_START_SPAN + 3 + 255) / 256 * 64 < PLANE_STAGE_DWORDS, "a start-up span");

__device__ __forceinline__ void plane_convert_chunk(uint32_t *stage, uint32_t sh, int count, int lane)
{
    uint32_t V[4][3], bad = 0;
    if (lane < count) {
        uint32_t x[21];
        plane_stage_words(stage, sh + 81u * (uint32_t)lane, x);
        bad = plane::slices_from_words(x, V);
    }
    // every lane's bytes are read (the loads above complete before their
    // values are used) before any record overwrites them
    if (lane < count) {
        uint32_t *rec = stage + PLANE_REC * lane;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int b = 0; b < 3; ++b) rec[3 * s + b] = V[s][b];
        rec[12] = bad;
    }
}

// ---- the store path's outbox
// a record per solved board: value bit-slices V[k][b] (bit 10r + c of band
// b = bit k of the value at cell (3b + r, c)) and the board index, as
// V00 V01 V02 V10 | V11 V12 V20 V21 | V22 V30 V31 V32 | p_lo p_hi - -
enum { PLANE_OUTBOX = 64, PLANE_OB_WORDS = 16 };

// 27 cells of a band word without its guard bits (bit 9r + c)
__device__ __forceinline__ uint32_t plane_unguard(uint32_t v)
{
    return plane::or3(v & 0x1FFu, (v >> 1) & 0x3FE00u, (v >> 2) & 0x7FC0000u);
}

// Lane j < count writes outbox board j: its 81 bytes as the 21 dwords of its
// span (sh = the board's offset in its first dword): dwords 1..19 whole, 0
// and 20 whole when the span starts / ends on a dword boundary, byte by
// byte otherwise (they hold neighbouring boards' bytes).  Byte expansion:
// value bit k of 4 consecutive cells, a nibble of the slice's 81-bit cell
// stream, spreads to bit k of 4 bytes with one multiply (bit i -> bit 8i).
template <class IO>
__device__ __forceinline__ void plane_flush_outbox(const uint32_t *outbox, uint32_t count, int lane, const IO &io)
{
    if ((uint32_t)lane < count) {
        const sdk_v4u *rec = (const sdk_v4u *)(outbox + PLANE_OB_WORDS * lane);
        const sdk_v4u r0 = rec[0], r1 = rec[1], r2 = rec[2], r3 = rec[3];
        const uint32_t V[4][3] = {{r0.x, r0.y, r0.z}, {r0.w, r1.x, r1.y}, {r1.z, r1.w, r2.x}, {r2.y, r2.z, r2.w}};
        const int64_t pb = ((int64_t)r3.y << 32) | r3.x;
        uint8_t *dst = io.dst(pb);
        const uint32_t sh = (uint32_t)(uintptr_t)dst & 3u;
        uint32_t *dw = (uint32_t *)(dst - sh);
        // per slice: the 81-bit cell stream, shifted up by sh bits (byte
        // offset sh in the first dword: bit 8i + k of dword j <- cell 4j + i - sh)
        uint32_t T[4][3];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w0 = plane_unguard(V[k][0]), w1 = plane_unguard(V[k][1]), w2 = plane_unguard(V[k][2]);
            const uint32_t s0 = w0 | (w1 << 27), s1 = (w1 >> 5) | (w2 << 22), s2 = w2 >> 10;  // cells 0..80
            // (x >> 1) >> (31 - sh): the bits carried up, 0 for sh = 0
            T[k][0] = s0 << sh;
            T[k][1] = (s1 << sh) | ((s0 >> 1) >> (31u - sh));
            T[k][2] = (s2 << sh) | ((s1 >> 1) >> (31u - sh));
        }
        // dword j of the span from the slices' nibbles 4j..4j+3
        auto word = [&](const int j) {
            const int sw = j / 8, sb = (4 * j) % 32;
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t nib = (sb >= k ? (T[k][sw] >> (sb - k)) : (T[k][sw] << (k - sb))) & (0xFu << k);
                acc |= plane::mul24(nib, 0x204081u) & (0x01010101u << k);
            }
            return acc;
        };
        // each dword stored as soon as it is made (few live registers)
#pragma unroll
        for (int j = 1; j < 20; ++j) dw[j] = word(j);
        const uint32_t first = word(0), last = word(20);
        if (sh == 0) {
            dw[0] = first;
        } else {
#pragma unroll
            for (int i = 1; i < 4; ++i)
                if ((uint32_t)i >= sh) dst[i - (int)sh] = (uint8_t)(first >> (8 * i));
        }
        if (sh == 3) {
            dw[20] = last;
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if ((uint32_t)i <= sh) dst[80 - (int)sh + i] = (uint8_t)(last >> (8 * i));
        }
    }
}

// ---- the wave-wide tail (plane_wide.h)
// a record per handed-over board in the wave's staging area (stride: odd, so
// 64 lanes writing one word each hit 64 banks): 27 plane words, board index
// lo / hi, depth, stack line offset, guesses so far
enum { PLANE_TAIL_REC = 33, PLANE_TAIL_MAX = 40 };  // word 32: the board's search mode (mst)
// the last record, read up to word 48 (pad lanes), stays below the zero byte
static_assert((PLANE_TAIL_MAX - 1) * PLANE_TAIL_REC + 48 < PLANE_STAGE_DWORDS - 1, "tail records");

// The board's stack in the wide layout: lane 16b+d owns word 3d+b of each
// level's line; the branch entry (word 27) goes through lane 48 (a pad lane)
// on a push, lane 0 on an update; every lane reads it.
struct WideStack {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t lane_off;  // the board's stack (uniform)
    uint32_t off;       // this lane's word: 4 * (3d + b); pad lanes the entry (108)
    bool valid, entry_lane;
    __device__ __forceinline__ void push(uint32_t level, uint32_t w, const wide::Lanes &, uint32_t entry) const
    {
        if (valid || entry_lane)
            __builtin_amdgcn_raw_buffer_store_b32(valid ? w : entry, rsrc, (int)(lane_off + level * 128u + off), 0, 0);
    }
    __device__ __forceinline__ uint32_t entry(uint32_t level) const
    {
        return __builtin_amdgcn_readfirstlane(
            __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(lane_off + level * 128u + 108u), 0, 0));
    }
    __device__ __forceinline__ uint32_t restore(uint32_t level, const wide::Lanes &) const
    {
        const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(lane_off + level * 128u + off), 0, 0);
        return valid ? x : 0u;
    }
    __device__ __forceinline__ void put_entry(uint32_t level, uint32_t e) const
    {
        if (__lane_id() == 0) __builtin_amdgcn_raw_buffer_store_b32(e, rsrc, (int)(lane_off + level * 128u + 108u), 0, 0);
    }
};

// A board's answer from the wave-wide solver (result r, completion in w on
// W_SOLVED): its bytes and status written.  st: solved, guesses (net of a
// deferred board's), -, deferred, answered -- wave-uniform.
template <class IO>
__device__ __forceinline__ void plane_wide_answer(int r, uint32_t w, int64_t pb, uint32_t bguess, int lane,
                                               const wide::Lanes &L, const IO &io, unsigned long long *__restrict__ ws,
                                               int64_t *__restrict__ defer_list, const int64_t *best,
                                               uint32_t (&st)[5])
{
    const int c0 = plane_slot_cell(lane, 0), c1 = plane_slot_cell(lane, 1);
    const uint32_t pos = (uint32_t)lane & 31u, a0 = ((uint32_t)lane >> 5) << 6;  // store: slot 0's band row
    const uint8_t *src = io.src(pb);
    uint8_t *dst = io.dst(pb);
    if (r == wide::W_SOLVED) {
        uint32_t sl[4];
        wide::value_slices(w, L, sl);
        uint32_t v0 = 0, v1 = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            v0 |= ((wide::bperm(sl[b], a0) >> pos) & 1u) << b;
            v1 |= ((wide::rdl(sl[b], 32) >> pos) & 1u) << b;
        }
        if (c0 >= 0) dst[c0] = (uint8_t)v0;
        if (c1 >= 0) dst[c1] = (uint8_t)v1;
        if (lane == 0) {
            *io.stat(pb) = SDK_SOLVED;
            if (best) __hip_atomic_fetch_min((int64_t *)&ws[WS_BEST], pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        st[0]++;
        st[4]++;
    } else if (r == wide::W_CANCELLED) {
        plane_copy_board(src, dst, lane);
        if (lane == 0) *io.stat(pb) = SDK_CANCELLED;
        st[4]++;
    } else if (r == wide::W_OVERFLOW || plane_givens_clash(src, c0, c1)) {
        // too deep for the stack, or no completion on clashing givens
        // (rules B/C unsound): the wave kernel's
        if (lane == 0) plane_defer(io.stat(pb), pb, ws, defer_list);
        st[3]++;
        st[1] -= bguess;
    } else {
        plane_copy_board(src, dst, lane);
        if (lane == 0) *io.stat(pb) = SDK_UNSOLVABLE;
        st[4]++;
    }
}

// ---- the tail pool (tail mode 2; layout in common.h)
// A drained wave's last boards go, as records in the tail record layout, to
// its XCD's pool instead of its own LDS; every wave of the XCD takes records
// from the pool, one at a time, before it exits.  Without it a wave finishes
// its 8 tail boards one after another on the wide solver while the waves
// around it have exited: the launch's end is one wave's serial tail.  One
// pool per XCD so that producer and consumer share an L2: the records and
// the donated stack lines are read back from that L2, and publishing them
// takes no L2 writeback, only the producer's own store completions (vmcnt)
// before the ready flag.
//
// Claims never retry on a shared word: a consumer takes one of the
// PUBLISHED records by decrementing `avail` (and puts the unit back if the
// count was already used up, then looks again), and only then draws its
// slot from `head` with a fetch-add -- a slot below the published count, so
// one a producer has reserved and is writing or has written.  (A
// compare-and-swap on the head, 128 waves per XCD racing, measured 66 failed
// swaps per record and a 25x slower launch.)
#ifndef SDK_PLANE_POOL_INV
#define SDK_PLANE_POOL_INV 1
#endif
// control words of an XCD's pool (one 128-byte line, re-armed per call by arm_kernel)
enum { POOL_RESERVED = 0, POOL_AVAIL = 1, POOL_HEAD = 2 };
static_assert(POOL_HEAD < PLANE_POOL_ARM_WORDS, "pool control words re-armed per call (arm_kernel)");

struct PlanePool {
    uint32_t *ctl;    // the control words (POOL_*)
    uint32_t *recs;   // PLANE_POOL_CAP records of PLANE_POOL_REC dwords
    uint32_t *flags;  // the generation of the launch that published the record
    __device__ __forceinline__ int32_t *word(int k) const { return (int32_t *)(ctl + k); }
};

__device__ __forceinline__ PlanePool plane_pool(int64_t *defer_list)
{
    // the XCD this wave runs on (HW_REG_XCC_ID, bits 0..3)
    const uint32_t x = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & (PLANE_POOL_XCDS - 1);
    uint32_t *base = (uint32_t *)(defer_list + PLANE_DEFER_CAP) + (size_t)x * PLANE_POOL_STRIDE;
    uint32_t *recs = base + PLANE_POOL_CTL;
    return {base, recs, recs + (size_t)PLANE_POOL_CAP * PLANE_POOL_REC};
}

// wave-uniform agent-scope atomic on lane 0
__device__ __forceinline__ int32_t pool_add(int32_t *p, int32_t v)
{
    int32_t r = 0;
    if (__lane_id() == 0) r = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(r);
}
__device__ __forceinline__ int32_t pool_load(const int32_t *p)
{
    int32_t r = 0;
    if (__lane_id() == 0) r = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(r);
}

// Publish `k` records already written to slots s0.. (their stores complete,
// then the ready flags, then the published count).
__device__ __forceinline__ void pool_publish(const PlanePool &pool, uint32_t s0, uint32_t k, uint32_t gen, int lane)
{
    __builtin_amdgcn_s_waitcnt(SDK_WAIT_VM0);  // the records are in this XCD's L2
    if ((uint32_t)lane < k)
        __hip_atomic_store(pool.flags + s0 + (uint32_t)lane, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(SDK_WAIT_VM0);  // flags set before the records count as published
    pool_add(pool.word(POOL_AVAIL), (int32_t)k);
}

// wide::solve's hook: ordered mode, a lower board has a completion
struct CancelHook {
    const int64_t *best;
    int64_t pb;  // the board
    __device__ __forceinline__ bool cancelled() const
    {
        return best && __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < pb;
    }
};

// Continue board pb (this lane's plane word w, its search state as the tail
// record holds it: depth, stack line, guesses so far, search mode) on the
// wave-wide solver and write its answer.  st: solved, guesses (net of
// deferred boards'), passes, deferred, answered -- wave-uniform.
template <class IO>
__device__ __forceinline__ void plane_wide_record(uint32_t w, int64_t pb, uint32_t depth, uint32_t stack_off,
                                                  uint32_t bguess, uint32_t mst, const wide::Lanes &L, int lane,
                                                  __amdgpu_buffer_rsrc_t stack_rsrc, const IO &io,
                                                  unsigned long long *__restrict__ ws, int64_t *__restrict__ defer_list,
                                                  const int64_t *best, int node_order, uint32_t mrv_after,
                                                  uint32_t (&st)[5])
{
    const WideStack stk = {stack_rsrc, stack_off, L.valid ? 4u * L.word : 108u, L.valid, lane == 48};
    wide::Stats ws_ = {0u, 0u, bguess};
    CancelHook hk = {best, pb};
    const int r = wide::solve(w, depth, stk, L, node_order, PLANE_MAX_DEPTH, ws_, hk, mst, mrv_after);
    st[2] += ws_.passes;
    st[1] += ws_.guesses;
    plane_wide_answer(r, w, pb, ws_.bguess, lane, L, io, ws, defer_list, best, st);
}

// Solve the k boards recorded in `recs` on the wave-wide solver, one after
// the other (a wave's own tail).  st as plane_wide_record's.
template <class IO>
__device__ __forceinline__ void plane_wide_tail(const uint32_t *recs, int k, int lane, __amdgpu_buffer_rsrc_t stack_rsrc,
                                             const IO &io, unsigned long long *__restrict__ ws,
                                             int64_t *__restrict__ defer_list, const int64_t *best, int node_order,
                                             uint32_t mrv_after, uint32_t (&st)[5])
{
    const wide::Lanes L = wide::lanes();
    for (int s = 0; s < k; ++s) {
        const uint32_t *rec = recs + PLANE_TAIL_REC * s;
        uint32_t w = rec[L.valid ? L.word : 0u];
        w = L.valid ? w : 0u;
        const int64_t pb = ((int64_t)__builtin_amdgcn_readfirstlane(rec[28]) << 32) |
                           (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane(rec[27]);
        plane_wide_record(w, pb, __builtin_amdgcn_readfirstlane(rec[29]), __builtin_amdgcn_readfirstlane(rec[30]),
                          __builtin_amdgcn_readfirstlane(rec[31]), __builtin_amdgcn_readfirstlane(rec[32]), L, lane,
                          stack_rsrc, io, ws, defer_list, best, node_order, mrv_after, st);
    }
}

// Take records from the pool until none is published (wave-uniform).  A
// taken slot has a producer that reserved it and writes it without waiting
// on anything, so the flag wait is short (a flag holds the launch generation
// `gen`, so a flag an earlier launch left never reads as set).  It is bounded
// all the same (`polls` polls, ~1 s by default): a wave that gives up sets
// SDK_ERR_POOL_WAIT in the workspace -- that record's board is not answered,
// and sdk_verify_workspace turns the word into a failed call -- and leaves
// the pool.  st as plane_wide_record's.
template <class IO>
__device__ __forceinline__ void plane_pool_drain(const PlanePool &pool, int lane, __amdgpu_buffer_rsrc_t stack_rsrc,
                                              const IO &io, unsigned long long *__restrict__ ws,
                                              int64_t *__restrict__ defer_list, const int64_t *best, int node_order,
                                              uint32_t mrv_after, uint32_t gen, uint32_t polls, uint32_t (&st)[5])
{
#if SDK_PLANE_STAMPS
    // diagnostic: claims, backed-out claims, flag polls; cycles claiming, waiting, solving (ws words 24..29)
    uint64_t d_ok = 0, d_fail = 0, d_poll = 0, c_claim = 0, c_wait = 0, c_solve = 0;
    uint64_t d_t = __builtin_amdgcn_s_memtime();
#endif
    const wide::Lanes L = wide::lanes();
    while (pool_load(pool.word(POOL_AVAIL)) > 0) {
        // take one of the PUBLISHED records: decrement `avail` (putting the
        // unit back if it was already used up), then draw the slot
        uint32_t h = 0;
        int32_t a = 0;
        if (lane == 0) {
            a = __hip_atomic_fetch_add(pool.word(POOL_AVAIL), -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a > 0)
                h = __hip_atomic_fetch_add(pool.ctl + POOL_HEAD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                __hip_atomic_fetch_add(pool.word(POOL_AVAIL), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (__builtin_amdgcn_readfirstlane(a) <= 0) {
#if SDK_PLANE_STAMPS
            d_fail++;
#endif
            continue;  // another wave took the last one: look again
        }
        h = __builtin_amdgcn_readfirstlane(h);
#if SDK_PLANE_STAMPS
        d_ok++;
        {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            c_claim += t1 - d_t;
            d_t = t1;
        }
#endif
        bool ready = false;
        for (uint32_t tries = 0; tries < polls; ++tries) {
            uint32_t f = 0;
            if (lane == 0) f = __hip_atomic_load(pool.flags + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ready = __builtin_amdgcn_readfirstlane(f) == gen;
#if SDK_PLANE_STAMPS
            d_poll++;
#endif
            if (ready) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ready) {
            // loud, never silent: the host's sdk_verify_workspace raises on it
            if (lane == 0) {
                atomicOr(&ws[WS_ERROR], (unsigned long long)SDK_ERR_POOL_WAIT);
                __hip_atomic_store(&ws[WS_ERR_SLOT], (unsigned long long)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
        }
#if SDK_PLANE_STAMPS
        {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            c_wait += t1 - d_t;
            d_t = t1;
        }
#endif
#if SDK_PLANE_POOL_INV == 2
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#elif SDK_PLANE_POOL_INV == 1
        asm volatile("buffer_inv sc0" ::: "memory");  // this CU's L1 only
#endif
        const uint32_t *rec = pool.recs + (size_t)h * PLANE_POOL_REC;
        const uint32_t rw = lane < 36 ? __hip_atomic_load(rec + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        uint32_t w = __builtin_amdgcn_ds_bpermute((int)(4u * (L.valid ? L.word : 0u)), (int)rw);
        w = L.valid ? w : 0u;
        const int64_t pb = ((int64_t)rdlane(rw, 28) << 32) | (int64_t)rdlane(rw, 27);
        plane_wide_record(w, pb, rdlane(rw, 29), rdlane(rw, 30), rdlane(rw, 31), rdlane(rw, 32), L, lane, stack_rsrc,
                          io, ws, defer_list, best, node_order, mrv_after, st);
#if SDK_PLANE_STAMPS
        {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            c_solve += t1 - d_t;
            d_t = t1;
        }
#endif
    }
#if SDK_PLANE_STAMPS
    c_claim += __builtin_amdgcn_s_memtime() - d_t;
    if (lane == 0) {
        atomicAdd(&ws[24], (unsigned long long)d_ok);
        atomicAdd(&ws[25], (unsigned long long)d_fail);
        atomicAdd(&ws[26], (unsigned long long)d_poll);
        atomicAdd(&ws[27], (unsigned long long)c_claim);
        atomicAdd(&ws[28], (unsigned long long)c_wait);
        atomicAdd(&ws[29], (unsigned long long)c_solve);
    }
#endif
}

// sum of a per-lane counter over the wave (all lanes active)
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// lane states; the two "original" states store the input board back
enum { PL_IDLE = 0, PL_ACTIVE = 1, PL_SOLVED = 2, PL_UNSOLVABLE = 3, PL_CANCELLED = 4 };

__device__ __forceinline__ unsigned long long rdlane64(unsigned long long v, int l)
{
    return ((unsigned long long)rdlane((uint32_t)(v >> 32), l) << 32) | rdlane((uint32_t)v, l);
}


#ifndef SDK_PLANE_WAVES_PER_EU
#define SDK_PLANE_WAVES_PER_EU 4
#endif
// The kernel body over either board I/O (plane_kernel: one batch;
// plane_kernel_multi: several, unordered).
template <class IO>
__device__ __forceinline__ void plane_body(const IO &io, unsigned long long *__restrict__ ws,
                                           uint32_t *__restrict__ stack, int64_t *__restrict__ defer_list,
                                           int ordered, int order, int refill, int tail, int tail_mode, int chunk,
                                           uint32_t mrv_after, uint32_t pool_polls)
{
    const int64_t n = io.total();  // boards of the launch (virtual indices 0..n-1)
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&ws[WS_ASSIGNED], (unsigned long long)n);  // sdk_verify_workspace
    __shared__ __attribute__((aligned(16))) uint32_t stage_lds[PLANE_THREADS / 64][PLANE_STAGE_DWORDS];
    __shared__ __attribute__((aligned(16))) uint32_t outbox_lds[PLANE_THREADS / 64][PLANE_OUTBOX * PLANE_OB_WORDS];
#if SDK_PLANE_LDS_PAD
    __shared__ uint32_t lds_pad[PLANE_THREADS / 64][SDK_PLANE_LDS_PAD];  // A/B: occupancy by LDS
    asm volatile("" ::"v"((uint32_t)(uintptr_t)&lds_pad[0][0]));
#endif
    uint32_t *stage = stage_lds[threadIdx.x >> 6];
    uint32_t *outbox = outbox_lds[threadIdx.x >> 6];
    uint32_t ob_count = 0;  // boards waiting in the outbox (wave-uniform)
    if ((threadIdx.x & 63) == 0) stage[PLANE_STAGE_DWORDS - 1] = 0u;  // the zero byte
    const int64_t nt = (int64_t)gridDim.x * PLANE_THREADS;
    const int64_t g = (int64_t)blockIdx.x * PLANE_THREADS + threadIdx.x;
    PlaneStack stk = {
        __builtin_amdgcn_make_buffer_rsrc(stack, 0, (int)(nt * PLANE_MAX_DEPTH * 128), 0x00020000),
        (uint32_t)g * (uint32_t)(PLANE_MAX_DEPTH * 128)};
    const int64_t *best = ordered ? (const int64_t *)&ws[WS_BEST] : nullptr;
    const int node_order = order == SDK_ORDER_NODE;
    const int lane = threadIdx.x & 63;

    plane::Board B;
    int64_t p = -1;       // this lane's board
    int state = PL_IDLE;
    uint32_t depth = 0;
    // per-lane statistics (each lane counts its own boards' events; summed
    // over the wave at exit)
    uint32_t fin = 0, solved = 0, guesses = 0, passes = 0, deferred = 0;
    uint32_t bguess = 0;  // guesses on the current board (dropped if it is handed off)
    uint32_t mst = 0;     // the board's search mode and pass count (plane::search_step)
    bool drained = false;  // the queue is empty and this wave's reservoir too
    // Board hand-out.  The first nt boards go out statically, 64 consecutive
    // ones per wave; the rest through the queue head (board nt + head).  A
    // wave claims a CHUNK of boards at a time into its reservoir [res_lo,
    // res_hi) and refills from it: one queue atomic per chunk instead of per
    // refill (the head is one device-scope atomic for 4096 waves).  Chunks
    // shrink towards the end of the batch (guided: remaining / (SDK_PLANE_GUIDE waves)).
    int64_t res_lo = 0, res_hi = 0;
    int64_t rec_base = 0;  // virtual index of chunk record 0
    int64_t rec_id = 0;    // its board id
    int64_t seg_hi = 0;    // [res_lo, seg_hi) converted (one batch segment), [seg_hi, res_hi) claimed only
    bool queue_out = false;
    const int64_t nwaves = (int64_t)gridDim.x * (PLANE_THREADS / 64);
    uint64_t tail_act = 0;  // lanes whose boards the wave solver restarts after the loop
#if SDK_PLANE_STAMPS
    const uint64_t st_t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t st_t1 = 0;
    uint32_t st_after = 0, st_iters = 0;
    // one lane's (lane 16's) passes and the active lanes summed over them,
    // search-step cycles, iterations where some lane guessed / backtracked
    uint64_t st_piters = 0, st_lanes = 0, st_step = 0, st_push = 0, st_pop = 0;
    // shader-clock cycles spent in the pass step / the store + refill block /
    // the tail restarts (s_memtime at wave-uniform points)
    uint64_t st_pass = 0, st_io = 0, st_tail = 0, st_tb = 0;
    uint64_t st_atom = 0, st_dep = 0;  // parts of st_io: queue atomic, per-board deposit
    uint64_t st_store = 0;                          // part of st_io: storing finished boards
    uint64_t st_claims = 0;                         // queue claims: count | last size << 32
#endif

    // Start-up: the wave's first 64 boards arrive as staged spans (one per
    // batch segment of the window, at most PLANE_START_SPAN boards each);
    // each lane then converts its own board (plane::load_words), all at once.
    {
        const int64_t v0 = g - lane;
        queue_out = nt >= n;
        drained = queue_out;
        const int64_t kk = v0 < n ? (n - v0 < 64 ? n - v0 : 64) : 0;
        for (int64_t s0 = 0; s0 < kk;) {
            const int64_t sv = v0 + s0, cap = sv + PLANE_START_SPAN < v0 + kk ? sv + PLANE_START_SPAN : v0 + kk;
            const int64_t se = io.seg_end(sv, cap);
            const int cnt = (int)(se - sv);
            const uint32_t sh = plane_stage_span(io.seg_in(sv), io.seg_n(sv), io.seg_local(sv), cnt, stage, lane);
            const int r = lane - (int)s0;
            if (r >= 0 && r < cnt) {
                const int64_t q = io.id(sv) + r;
                uint32_t x[21];
                plane_stage_words(stage, sh + 81u * (uint32_t)r, x);
                bool clash;  // tested lazily (see the unsolvable store above)
                const bool ok = plane::load_words(B, x, clash);
                const bool cancel = ok && best && __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < q;
                if (ok && !cancel) {
                    p = q;
                    depth = 0;
                    bguess = 0;
                    mst = 0;
                    state = PL_ACTIVE;
                } else {
                    const uint8_t *src = io.src(q);
                    uint8_t *dst = io.dst(q);
                    for (int i = 0; i < 81; ++i) dst[i] = src[i];  // raw input back
                    *io.stat(q) = ok ? SDK_CANCELLED : SDK_INVALID;
                    fin++;  // (a board counts as finished when its answer is written)
                }
            }
            s0 = se - v0;
            // the next span's DMA overwrites the stage: every lane has its words
            if (s0 < kk) wave_lds_sync();
        }
    }

    for (;;) {
#if SDK_PLANE_STAMPS
        const uint64_t st_ta = __builtin_amdgcn_s_memtime();
        if (st_tb) st_pass += st_ta - st_tb;
        st_iters++;
        if (drained) {
            if (!st_t1) st_t1 = __builtin_amdgcn_s_memrealtime();
            st_after++;
        }
#endif
        const uint64_t active = __builtin_amdgcn_ballot_w64(state == PL_ACTIVE);
        if (__builtin_popcountll(~active) >= refill || active == 0) {
            const int c0 = plane_slot_cell(lane, 0), c1 = plane_slot_cell(lane, 1);
            // ---- store finished boards, through the wave's LDS outbox: every
            // solved lane appends its board's value bit-slices (12 words) and
            // index; once 64 are waiting, each lane turns one of them into
            // bytes and writes it as dwords (plane_flush_outbox).  No per-board
            // serial loop: ~8 lane-parallel VALU per board instead of ~60
            // wave instructions of per-board bookkeeping.
#if SDK_PLANE_STAMPS
            const uint64_t st_s0 = __builtin_amdgcn_s_memtime();
#endif
            uint64_t m = __builtin_amdgcn_ballot_w64(state == PL_SOLVED);
            solved += state == PL_SOLVED;
            fin += state == PL_SOLVED;
            if (m) {
                const uint32_t ns = (uint32_t)__builtin_popcountll(m);
                if (ob_count + ns > (uint32_t)PLANE_OUTBOX) {
                    plane_flush_outbox(outbox, ob_count, lane, io);
                    ob_count = 0;
                }
                if (state == PL_SOLVED) {
                    sdk_v4u *rec = (sdk_v4u *)(outbox + PLANE_OB_WORDS * (ob_count + lanes_below(m)));
                    uint32_t V[4][3];
#pragma unroll
                    for (int b = 0; b < 3; ++b) {
                        V[0][b] = plane::or3(plane::or3(B.P[0][b], B.P[2][b], B.P[4][b]), B.P[6][b], B.P[8][b]);
                        V[1][b] = plane::or3(B.P[1][b], B.P[2][b], B.P[5][b] | B.P[6][b]);
                        V[2][b] = plane::or3(B.P[3][b], B.P[4][b], B.P[5][b] | B.P[6][b]);
                        V[3][b] = B.P[7][b] | B.P[8][b];
                    }
                    rec[0] = (sdk_v4u){V[0][0], V[0][1], V[0][2], V[1][0]};
                    rec[1] = (sdk_v4u){V[1][1], V[1][2], V[2][0], V[2][1]};
                    rec[2] = (sdk_v4u){V[2][2], V[3][0], V[3][1], V[3][2]};
                    rec[3] = (sdk_v4u){(uint32_t)p, (uint32_t)(p >> 32), 0u, 0u};
                    *io.stat(p) = SDK_SOLVED;  // every solved lane its own, one store
                }
                ob_count += ns;
            }
            // ---- unsolvable / cancelled: the input board back
            m = __builtin_amdgcn_ballot_w64(state >= PL_UNSOLVABLE);
            while (m) {
                const int i = __builtin_ctzll(m);
                m &= m - 1;
                const int64_t pi = ((int64_t)rdlane((uint32_t)(p >> 32), i) << 32) | rdlane((uint32_t)p, i);
                const bool cancelled = rdlane((uint32_t)state, i) == PL_CANCELLED;
                if (!cancelled && plane_givens_clash(io.src(pi), c0, c1)) {
                    // rules B/C are unsound on givens that repeat a digit in a
                    // unit: "no completion" is the packed kernel's call.  (A
                    // SOLVED result needs every unit to hold every digit, so
                    // such givens never reach the store above.)
                    if (lane == i) {
                        plane_defer(io.stat(pi), pi, ws, defer_list);
                        deferred++;
                        guesses -= bguess;
                    }
                    continue;
                }
                plane_copy_board(io.src(pi), io.dst(pi), lane);
                if (lane == 0) {
                    *io.stat(pi) = cancelled ? SDK_CANCELLED : SDK_UNSOLVABLE;
                    fin++;
                }
            }
            if (state != PL_ACTIVE) state = PL_IDLE;
            // ---- refill the free lanes: one queue add per wave; the boards'
            // bytes come into LDS as one span (plane_stage_span); then, one
            // board at a time, six ballots over the wave give its value
            // bit-slices (slot 0: four, one per value bit; slot 1: two, lanes
            // 0-31 and 32-63 testing different bits of the same band-2
            // cell) and v_writelane drops the 12 slice words into the
            // board's lane, into plane words the idle lane does not use;
            // finally every loaded lane turns its slices into planes at once
#if SDK_PLANE_STAMPS
            st_store += __builtin_amdgcn_s_memtime() - st_s0;
#endif
            if (!drained) {
                const uint64_t idle = ~active;
                const int k = __builtin_popcountll(idle);
                unsigned long long base = 0;
                const int leader = __builtin_ctzll(idle);
#if SDK_PLANE_STAMPS
                const uint64_t st_r0 = __builtin_amdgcn_s_memtime();
#endif
                if (res_lo == res_hi && !queue_out) {
                    // guided chunk: this wave's share of what is left (as of its
                    // own last claim), at least k.  Sizing by a fresh view of
                    // the head (an agent-scope load of it, or a per-XCD hint
                    // in L2) measured slower: more claims, each a span DMA and
                    // a conversion, and all waves then drain at once
                    const int64_t seen = res_hi > nt ? res_hi : nt;
                    int64_t c = chunk > 0 ? (n - seen) / (SDK_PLANE_GUIDE * nwaves) : 0;
                    c = c > chunk ? chunk : c;
                    // a chunk is staged and converted in one go: at most 64 records
                    // fit the staging area (the host also rejects chunk > 64)
                    c = c < k ? k : c;
                    c = c > PLANE_CHUNK_MAX ? PLANE_CHUNK_MAX : c;  // (then some idle lanes wait a pass)
                    if (lane == leader) base = atomicAdd(&ws[WS_QUEUE], (unsigned long long)c);
#if SDK_PLANE_STAMPS
                    st_claims = ((st_claims & 0xFFFFFFFFull) + 1) | ((uint64_t)c << 32);  // count, last size
#endif
                    base = __shfl(base, leader);
                    res_lo = nt + (int64_t)base;
                    res_hi = res_lo + c < n ? res_lo + c : n;
                    if (res_lo > n) res_lo = n;
                    queue_out = res_lo + c >= n;
                    if constexpr (!IO::multi) {
                        // the whole chunk staged and converted once (chunk records)
                        const int cc = __builtin_amdgcn_readfirstlane((int)(res_hi - res_lo));
                        rec_base = res_lo;
                        if (cc) {
                            const uint32_t sh = plane_stage_span(io.in, n, res_lo, cc, stage, lane);
                            plane_convert_chunk(stage, sh, cc, lane);
                        }
                    }
                    seg_hi = IO::multi ? res_lo : res_hi;  // (multi: nothing converted yet)
                }
                if (IO::multi && res_lo == seg_hi && res_lo < res_hi) {
                    // the claimed chunk staged and converted once (chunk
                    // records), a batch segment at a time (one for one batch)
                    seg_hi = io.seg_end(res_lo, res_hi);
                    const int cc = __builtin_amdgcn_readfirstlane((int)(seg_hi - res_lo));
                    rec_base = res_lo;
                    rec_id = io.id(res_lo);
                    const uint32_t sh = plane_stage_span(io.seg_in(res_lo), io.seg_n(res_lo), io.seg_local(res_lo), cc,
                                                         stage, lane);
                    plane_convert_chunk(stage, sh, cc, lane);
                }
                base = (unsigned long long)res_lo;
                // (wave-uniform: readfirstlane keeps the deposit loop a scalar loop)
                const int64_t avail = (IO::multi ? seg_hi : res_hi) - res_lo;
                const int kk = __builtin_amdgcn_readfirstlane((int)(avail < k ? avail : k));
                res_lo += kk;
                drained = queue_out && res_lo == res_hi;
#if SDK_PLANE_STAMPS
                const uint64_t st_r1 = __builtin_amdgcn_s_memtime();
                st_atom += st_r1 - st_r0;
#endif
                if (kk) {
#if SDK_PLANE_STAMPS
                    const uint64_t st_r2 = __builtin_amdgcn_s_memtime();
#endif
                    // idle lane of rank i < kk takes record base - rec_base + i
                    const uint32_t rank = lanes_below(idle);
                    const bool take = ((idle >> lane) & 1u) && rank < (uint32_t)kk;
                    const uint64_t loaded = __builtin_amdgcn_ballot_w64(take);
                    bool bad = false;
                    if (take) {
                        const uint32_t *rec = stage + PLANE_REC * ((uint32_t)(base - (unsigned long long)rec_base) + rank);
                        uint32_t V[4][3], given[3];
#pragma unroll
                        for (int s = 0; s < 4; ++s)
#pragma unroll
                            for (int b = 0; b < 3; ++b) V[s][b] = rec[3 * s + b];
                        bad = rec[12] != 0u;
                        p = (IO::multi ? rec_id + ((int64_t)base - rec_base) : (int64_t)base) + (int64_t)rank;
                        depth = 0;
                        bguess = 0;
                        mst = 0;
                        if (!bad && !(best && __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p)) {
                            plane::planes_from_slices(B, V, given);
                            state = PL_ACTIVE;
                        } else {
                            state = PL_CANCELLED;  // (bad: SDK_INVALID below)
                        }
                    }
                    const uint64_t badm = __builtin_amdgcn_ballot_w64(bad);
                    // boards with a byte > 9 (or cancelled): the raw input back
                    uint64_t r = loaded & __builtin_amdgcn_ballot_w64(state != PL_ACTIVE);
                    while (r) {
                        const int i = __builtin_ctzll(r);
                        r &= r - 1;
                        const int64_t q = (IO::multi ? rec_id + ((int64_t)base - rec_base) : (int64_t)base) +
                                          (int64_t)__builtin_popcountll(loaded & ((1ull << i) - 1));
                        plane_copy_board(io.src(q), io.dst(q), lane);
                        if (lane == 0) {
                            *io.stat(q) = ((badm >> i) & 1u) ? SDK_INVALID : SDK_CANCELLED;
                            fin++;
                        }
                    }
                    if (state == PL_CANCELLED) state = PL_IDLE;
#if SDK_PLANE_STAMPS
                    st_dep += __builtin_amdgcn_s_memtime() - st_r2;
#endif
                }
            }
            // ---- tail: the queue is empty and the wave is down to a few
            // boards.  A pass costs the whole wave whatever its active
            // lanes, so the wave would idle on its slowest board for tens of
            // passes; instead it hands them to the wave-wide solver
            // (plane_wide.h: the search continues, ~200 instructions per
            // pass) -- through its XCD's pool (tail mode 2), or one after
            // the other itself (1) -- and exits.
            if (drained && tail > 0) {
                const uint64_t act = __builtin_amdgcn_ballot_w64(state == PL_ACTIVE);
                if (act && __builtin_popcountll(act) <= tail) {
                    tail_act = act;
                    break;
                }
            }
            if (drained && __builtin_amdgcn_ballot_w64(state != PL_IDLE) == 0) break;  // nothing left here
        }
#if SDK_PLANE_STAMPS
        st_tb = __builtin_amdgcn_s_memtime();
        st_io += st_tb - st_ta;
#endif
        if (state != PL_ACTIVE) continue;

        // ---- one pass of this lane's board
        passes++;
#if SDK_PLANE_STAMPS
        st_lanes += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(true));
        st_piters++;
#endif
        uint32_t und[3];
        const int r = plane::pass(B, und);
        if (r == plane::STUCK && best && __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p) {
            state = PL_CANCELLED;  // ordered mode: a lower board is solved
            continue;
        }
        // guess / backtrack / search-mode switch (plane::search_step: the
        // lane solver's own step, checked on the host against the oracle)
        const uint32_t gb = bguess;
#if SDK_PLANE_STAMPS
        const uint32_t st_d0 = depth;
        const uint64_t st_s0 = __builtin_amdgcn_s_memtime();
#endif
        const int s = plane::search_step(B, und, r, depth, mst, stk, node_order, PLANE_MAX_DEPTH, mrv_after, bguess);
#if SDK_PLANE_STAMPS
        st_step += __builtin_amdgcn_s_memtime() - st_s0;
        st_push += wany(bguess != gb) ? 1u : 0u;
        st_pop += wany(depth < st_d0) ? 1u : 0u;
#endif
        guesses += bguess - gb;
        if (s == plane::S_SOLVED) {
            state = PL_SOLVED;
            if (best)
                __hip_atomic_fetch_min((int64_t *)&ws[WS_BEST], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (s == plane::S_NONE) {
            state = PL_UNSOLVABLE;
        } else if (s == plane::S_DEEP) {
            plane_defer(io.stat(p), p, ws, defer_list);  // too deep for the stack: the wave kernel's
            deferred++;
            guesses -= bguess;
            state = PL_IDLE;
        }
    }
    if (ob_count) plane_flush_outbox(outbox, ob_count, lane, io);
#if SDK_PLANE_STAMPS
    const uint64_t st_tt = __builtin_amdgcn_s_memtime();
    const uint64_t st_t3 = __builtin_amdgcn_s_memrealtime();  // the lane loop ended
    const uint32_t st_tailn = (uint32_t)__builtin_popcountll(tail_act);
    uint32_t st_tailp = 0;
#endif
    // tail mode 2: the tail boards go to this XCD's pool, which every wave
    // of the XCD drains before it exits (plane_pool_drain)
    const PlanePool pool = plane_pool(defer_list);
    // this launch's generation (arm_kernel, an earlier launch on the stream)
    const uint32_t gen = tail_mode >= 2 ? __builtin_amdgcn_readfirstlane((uint32_t)ws[WS_GEN]) : 0u;
    if (tail_act) {
        // ---- wave-wide tail: the lanes' boards go to LDS records (27 plane
        // words, index, depth, stack line, guesses; stride 33 dwords, so the
        // lanes' writes and a record's reads are conflict-free) and the wave
        // continues each search in turn on the wide solver
        __builtin_amdgcn_s_waitcnt(SDK_WAIT_VM0);  // the lanes' stack pushes have landed
        const uint32_t k = (uint32_t)__builtin_popcountll(tail_act);
        const uint32_t rank = lanes_below(tail_act);
        uint32_t fit = 0, slot0 = 0;
        if (tail_mode >= 2) {
            slot0 = (uint32_t)pool_add(pool.word(POOL_RESERVED), (int32_t)k);
            fit = slot0 >= PLANE_POOL_CAP ? 0u : (PLANE_POOL_CAP - slot0 < k ? PLANE_POOL_CAP - slot0 : k);
        }
        if ((tail_act >> lane) & 1u) {
            uint32_t v[PLANE_POOL_REC];
#pragma unroll
            for (int w = 0; w < 27; ++w) v[w] = B.P[w / 3][w % 3];
            v[27] = (uint32_t)p;
            v[28] = (uint32_t)(p >> 32);
            v[29] = depth;
            v[30] = stk.lane_off;
            v[31] = bguess;
            v[32] = mst;
            v[33] = v[34] = v[35] = 0u;
            if (rank < fit) {
                sdk_v4u *q = (sdk_v4u *)(pool.recs + (size_t)(slot0 + rank) * PLANE_POOL_REC);
#pragma unroll
                for (int i = 0; i < PLANE_POOL_REC / 4; ++i)
                    q[i] = sdk_v4u{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
            } else {
                uint32_t *rec = stage + PLANE_TAIL_REC * (rank - fit);
#pragma unroll
                for (int w = 0; w < PLANE_TAIL_REC; ++w) rec[w] = v[w];
            }
        }
        if (fit) pool_publish(pool, slot0, fit, gen, lane);
        wave_lds_sync();
        uint32_t wst[5] = {0u, 0u, 0u, 0u, 0u};
        if (k > fit)
            plane_wide_tail(stage, (int)(k - fit), lane, stk.rsrc, io, ws, defer_list, best, node_order, mrv_after,
                            wst);
#if SDK_PLANE_STAMPS
        st_tailp = wst[2];
#endif
        if (lane == 0) {
            solved += wst[0];
            guesses += wst[1];
            passes += wst[2];
            fin += wst[4];
            deferred += wst[3];
        }
    }
    if (tail_mode >= 2) {
        uint32_t wst[5] = {0u, 0u, 0u, 0u, 0u};
        plane_pool_drain(pool, lane, stk.rsrc, io, ws, defer_list, best, node_order, mrv_after, gen, pool_polls, wst);
        if (lane == 0) {
            solved += wst[0];
            guesses += wst[1];
            passes += wst[2];
            fin += wst[4];
            deferred += wst[3];
        }
    }
#if SDK_PLANE_STAMPS
    {
        st_tail = __builtin_amdgcn_s_memtime() - st_tt;
        int64_t *st = defer_list + (PLANE_DEFER_CAP / 2) + 32 * (g >> 6);
        const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) st[0] = (int64_t)st_t0;
        if (lane == 1) st[1] = (int64_t)(st_t1 ? st_t1 : t2);
        if (lane == 2) st[2] = (int64_t)t2;
        if (lane == 3) st[3] = (int64_t)st_after;
        if (lane == 4) st[4] = (int64_t)st_pass;
        if (lane == 5) st[5] = (int64_t)st_io;
        if (lane == 6) st[6] = (int64_t)st_tail;
        if (lane == 7) st[7] = (int64_t)st_iters;
        if (lane == 8) st[8] = (int64_t)st_atom;
        if (lane == 9) st[9] = 0;
        if (lane == 10) st[10] = (int64_t)st_dep;
        if (lane == 11) st[11] = (int64_t)st_store;
        if (lane == 12) st[12] = (int64_t)st_t3;
        if (lane == 13) st[13] = (int64_t)st_tailn;
        if (lane == 14) st[14] = (int64_t)st_tailp;
        if (lane == 15) st[15] = (int64_t)st_claims;
        if (lane == 16) st[16] = (int64_t)st_piters;
        if (lane == 17) st[17] = (int64_t)st_lanes;
        if (lane == 18) st[18] = (int64_t)st_step;
        if (lane == 19) st[19] = (int64_t)st_push;
        if (lane == 20) st[20] = (int64_t)st_pop;
    }
#endif
    // per-wave statistics: the lanes' counts summed, one atomic per counter and wave
    fin = wave_sum(fin);
    solved = wave_sum(solved);
    guesses = wave_sum(guesses);
    passes = wave_sum(passes);
    deferred = wave_sum(deferred);
    if (lane == 0 && deferred) atomicAdd(&ws[WS_DEFERRED], (unsigned long long)deferred);
    if (lane == 0 && (fin | deferred | passes)) {
        // (sign-extended: a wave that took deferred boards from the pool can
        // end with a negative count of its own)
        atomicAdd(&ws[WS_FINISHED], (unsigned long long)(long long)(int32_t)fin);
        atomicAdd(&ws[WS_SOLVED], (unsigned long long)solved);
        atomicAdd(&ws[WS_GUESSES], (unsigned long long)(long long)(int32_t)guesses);
        atomicAdd(&ws[WS_SWEEPS], (unsigned long long)passes);
    }
}

__global__ __launch_bounds__(PLANE_THREADS, SDK_PLANE_WAVES_PER_EU) void plane_kernel(
    const uint8_t *__restrict__ puzzles, uint8_t *__restrict__ sols, int32_t *__restrict__ status, int64_t n,
    unsigned long long *__restrict__ ws, uint32_t *__restrict__ stack, int64_t *__restrict__ defer_list, int ordered,
    int order, int refill, int tail, int tail_mode, int chunk, uint32_t mrv_after, uint32_t pool_polls)
{
    const PlaneIO1 io = {puzzles, sols, status, n};
    plane_body(io, ws, stack, defer_list, ordered, order, refill, tail, tail_mode, chunk, mrv_after, pool_polls);
}

// several batches, one queue over them (sdk_solve_batches; unordered)
__global__ __launch_bounds__(PLANE_THREADS, SDK_PLANE_WAVES_PER_EU) void plane_kernel_multi(
    const PlaneBatches bs, unsigned long long *__restrict__ ws, uint32_t *__restrict__ stack,
    int64_t *__restrict__ defer_list, int order, int refill, int tail, int tail_mode, int chunk, uint32_t mrv_after,
    uint32_t pool_polls)
{
    const PlaneIOn io = {bs};
    plane_body(io, ws, stack, defer_list, 0, order, refill, tail, tail_mode, chunk, mrv_after, pool_polls);
}

#endif  // SDK_PLANE_KERNEL_H
