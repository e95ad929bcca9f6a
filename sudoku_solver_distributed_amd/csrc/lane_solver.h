// lane_solver.h -- one board per LANE: the whole walk in registers.
//
// Same contract as the wave-per-board kernel (sudoku_kernels.hip): the first
// completion of the reference walk `order` (gen.py:6-28 / node.py:62-74),
// found with sound propagation + branching on the walk's next cell, digits
// ascending.  Differences in execution:
//   * the 27 unit masks live in 27 registers and every cell index is a
//     compile-time constant (fully unrolled 81-cell passes), so propagation
//     is Gauss-Seidel: a placement is seen by every later cell of the same
//     pass, with no cross-lane traffic and no LDS;
//   * a guess saves the 81 nibbles of the board (11 words) plus the branch
//     entry to a per-lane stack (scratch memory on the GPU); a backtrack
//     restores them and rebuilds the masks.
// Plain C++ usable on host and device: tests compile it for the CPU and
// check it against the oracle before the GPU runs it.
#ifndef SDK_LANE_SOLVER_H
#define SDK_LANE_SOLVER_H

#include <stdint.h>

#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
// Pin an accumulator (dead flags, placement counts) at the end of each unit
// / cell: left alone, LLVM re-associates the OR / ADD chain of a whole
// unrolled pass into a tree and keeps every term live to the end (~25 VGPRs
// per unit).
#define LS_PIN(x) asm volatile("" : "+v"(x))
#define LS_SCHED_FENCE() ((void)0)
#else
#define LS_PIN(x) ((void)0)
#define LS_SCHED_FENCE() ((void)0)
#endif

#ifdef __HIPCC__
#define LS_FN __host__ __device__ __forceinline__
#define LS_FN_STATIC __host__ __device__ __forceinline__ static
#else
#define LS_FN inline
#define LS_FN_STATIC static inline
#endif

namespace lane {

enum { DEAD = 1, SOLVED = 2, OPEN = 0 };

LS_FN int popc(uint32_t x) { return __builtin_popcount(x); }
LS_FN int ctz32(uint32_t x) { return __builtin_ctz(x); }
LS_FN int clz64(uint64_t x) { return __builtin_clzll(x); }
LS_FN int ctz64(uint64_t x) { return __builtin_ctzll(x); }

// compile-time geometry
LS_FN constexpr int ROW(int i) { return i / 9; }
LS_FN constexpr int COL(int i) { return i % 9; }
LS_FN constexpr int BOX(int i) { return (i / 27) * 3 + (i % 9) / 3; }
// cell k (0..8) of unit u (rows 0-8, columns 9-17, boxes 18-26)
LS_FN constexpr int UCELL(int u, int k)
{
    return u < 9 ? u * 9 + k
         : u < 18 ? k * 9 + (u - 9)
                  : ((u - 18) / 3 * 3 + k / 3) * 9 + ((u - 18) % 3) * 3 + k % 3;
}

struct Board {
    uint32_t V[11];  // cell i: nibble i%8 of V[i/8] (0 = empty)
    uint32_t E[3];   // cell i: bit i%32 of E[i/32] set = empty
    uint32_t U[27];  // unit masks: bit d-1 = digit d used
    uint32_t bad;    // units whose GIVENS clash (hidden-single rules off)
};

LS_FN uint32_t getv(const Board &b, int i) { return (b.V[i >> 3] >> ((i & 7) * 4)) & 15u; }

// Make every later computation consume the board as it stands here: one
// empty asm per state word (no instruction is emitted).  Placed between the
// units / cell groups of an unrolled pass it stops the optimiser from hoisting
// a whole pass worth of independent work and running out of registers.
LS_FN void pin_board(Board &b)
{
#pragma unroll
    for (int w = 0; w < 11; ++w) LS_PIN(b.V[w]);
#pragma unroll
    for (int w = 0; w < 3; ++w) LS_PIN(b.E[w]);
#pragma unroll
    for (int u = 0; u < 27; ++u) LS_PIN(b.U[u]);
    LS_PIN(b.bad);  // else 27 loop-invariant "unit ok" masks get hoisted and stay live
}

// Rebuild the unit masks U from V, one unit at a time (a fence between
// units keeps the unrolled work from being interleaved into a register
// blow-up).  Returns the units in which two filled cells share a digit (at
// load time: the clashing givens).
template <int U_>
LS_FN void unit_from_v(Board &b, uint32_t &clash)
{
    uint32_t once = 0, twice = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const uint32_t v = getv(b, UCELL(U_, k));
        const uint32_t bit = (1u << v) >> 1;  // 0 for an empty cell
        twice |= once & bit;
        once |= bit;
    }
    b.U[U_] = once;
    clash |= twice ? 1u << U_ : 0u;
    LS_PIN(clash);
}

template <int U_>
struct UnitsFromV {
    LS_FN_STATIC void run(Board &b, uint32_t &clash)
    {
        unit_from_v<U_>(b, clash);
        pin_board(b);
        UnitsFromV<U_ + 1>::run(b, clash);
    }
};
template <>
struct UnitsFromV<27> {
    LS_FN_STATIC void run(Board &, uint32_t &) {}
};

LS_FN uint32_t rebuild_units(Board &b)
{
    uint32_t clash = 0;
    UnitsFromV<0>::run(b, clash);
    return clash;
}

// place digit bit `m` (one bit) at compile-time cell I
template <int I>
LS_FN void place_c(Board &b, uint32_t m)
{
    b.U[ROW(I)] |= m;
    b.U[9 + COL(I)] |= m;
    b.U[18 + BOX(I)] |= m;
    b.E[I >> 5] &= ~(m ? 1u << (I & 31) : 0u);
    b.V[I >> 3] |= m ? (uint32_t)(ctz32(m) + 1) << ((I & 7) * 4) : 0u;
    LS_PIN(b.V[I >> 3]);  // V is write-only in a pass: without this its OR chain is deferred
}

// One naked-single pass, Gauss-Seidel.  Returns DEAD / OPEN; `placed` counts.
template <int I>
LS_FN void naked_cell(Board &b, uint32_t &dead, uint32_t &placed)
{
    const uint32_t e = (b.E[I >> 5] >> (I & 31)) & 1u;
    const uint32_t cand = ~(b.U[ROW(I)] | b.U[9 + COL(I)] | b.U[18 + BOX(I)]) & 0x1FFu;
    const bool single = e && cand && !(cand & (cand - 1));
    dead |= e && !cand ? 1u : 0u;
    placed += single ? 1u : 0u;
    place_c<I>(b, single ? cand : 0u);
    LS_PIN(dead);
    LS_PIN(placed);
}

template <int I>
struct NakedPass {
    LS_FN_STATIC void run(Board &b, uint32_t &dead, uint32_t &placed)
    {
        naked_cell<I>(b, dead, placed);
        if ((I % 9) == 8) pin_board(b);
        NakedPass<I + 1>::run(b, dead, placed);
    }
};
template <>
struct NakedPass<81> {
    LS_FN_STATIC void run(Board &, uint32_t &, uint32_t &) {}
};

// Hidden singles of unit U_ (off when its givens clash).  Candidates are
// taken from the masks as they stand (earlier units' placements included).
// Branch-free: a lane-divergent early exit per unit would split the
// unrolled pass into 27 regions and blow up register pressure.
template <int U_>
LS_FN void hidden_unit(Board &b, uint32_t &dead, uint32_t &placed)
{
    const uint32_t ok = ((b.bad >> U_) & 1u) ? 0u : 0x1FFu;
    uint32_t cand[9];
    uint32_t once = 0, twice = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int i = UCELL(U_, k);
        const uint32_t e = 0u - ((b.E[i >> 5] >> (i & 31)) & 1u);  // all ones if empty
        cand[k] = ~(b.U[ROW(i)] | b.U[9 + COL(i)] | b.U[18 + BOX(i)]) & e & 0x1FFu;
        twice |= once & cand[k];
        once |= cand[k];
    }
    dead |= ((once | b.U[U_] | ~ok) & 0x1FFu) != 0x1FFu ? 1u : 0u;
    const uint32_t hid = once & ~twice & ok;
#define SDK_HID_PLACE(K)                                                         \
    {                                                                            \
        constexpr int i = UCELL(U_, K);                                          \
        const uint32_t m = cand[K] & hid;                                        \
        const bool multi = (m & (m - 1)) != 0;                                   \
        dead |= multi ? 1u : 0u;                                                 \
        placed += m ? 1u : 0u;                                                   \
        place_c<i>(b, multi ? 0u : m);                                           \
    }
    SDK_HID_PLACE(0) SDK_HID_PLACE(1) SDK_HID_PLACE(2) SDK_HID_PLACE(3) SDK_HID_PLACE(4)
    SDK_HID_PLACE(5) SDK_HID_PLACE(6) SDK_HID_PLACE(7) SDK_HID_PLACE(8)
#undef SDK_HID_PLACE
    LS_PIN(dead);
    LS_PIN(placed);
}

template <int U_>
struct HiddenPass {
    LS_FN_STATIC void run(Board &b, uint32_t &dead, uint32_t &placed)
    {
        hidden_unit<U_>(b, dead, placed);
        pin_board(b);
        HiddenPass<U_ + 1>::run(b, dead, placed);
    }
};
template <>
struct HiddenPass<27> {
    LS_FN_STATIC void run(Board &, uint32_t &, uint32_t &) {}
};

// the walk's next cell among the empty cells (eb0: cells 0..63, eb1: 64..80)
LS_FN int order_cell(uint64_t eb0, uint64_t eb1, int node_order)
{
    if (node_order) return eb0 ? ctz64(eb0) : 64 + ctz64(eb1);
    const int hi = eb1 ? 64 + 63 - clz64(eb1) : 63 - clz64(eb0);
    const int start = (hi / 9) * 9;
    if (start >= 64) return start + ctz64(eb1 >> (start - 64));
    const uint64_t m = eb0 & (~0ull << start);
    return m ? ctz64(m) : 64 + ctz64(eb1);
}

// candidates of a runtime cell index (guess time only)
LS_FN uint32_t cand_at(const Board &b, int cell)
{
    const int r = cell / 9, c = cell % 9, x = (r / 3) * 3 + c / 3;
    uint32_t u = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        u |= (k == r) ? b.U[k] : 0u;
        u |= (k == c) ? b.U[9 + k] : 0u;
        u |= (k == x) ? b.U[18 + k] : 0u;
    }
    return ~u & 0x1FFu;
}

// set a runtime cell to digit bit m (guess / backtrack time only)
LS_FN void place_at(Board &b, int cell, uint32_t m)
{
    const int r = cell / 9, c = cell % 9, x = (r / 3) * 3 + c / 3;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        b.U[k] |= (k == r) ? m : 0u;
        b.U[9 + k] |= (k == c) ? m : 0u;
        b.U[18 + k] |= (k == x) ? m : 0u;
    }
    const uint32_t d = (uint32_t)(ctz32(m) + 1);
#pragma unroll
    for (int w = 0; w < 3; ++w) b.E[w] &= (w == (cell >> 5)) ? ~(1u << (cell & 31)) : ~0u;
#pragma unroll
    for (int w = 0; w < 11; ++w) b.V[w] |= (w == (cell >> 3)) ? d << ((cell & 7) * 4) : 0u;
}

// stack entry: V[11], E[3], (cell << 9 | untried digits)
enum { STACK_WORDS = 15, STACK_ENTRY = 14, MAX_DEPTH = 82 };

struct Stats {
    uint32_t guesses, passes;
};

// Solve in place.  `stk` holds MAX_DEPTH * STACK_WORDS words (per lane).
// Returns 1 solved, 0 no completion.  V must hold the board; bad the clash
// mask from the load-time rebuild().
template <typename Stack>
LS_FN int solve(Board &b, Stack &stk, int node_order, Stats &st)
{
    uint32_t depth = 0;
    for (;;) {
        uint32_t dead = 0, placed = 0;
        NakedPass<0>::run(b, dead, placed);
        st.passes++;
        if (!dead && !placed && (b.E[0] | b.E[1] | b.E[2])) {
            HiddenPass<0>::run(b, dead, placed);
            st.passes++;
        }
        if (!dead) {
            if (!(b.E[0] | b.E[1] | b.E[2])) return 1;
            if (placed) continue;
            // branch on the walk's next cell, smallest digit first
            const int cell = order_cell((uint64_t)b.E[0] | ((uint64_t)b.E[1] << 32), (uint64_t)b.E[2], node_order);
            const uint32_t cand = cand_at(b, cell);
            const uint32_t d = cand & (0u - cand);
#pragma unroll
            for (int w = 0; w < 11; ++w) stk.put(depth, w, b.V[w]);
#pragma unroll
            for (int w = 0; w < 3; ++w) stk.put(depth, 11 + w, b.E[w]);
            stk.put(depth, STACK_ENTRY, ((uint32_t)cell << 9) | (cand ^ d));
            depth++;
            st.guesses++;
            place_at(b, cell, d);
            continue;
        }
        // dead: back to the deepest level with an untried digit
        for (;;) {
            if (depth == 0) return 0;
            depth--;
            const uint32_t entry = stk.get(depth, STACK_ENTRY);
            const uint32_t rem = entry & 0x1FFu;
            if (!rem) continue;
            const int cell = (int)(entry >> 9);
            const uint32_t d = rem & (0u - rem);
#pragma unroll
            for (int w = 0; w < 11; ++w) b.V[w] = stk.get(depth, w);
#pragma unroll
            for (int w = 0; w < 3; ++w) b.E[w] = stk.get(depth, 11 + w);
            rebuild_units(b);
            stk.put(depth, STACK_ENTRY, ((uint32_t)cell << 9) | (rem ^ d));
            depth++;
            st.guesses++;
            place_at(b, cell, d);
            break;
        }
    }
}

// load 81 bytes (values must be <= 9)
LS_FN void load(Board &b, const uint8_t *src)
{
#pragma unroll
    for (int w = 0; w < 11; ++w) b.V[w] = 0;
    b.E[0] = b.E[1] = b.E[2] = 0;
#pragma unroll
    for (int i = 0; i < 81; ++i) {
        const uint32_t v = src[i];
        b.V[i >> 3] |= v << ((i & 7) * 4);
        b.E[i >> 5] |= v ? 0u : 1u << (i & 31);
    }
    b.bad = rebuild_units(b);
}

#if defined(__HIPCC__) || defined(LS_HOST_ALIGNBYTE)
// Device load: the board's 81 bytes start at any byte offset; read the 21
// aligned dwords that cover them, realign with v_alignbyte, then pack the
// nibbles and the empty bits with bit tricks (no 81-register byte burst).
// Returns false if a byte is > 9.
LS_FN bool load_dw(Board &b, const uint8_t *src)
{
    const uintptr_t a = (uintptr_t)src;
    const uint32_t *base = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    // 21 dwords: each holds at least one byte of the board (byte 80 lies in
    // dword 20 for every start offset), so no read leaves the board's words
    uint32_t raw[22];
#pragma unroll
    for (int k = 0; k < 21; ++k) raw[k] = base[k];
    raw[21] = raw[20];  // only feeds bytes 81.. of the last group, masked below
    uint32_t bad = 0;
#pragma unroll
    for (int w = 0; w < 11; ++w) b.V[w] = 0;
    b.E[0] = b.E[1] = b.E[2] = 0;
#pragma unroll
    for (int k = 0; k < 21; ++k) {
        uint32_t x = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh);  // bytes 4k .. 4k+3
        if (k == 20) x &= 0xFFu;                                          // byte 80 only
        bad |= ((x + 0x76767676u) | x) & 0x80808080u;                     // some byte > 9
        // four nibbles
        const uint32_t nib = (x & 0xFu) | ((x >> 4) & 0xF0u) | ((x >> 8) & 0xF00u) | ((x >> 12) & 0xF000u);
        b.V[k >> 1] |= nib << ((k & 1) * 16);
        // zero bytes -> empty bits; exact per byte (no borrow/carry crosses
        // a byte because bit 7 is masked off before the add)
        const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
        const uint32_t zb = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
        const int cell = 4 * k;
        b.E[cell >> 5] |= (k == 20 ? (zb & 1u) : zb) << (cell & 31);
    }
    b.bad = rebuild_units(b);
    return bad == 0;
}
#endif

LS_FN void store(const Board &b, uint8_t *dst)
{
#pragma unroll
    for (int i = 0; i < 81; ++i) dst[i] = (uint8_t)getv(b, i);
}

}  // namespace lane

#endif  // SDK_LANE_SOLVER_H
