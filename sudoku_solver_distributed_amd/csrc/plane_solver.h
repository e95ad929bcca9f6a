// plane_solver.h -- one board per LANE on digit-plane bitboards.
//
// Same contract as the wave-per-board kernels (sudoku_kernels.hip): the
// first completion of the reference walk `order` (gen.py:6-28 /
// node.py:62-74), found with sound propagation + branching on the walk's
// next undetermined cell, digits ascending.  The state of a
// board is nine digit planes: P[d][b] is the set of cells of band b (rows
// 3b..3b+2) where digit d+1 is still possible, one 32-bit word per band:
//
//     bit 10*k + c  = cell (3b+k, c)      k = 0..2, c = 0..8
//     bits 9, 19, 29 = guard bits (always 0), bits 30-31 unused
//
// A cell whose only candidate is d is "determined" (it is the reference's
// filled cell).  The guard bits let one add / subtract act on the three
// 9-cell rows of a word at once without carries crossing rows.
//
// One pass (pass()) applies, to every cell and unit of the board:
//   A. determined cells: cells with one candidate; a cell with none is dead;
//   B. each newly determined cell removes its digit from its row, column and
//      box (a clash with an older determined cell empties that cell: dead);
//   C. hidden singles: a digit with exactly one place in a unit goes there;
//      a digit with no place in a unit kills the node; two digits forced into
//      one cell kill it;
//   D. locked candidates (SDK_PLANE_LC flags): a box whose places for a
//      digit lie in one column takes the digit out of that column's cells in
//      the other two bands (1, the default); one whose places lie in one
//      row, out of that row's cells in the other two boxes (2); a column
//      whose places lie in one band, out of the rest of its box (4).  Fewer
//      passes and branch nodes for ~250 VALU per pass.
// Rules B, C and D are sound only when the givens do not repeat a digit in a
// unit (the walk never tests givens, gen.py:8-28): such boards are reported
// as `bad` by load() and left to the wave-per-board kernel, which handles
// them.  Two determined cells sharing a digit in one unit are not flagged
// the moment they appear; the search can only end on a board where every
// unit holds every digit (pass(): all cells determined and rule C's
// empty-unit test clean), so such a node still dies, a few passes later.
//
// Everything here is plain C++ usable on host and device: the CPU tests
// compile it with g++ (tests/native/plane_host.cpp) and check it against
// the oracle before the GPU runs it.
#ifndef SDK_PLANE_SOLVER_H
#define SDK_PLANE_SOLVER_H

#include <stdint.h>

#ifdef __HIPCC__
#define PS_FN __host__ __device__ __forceinline__
#define PS_MF __host__ __device__ __forceinline__
#else
#define PS_FN static inline
#define PS_MF inline
#endif

#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
// Make later code consume a value as it stands here (no instruction is
// emitted).  Pinning the board between the digits of a pass keeps the
// scheduler from hoisting nine digits' worth of independent work and running
// the pass at ~130 VGPRs instead of ~60.
#define PS_PIN(x) asm volatile("" : "+v"(x))
#else
#define PS_PIN(x) ((void)0)
#endif
#ifndef SDK_PLANE_PIN_ACC
#define SDK_PLANE_PIN_ACC 1
#endif
// pass() rule D (locked candidates), flags: 1 box -> column, 2 box -> row,
// 4 column -> box; 0 off.  3 pays since round 6 made the rest of the pass
// cheaper: 28 % fewer passes and 39 % fewer branch nodes per board for 37 %
// more VALU per pass, and fewer search steps
#ifndef SDK_PLANE_LC
#define SDK_PLANE_LC 3
#endif
// the same flags for the wave-wide tail solver (plane_wide.h), whose passes
// are latency- rather than issue-bound
#ifndef SDK_WIDE_LC
#define SDK_WIDE_LC SDK_PLANE_LC
#endif
// pass() rule C's hidden singles, applied in groups of SDK_PLANE_GROUP
// digits: a digit's plane drops the singles of the EARLIER groups' digits
// before its rules run, and those of its own group's lower digits after
// them.  1 is Gauss-Seidel (one dependency chain through all nine digits);
// with larger groups a group's rule chains are independent of each other
// and the board is pinned once per group, so the group's chains interleave.
// Every grouping is sound and reaches the same fixpoints.
#ifndef SDK_PLANE_GROUP
#define SDK_PLANE_GROUP 1
#endif
// rule C's box singles through rule D's one-column boxes: a box with one
// place is a box with one column (vp) whose column holds one place, and
// that column's cells in the band stand for the box's; the box and column
// singles then share one spread over the rows (27 multiplies and ~80 VALU
// fewer per pass; same hidden singles).  Needs rule D's box -> column form.
#ifndef SDK_PLANE_HX
#define SDK_PLANE_HX 1
#endif
#if SDK_PLANE_HX && !(SDK_PLANE_LC & 1)
#undef SDK_PLANE_HX
#define SDK_PLANE_HX 0
#endif

namespace plane {

enum : uint32_t {
    ROWS = 0x1FFu | (0x1FFu << 10) | (0x1FFu << 20),  // the 27 cells of a band word
    GUARDS = (1u << 9) | (1u << 19) | (1u << 29),     // one guard bit above each row
    ONES = 1u | (1u << 10) | (1u << 20),              // bit 0 of each row
    KDEC = GUARDS - ONES,                             // y + KDEC == (y | GUARDS) - ONES
    BOXC = 0x49u,                                     // bit 0 of each 3-column box group
};

enum { OPEN = 0, DEAD = 1, SOLVED = 2, STUCK = 3 };

struct Board {
    uint32_t P[9][3];  // P[d][b]: cells of band b where digit d+1 is possible
    uint32_t Det[3];   // determined cells already eliminated from their peers
};

PS_FN void pin_board(Board &B)
{
#pragma unroll
    for (int d = 0; d < 9; ++d)
#pragma unroll
        for (int b = 0; b < 3; ++b) PS_PIN(B.P[d][b]);
}

PS_FN constexpr int cell_band(int i) { return i / 27; }
PS_FN constexpr int cell_pos(int i) { return 10 * ((i / 9) % 3) + i % 9; }
// cell index of (band, bit position)
PS_FN int pos_cell(int b, int pos) { return 27 * b + 9 * (pos / 10) + pos % 10; }

// ---- three-input logic at full issue rate
// gfx950 issues a wave64 VALU instruction every 2 cycles only for some forms
// (scripts/microbench/exec_rate.hip, profiles/r02_valu_rates.json): VOP2
// and/or/xor/add/sub/lshrrev with VGPR, inline or literal operands, and
// v_bitop3_b32 with VGPR or inline operands.  Every form reading an SGPR,
// v_or3 / v_and_or / v_bfi / v_bfe / v_lshl* and the multiplies take 4.
// LLVM builds 3-input logic from v_or3 / v_bfi / v_and_or and keeps
// constants in SGPRs, so the pass spells its 3-input logic as v_bitop3_b32
// on VGPR operands (truth table f(0xF0, 0xCC, 0xAA) over src0, src1, src2).
#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
// a constant as a VGPR value the compiler cannot turn back into an SGPR
// operand (a VOP3 on gfx9 takes no literal: LLVM would put it in an SGPR)
template <uint32_t K>
__device__ __forceinline__ uint32_t vconst()
{
    uint32_t r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "i"(K));
    return r;
}
template <unsigned TT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}
#define PS_BOP3(TT, a, b, c, host) bop3<TT>(a, b, c)
#else
#define PS_BOP3(TT, a, b, c, host) (host)
#endif
PS_FN uint32_t or3(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0xFE, a, b, c, a | b | c); }
PS_FN uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0xE8, a, b, c, (a & b) | (c & (a | b))); }
PS_FN uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0x96, a, b, c, a ^ b ^ c); }
PS_FN uint32_t andn(uint32_t a, uint32_t b) { return PS_BOP3(0x30, a, b, b, a & ~b); }
PS_FN uint32_t andn2(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0x10, a, b, c, a & ~b & ~c); }
PS_FN uint32_t and_andn(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0x40, a, b, c, a & b & ~c); }
PS_FN uint32_t or_and(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0xF8, a, b, c, a | (b & c)); }
PS_FN uint32_t or_andn(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0xF4, a, b, c, a | (b & ~c)); }
PS_FN uint32_t and3(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0x80, a, b, c, a & b & c); }
PS_FN uint32_t andn_and(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0x70, a, b, c, a & ~(b & c)); }
PS_FN uint32_t sel(uint32_t m, uint32_t a, uint32_t b) { return PS_BOP3(0xCA, m, a, b, (m & a) | (~m & b)); }
// ~a | b | c: a cell of y is a hidden single if its row has one place (not
// in a), or its box (b) or its column (c) has one
PS_FN uint32_t bop3_nor(uint32_t a, uint32_t b, uint32_t c) { return PS_BOP3(0xEF, a, b, c, ~a | b | c); }
// 9-bit set (low 24 bits of c may hold no other bit) times k: one v_mul_u32_u24
PS_FN uint32_t mul24(uint32_t c, uint32_t k) { return (c & 0xFFFFFFu) * k; }
// box bits (0 / 3 / 6, nothing else below bit 16) -> the boxes' nine
// columns.  SDK_PLANE_MUL16: as a 16-bit multiply (v_mul_lo_u16 issues at
// full rate on gfx950, v_mul_u32_u24 at half: profiles/r02_valu_rates.json)
#ifndef SDK_PLANE_MUL16
#define SDK_PLANE_MUL16 1
#endif
// the box bits of x & ~m: one v_bitop3 with BOXC in a VGPR instead of two ops
PS_FN uint32_t box_one(uint32_t x, uint32_t m)
{
#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
    return bop3<0x20>(x, m, vconst<BOXC>());
#else
    return x & ~m & BOXC;
#endif
}
PS_FN uint32_t box_cols(uint32_t c)
{
#if SDK_PLANE_MUL16 && defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
    // in place: the high half of the register is c's (zero) whether the
    // instruction keeps or clears it (LLVM itself widens the i16 multiply
    // back to v_mul_u32_u24)
    uint32_t r = c;
    asm("v_mul_lo_u16 %0, 7, %0" : "+v"(r));
    return r;
#else
    return mul24(c, 7u);
#endif
}

// rule D, box -> row, on one band word y of a digit's plane: the cells to
// clear because a box of the band holds all its places in one row -- that
// row outside the box.  (Two boxes pointing into two rows: each one's cells
// in the other's row hold no place already.)  16 VALU, applied.
// point_rows_parts: the rows to clear and the pointing boxes' area (clear =
// rows outside the area); point_rows(y) = the cells to clear; point_rows_apply
// clears them from y in one v_bitop3.
PS_FN void point_rows_parts(uint32_t y, uint32_t &rows, uint32_t &area)
{
    const uint32_t r3 = or3(y, y >> 1, y >> 2) & 0x4912449u;  // row k of box j has a place: bit 10k + 3j
    const uint32_t a1 = r3 >> 10, a2 = r3 >> 20;
    const uint32_t hbox = box_one(xor3(r3, a1, a2), maj3(r3, a1, a2));  // boxes with places in one row
    area = mul24(hbox, 0x701C07u);
    const uint32_t rn = ((r3 & area) + ROWS) & GUARDS;  // the rows of those boxes' places (r3 holds bits 10k + 3j only)
    rows = rn - (rn >> 9);
}
PS_FN uint32_t point_rows(uint32_t y)
{
    uint32_t rows, area;
    point_rows_parts(y, rows, area);
    return andn(rows, area);
}
PS_FN uint32_t point_rows_apply(uint32_t y)
{
    uint32_t rows, area;
    point_rows_parts(y, rows, area);
    return PS_BOP3(0xB0, y, rows, area, y & ~(rows & ~area));  // y & (~rows | area)
}

PS_FN uint32_t spread_rows(uint32_t c) { return c | (c << 10) | (c << 20); }  // 9-bit column set -> 3 rows
PS_FN uint32_t guard_rows(uint32_t g) { return g - (g >> 9); }               // guard flags -> whole rows
PS_FN uint32_t row_nonzero(uint32_t y) { return (y + ROWS) & GUARDS; }        // guard set iff row != 0
PS_FN uint32_t fold_rows(uint32_t y) { return (y | (y >> 10) | (y >> 20)) & 0x1FFu; }

struct Board;
PS_FN void pin_board(Board &B);

// One propagation pass (rules A-D above).  Returns DEAD, SOLVED, STUCK (no
// single found: und[] = the undetermined cells; rule D may still have
// removed places, which the next pass sees) or OPEN (pass again).
//
// Written for the full-rate issue forms (see or3() above): two-input ops
// with literal constants, three-input logic as v_bitop3_b32 on VGPRs, right
// shifts only, 16-bit multiplies for 9-bit results, and one v_mul_u32_u24
// per spread of a set over a band's three rows.  1797 VALU per pass with
// SDK_PLANE_LC 3 (profiles/isa_plane_pass.json).
PS_FN int pass(Board &B, uint32_t und[3])
{
    uint32_t single[3], nd[3];
    uint32_t dead = 0;
    // ---- A: determined cells.  o: >= 1 candidate, t: >= 2 candidates
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        // (every 3-input OR spelled as one bitop3: LLVM would fuse the
        // 2-input ones into v_or3 / v_and_or)
        uint32_t o = B.P[0][b] | B.P[1][b];
        const uint32_t m23 = maj3(o, B.P[2][b], B.P[3][b]);
        o = or3(o, B.P[2][b], B.P[3][b]);
        const uint32_t m45 = maj3(o, B.P[4][b], B.P[5][b]);
        o = or3(o, B.P[4][b], B.P[5][b]);
        uint32_t t = or_and(m23, B.P[0][b], B.P[1][b]);
        t = or3(t, m45, maj3(o, B.P[6][b], B.P[7][b]));
        o = or3(o, B.P[6][b], B.P[7][b]);
        t = or_and(t, o, B.P[8][b]);
        o |= B.P[8][b];
        dead = or_andn(dead, ROWS, o);
        single[b] = andn(o, t);
        nd[b] = andn(single[b], B.Det[b]);
        B.Det[b] = single[b];
        und[b] = andn(ROWS, single[b]);
    }
    const bool all_single = and3(single[0], single[1], single[2]) == ROWS;
    const bool any_nd = or3(nd[0], nd[1], nd[2]) != 0;
    pin_board(B);

    uint32_t hall[3] = {0u, 0u, 0u};
#if SDK_PLANE_GROUP > 1
    uint32_t hgrp[3] = {0u, 0u, 0u};
#endif
    // per unit kind, "d has a place": row guard bits, columns, box bits 0/3/6
    uint32_t rowall = GUARDS, colall = 0x1FFu, boxall = BOXC;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        // hidden singles placed for digits < d this pass leave d's plane
        // (Gauss-Seidel: d sees them); digits < d are fixed up after the loop
        // ---- B: remove d from the peers of the newly determined cells holding d
        uint32_t x[3], f[3];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
#if SDK_PLANE_GROUP > 1
            if (d >= SDK_PLANE_GROUP) B.P[d][b] = andn(B.P[d][b], hgrp[b]);
#else
            if (d > 0) B.P[d][b] = andn(B.P[d][b], hall[b]);  // (the same code path as before groups existed)
#endif
            x[b] = nd[b] & B.P[d][b];
            f[b] = or3(x[b], x[b] >> 10, x[b] >> 20);  // bits 0-8: columns holding x (above: junk)
        }
        const uint32_t cpeer = mul24(or3(f[0], f[1], f[2]) & 0x1FFu, 0x100401u);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const uint32_t g = or3(f[b], f[b] >> 1, f[b] >> 2);           // box bits 0/3/6
            const uint32_t rn = (x[b] + ROWS) & GUARDS;                  // rows holding x
            const uint32_t peer = or3(rn - (rn >> 9), cpeer, mul24(g & BOXC, 0x701C07u));
            B.P[d][b] = sel(peer, x[b], B.P[d][b]);
        }
        // ---- C: hidden singles of d; units with no place left for d
        uint32_t o[3], t[3], gr[3], hb[3];
#if SDK_PLANE_LC
        uint32_t vp[3];  // rule D: per band, the column of each box whose places lie in one column
#endif
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const uint32_t y = B.P[d][b];
            const uint32_t y1 = y + ROWS;     // row guard set iff the row has a place; = y + KDEC
            rowall &= y1;
            const uint32_t z = y & y1;        // y without its lowest place per row
            const uint32_t nz = (z + ROWS) & GUARDS;
            gr[b] = nz - (nz >> 9);           // rows with >= 2 places
            const uint32_t s1 = y >> 10, s2 = y >> 20;
            o[b] = or3(y, s1, s2);            // bits 0-8: columns with >= 1 place in the band
            t[b] = maj3(y, s1, s2);           //           columns with >= 2
            const uint32_t o1 = o[b] >> 1, o2 = o[b] >> 2;
            const uint32_t ob = or3(o[b], o1, o2);     // box bits 0/3/6: >= 1 place
            boxall &= ob;
            const uint32_t mo = maj3(o[b], o1, o2);     // box bits: >= 2 columns with a place
#if SDK_PLANE_HX
            // a box with one place: its one column (vp) holding one place
            // (not in t); that column within the band lies in the box, so
            // the column's three cells stand for the box's nine (below)
            const uint32_t vb = box_one(xor3(o[b], o1, o2), mo);  // boxes with exactly one column
            vp[b] = o[b] & box_cols(vb);
            hb[b] = andn(vp[b], t[b]);
#else
            const uint32_t tb = or3(t[b], t[b] >> 1, t[b] >> 2);
            const uint32_t q = andn2(ob, tb, mo) & BOXC;  // boxes with exactly one
            hb[b] = mul24(q, 0x701C07u);
#if SDK_PLANE_LC
            const uint32_t vb = andn(xor3(o[b], o1, o2), mo) & BOXC;  // boxes with exactly one column
            vp[b] = o[b] & box_cols(vb);
#endif
#endif
        }
        const uint32_t O = or3(o[0], o[1], o[2]);
        colall &= O;
        const uint32_t mo3 = maj3(o[0], o[1], o[2]);  // columns with places in >= 2 bands
        const uint32_t hc = andn2(O, or3(t[0], t[1], t[2]), mo3) & 0x1FFu;
#if SDK_PLANE_HX
        // box and column singles share one spread over the band's rows
#pragma unroll
        for (int b = 0; b < 3; ++b) hb[b] = mul24(hb[b] | hc, 0x100401u);
        const uint32_t hcol = 0u;
#else
        const uint32_t hcol = mul24(hc, 0x100401u);
#endif
        // d's hidden singles: the cells of y alone in their row, column or
        // box.  Later digits drop these cells at their turn (above), earlier
        // ones after the loop.  A cell forced for two digits loses the later
        // one, whose unit then has no place for it: dead, as it must be.
#if SDK_PLANE_LC
        // ---- D: locked candidates (pointing): a box whose places for d lie
        // in one column holds d's place of that column, so the column's
        // cells in the other two bands lose d; likewise for a row
        // (point_rows).  The singles of d see it next pass.
        {
            const uint32_t vpa = or3(vp[0], vp[1], vp[2]);
            const uint32_t one_band = andn(xor3(o[0], o[1], o[2]), mo3) & 0x1FFu;  // columns with places in one band
            (void)vpa;
            (void)one_band;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                uint32_t ec = 0;  // columns of the band to clear
#if SDK_PLANE_LC & 1
                ec = andn(vpa, vp[b]);
#endif
#if SDK_PLANE_LC & 4
                {
                    // column -> box: a column whose places lie in this band
                    // holds the box's place: the box's other columns lose d
                    const uint32_t cc = o[b] & one_band;
                    ec |= andn(mul24(or3(cc, cc >> 1, cc >> 2) & BOXC, 7u), cc);
                }
#endif
                const uint32_t e = mul24(ec, 0x100401u);
                B.P[d][b] = andn(B.P[d][b], e);
            }
        }
#endif
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const uint32_t hs = bop3_nor(gr[b], hb[b], hcol);  // d's single places (where d is possible)
#if SDK_PLANE_GROUP > 1
            if (d % SDK_PLANE_GROUP) {
                // the singles of this group's lower digits leave d's plane, d's own stay
                const uint32_t p = B.P[d][b];
                B.P[d][b] = PS_BOP3(0xB0, p, hall[b], hs, p & ~(hall[b] & ~hs));
                hall[b] = or_and(hall[b], p, hs);
                continue;
            }
#endif
            hall[b] = or_and(hall[b], B.P[d][b], hs);
        }
#if SDK_PLANE_GROUP > 1
        if (d % SDK_PLANE_GROUP != SDK_PLANE_GROUP - 1 && d != 8) continue;
#pragma unroll
        for (int b = 0; b < 3; ++b) hgrp[b] = hall[b];  // what the next group's digits drop first
#endif
        pin_board(B);
        // the unit accumulators too: unpinned, the AND / OR chains over the
        // nine digits are re-associated into trees at the end of the pass,
        // keeping 27 row-test words live (~200 VGPRs instead of ~100)
#if SDK_PLANE_PIN_ACC
        PS_PIN(rowall);
        PS_PIN(colall);
        PS_PIN(boxall);
#pragma unroll
        for (int b = 0; b < 3; ++b) PS_PIN(hall[b]);
#endif
    }
    // A cell forced to digit d this pass is still in d's plane and, from the
    // clearing above, in no later digit's: so it leaves every EARLIER plane
    // that a later plane still holds.  Same state as clearing all eight
    // other planes the moment d's singles were found.
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        uint32_t later = B.P[8][b];
#pragma unroll
        for (int e = 7; e >= 0; --e) {
            B.P[e][b] = andn_and(B.P[e][b], hall[b], later);
            if (e) later |= B.P[e][b];
        }
    }
#if SDK_PLANE_LC & 2
    {
        // rule D's box -> row form, after the digit loop (its registers are
        // free again): every plane word once
#pragma unroll
        for (int d = 0; d < 9; ++d)
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                B.P[d][b] = point_rows_apply(B.P[d][b]);
                PS_PIN(B.P[d][b]);
            }
    }
#endif
    dead |= or3(rowall ^ GUARDS, colall ^ 0x1FFu, (boxall & BOXC) ^ BOXC);
    if (dead) return DEAD;
    if (all_single) return SOLVED;
    const bool newh = or3(hall[0] & und[0], hall[1] & und[1], hall[2] & und[2]) != 0;
    // (rule D's removals alone do not make the pass OPEN: the board then
    // branches one pass early, on sound planes -- host model: 21.389 against
    // 21.390 passes per board, DESIGN.md §4 -- and the step saves its
    // change tracking, 27 VALU)
    return (any_nd || newh) ? OPEN : STUCK;
}

// The walk's branch cell among the undetermined cells: node.py:63-65 takes
// the first in row-major order; gen.py:11-15 the first of the LAST row that
// has one (its column loop breaks, its row loop does not).
PS_FN void pick_cell(const uint32_t und[3], int node_order, int &band, int &pos)
{
    if (node_order) {
        band = und[0] ? 0 : und[1] ? 1 : 2;
        const uint32_t w = band == 0 ? und[0] : band == 1 ? und[1] : und[2];
        pos = __builtin_ctz(w);
    } else {
        band = und[2] ? 2 : und[1] ? 1 : 0;
        const uint32_t w = band == 0 ? und[0] : band == 1 ? und[1] : und[2];
        const int hi = 31 - __builtin_clz(w);
        const int k = hi >= 20 ? 2 : hi >= 10 ? 1 : 0;
        pos = 10 * k + __builtin_ctz(w >> (10 * k));
    }
}

// Fewest-candidates cell for the completion count (search mode M_COUNT
// below): the first undetermined cell (band order, then bit order) with
// exactly 2 candidates, else with exactly 3, else the first undetermined
// cell.  Saturating candidate counters over the nine planes, per band.
// the choice from the per-band masks of undetermined cells with exactly 2
// (e2) and exactly 3 (e3) candidates (shared with the wave-wide solver)
//
// SDK_PLANE_MRV_PICK 1 (round 5, off): among the two-candidate cells, one in
// the column holding the most of them (lowest such column, first band) -- a
// branch there constrains the most other two-candidate cells.  Column counts
// by a carry-save adder over the nine row words, the maximum by masking from
// the top count bit down: ~45 VALU.  4 % fewer passes, but measured 3 %
// slower on the GPU.
#ifndef SDK_PLANE_MRV_PICK
#define SDK_PLANE_MRV_PICK 0
#endif
PS_FN void pick_mrv_masks(const uint32_t (&e2)[3], const uint32_t (&e3)[3], const uint32_t und[3], int &band,
                          int &pos)
{
#if SDK_PLANE_MRV_PICK
    uint32_t r[9];
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        r[3 * b] = e2[b] & 0x1FFu;
        r[3 * b + 1] = (e2[b] >> 10) & 0x1FFu;
        r[3 * b + 2] = e2[b] >> 20;
    }
    const uint32_t sa = xor3(r[0], r[1], r[2]), ca = maj3(r[0], r[1], r[2]);
    const uint32_t sb = xor3(r[3], r[4], r[5]), cb = maj3(r[3], r[4], r[5]);
    const uint32_t sc = xor3(r[6], r[7], r[8]), cc = maj3(r[6], r[7], r[8]);
    const uint32_t c1 = xor3(sa, sb, sc), cd = maj3(sa, sb, sc);  // count bit 0, carry into 2
    const uint32_t se = xor3(ca, cb, cc), ce = maj3(ca, cb, cc);  // weight 2 (of three), carry into 4
    const uint32_t c2 = se ^ cd, cf = se & cd;
    const uint32_t c4 = ce ^ cf, c8 = ce & cf;                    // count bits 1, 2, 3 (<= 9)
    uint32_t m = or3(c1, c2, c4 | c8);                            // columns with one or more
    uint32_t t = m & c8;
    m = t ? t : m;
    t = m & c4;
    m = t ? t : m;
    t = m & c2;
    m = t ? t : m;
    t = m & c1;
    m = t ? t : m;                                                // the columns with the most
    if (m) {
        const uint32_t col = spread_rows(m & (0u - m));          // the lowest of them, over three rows
        band = (e2[0] & col) ? 0 : (e2[1] & col) ? 1 : 2;
        pos = __builtin_ctz((band == 0 ? e2[0] : band == 1 ? e2[1] : e2[2]) & col);
        return;
    }
#endif
    const uint32_t w[3] = {e2[0] ? e2[0] : e3[0] ? e3[0] : und[0], e2[1] ? e2[1] : e3[1] ? e3[1] : und[1],
                           e2[2] ? e2[2] : e3[2] ? e3[2] : und[2]};
    const int k2 = e2[0] ? 0 : e2[1] ? 1 : e2[2] ? 2 : -1;
    const int k3 = e3[0] ? 0 : e3[1] ? 1 : e3[2] ? 2 : -1;
    band = k2 >= 0 ? k2 : k3 >= 0 ? k3 : (und[0] ? 0 : und[1] ? 1 : 2);
    pos = __builtin_ctz(band == 0 ? w[0] : band == 1 ? w[1] : w[2]);
}

PS_FN void pick_mrv(const Board &B, const uint32_t und[3], int &band, int &pos)
{
    // per cell, the candidate count as bit-sliced binary s3 s2 s1 s0 from a
    // carry-save adder tree over the nine planes (full adder = one xor3 and
    // one maj3 bitop3): 19 ops per band where four saturating counters took 36
    uint32_t e2[3], e3[3];
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint32_t *p = &B.P[0][b];
#define PL(d) p[3 * (d)]
        const uint32_t sa = xor3(PL(0), PL(1), PL(2)), ca = maj3(PL(0), PL(1), PL(2));
        const uint32_t sb = xor3(PL(3), PL(4), PL(5)), cb = maj3(PL(3), PL(4), PL(5));
        const uint32_t sc = xor3(PL(6), PL(7), PL(8)), cc = maj3(PL(6), PL(7), PL(8));
#undef PL
        const uint32_t s0 = xor3(sa, sb, sc), cd = maj3(sa, sb, sc);  // weight 1, carry into weight 2
        const uint32_t se = xor3(ca, cb, cc), ce = maj3(ca, cb, cc);  // weight 2 (of three), carry into 4
        const uint32_t s1 = se ^ cd, cf = se & cd;                    // weight 2, carry into 4
        const uint32_t hi = ce | cf;                                  // weight >= 4 (ce, cf never both: <= 9)
        e2[b] = and_andn(und[b], s1, s0 | hi);                        // exactly 2
        e3[b] = and3(und[b], s1, s0) & ~hi;                           // exactly 3
    }
    pick_mrv_masks(e2, e3, und, band, pos);
}

PS_FN uint32_t band_word(const uint32_t (&w)[3], int band) { return band == 0 ? w[0] : band == 1 ? w[1] : w[2]; }

// candidates (bit d = digit d+1) of the cell at (band, pos).  Branch-free
// (band and pos differ per lane): the cell's bit of digit d's three words
// under a one-hot band mask, shifted down to bit 0, accumulated from digit 8
// down as c = 2c + bit -- right shifts and adds only, the full-rate forms.
PS_FN uint32_t cell_cand(const Board &B, int band, int pos)
{
    const uint32_t cb = 1u << pos;
    const uint32_t m0 = band == 0 ? cb : 0u, m1 = band == 1 ? cb : 0u, m2 = band == 2 ? cb : 0u;
    uint32_t c = 0;
#pragma unroll
    for (int d = 8; d >= 0; --d) {
        const uint32_t x = or_and(or_and(B.P[d][0] & m0, B.P[d][1], m1), B.P[d][2], m2);
        c = c + c + (x >> pos);
    }
    return c;
}

// fix the cell at (band, pos) to the digit bit `dbit` (bit d = digit d+1)
PS_FN void set_cell(Board &B, int band, int pos, uint32_t dbit)
{
    // one v_bitop3 per plane word: P & ~(cell-of-this-band & not-this-digit)
    const uint32_t cb = 1u << pos;
    const uint32_t m[3] = {band == 0 ? cb : 0u, band == 1 ? cb : 0u, band == 2 ? cb : 0u};
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        const uint32_t other = ((dbit >> d) & 1u) - 1u;  // 0 for the digit, all ones otherwise
#pragma unroll
        for (int b = 0; b < 3; ++b) B.P[d][b] = andn_and(B.P[d][b], m[b], other);
    }
}

// ---------------------------------------------------------- load / store
// Value bit-slices -> planes.  V[s][b]: cells whose value has bit s set;
// E[b]: empty cells.  Returns the given cells (non-empty).
PS_FN void planes_from_slices(Board &B, const uint32_t (&V)[4][3], uint32_t (&given)[3])
{
    // value v = (v1 v0) + 4 (v3 v2): one-hot over the low pair and over the
    // high pair, then each digit's plane is one AND of the two (plus the
    // empty cells): 18 operations per band instead of ~43
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint32_t v0 = V[0][b], v1 = V[1][b], v2 = V[2][b], v3 = V[3][b];  // cell bits only
        const uint32_t lo[4] = {andn2(ROWS, v0, v1), andn(v0, v1), andn(v1, v0), v0 & v1};
        const uint32_t hi[3] = {andn2(ROWS, v2, v3), andn(v2, v3), andn(v3, v2)};
        const uint32_t e = lo[0] & hi[0];
        given[b] = andn(ROWS, e);
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            const int v = d + 1;
            B.P[d][b] = or_and(e, lo[v & 3], hi[v >> 2]);
        }
        B.Det[b] = 0;
    }
}

// Do the givens repeat a digit in some row, column or box?  (Such boards
// are legal input -- the walk never tests the givens -- but rules B/C are
// unsound on them; the caller hands them to the wave-per-board kernel.)
PS_FN bool givens_clash(const Board &B, const uint32_t (&given)[3])
{
    uint32_t bad = 0;
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        uint32_t o[3], t[3];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const uint32_t y = B.P[d][b] & given[b];
            bad |= y & (y + KDEC);  // a row with two
            const uint32_t s1 = y >> 10, s2 = y >> 20;
            o[b] = (y | s1 | s2) & 0x1FFu;
            t[b] = ((y & s1) | (s2 & (y | s1))) & 0x1FFu;
            const uint32_t o1 = o[b] >> 1, o2 = o[b] >> 2;
            bad |= (t[b] | (t[b] >> 1) | (t[b] >> 2) | (o[b] & o1) | (o2 & (o[b] | o1))) & BOXC;
        }
        bad |= t[0] | t[1] | t[2] | (o[0] & o[1]) | (o[2] & (o[0] | o[1]));
    }
    return bad != 0;
}

// sum of the byte products of a and b, plus c (v_dot4_u32_u8 on the GPU)
PS_FN uint32_t dot4u8(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_udot4(a, b, c, false);
#else
    for (int i = 0; i < 32; i += 8) c += ((a >> i) & 0xFFu) * ((b >> i) & 0xFFu);
    return c;
#endif
}

// Value bit-slices V[s][b] of a board given as 21 words x[k] = bytes
// 4k..4k+3 (little endian; only byte 80 of x[20] is used).  Returns nonzero
// if a byte is > 9.
PS_FN uint32_t slices_from_words(const uint32_t (&x)[21], uint32_t (&V)[4][3])
{
    // Per value bit s, the 81-bit cell stream S (cell i = bit i) is built
    // eight cells at a time: bit s of the 8 bytes of two words, gathered by
    // one byte dot product each (weights 1, 2, 4, 8 and 16, 32, 64, 128 on
    // bytes that are 0 or 2^s), lands 2^s times the 8-bit group; then the
    // stream is cut into bands and the guard bits are inserted.  ~360 VALU
    // per board where a per-cell shift / mask / or per bit takes ~1000.
    const uint32_t x20 = x[20] & 0xFFu;
    uint32_t hiset = 0;  // bits 4-7 of any byte: value >= 16
#pragma unroll
    for (int k = 0; k < 20; k += 2) hiset = or3(hiset, x[k], x[k + 1]);
    hiset = (hiset | x20) & 0xF0F0F0F0u;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint32_t m = 0x01010101u << s;
        uint32_t S[3] = {0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 21; k += 2) {
            const uint32_t lo = (k == 20 ? x20 : x[k]) & m;
            uint32_t g = k < 20 ? dot4u8(x[k + 1] & m, 0x80402010u, 0u) : 0u;
            g = dot4u8(lo, 0x08040201u, g);  // 2^s * cells 4k..4k+7
            const int sh = (4 * k) % 32;     // 0, 8, 16, 24
            S[k / 8] |= sh >= s ? g << (sh - s) : g >> (s - sh);
        }
        // cells 27b..27b+26, then a guard bit above each row of nine
        const uint32_t c27[3] = {S[0] & 0x7FFFFFFu, ((S[0] >> 27) | (S[1] << 5)) & 0x7FFFFFFu,
                                 (S[1] >> 22) | (S[2] << 10)};
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const uint32_t w = c27[b];
            V[s][b] = or3(w & 0x1FFu, (w << 1) & (0x1FFu << 10), (w << 2) & (0x1FFu << 20));
        }
    }
    // a value of 10..15: bit 3 and bit 1 or 2
    uint32_t big = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) big = or3(big, V[3][b] & V[1][b], V[3][b] & V[2][b]);
    return hiset | big;
}

// Load from 21 words x[k] = bytes 4k..4k+3 of the board (little endian; only
// byte 80 of x[20] is used).  Returns false if a byte is > 9.
PS_FN bool load_words(Board &B, const uint32_t (&x)[21], bool &clash)
{
    uint32_t V[4][3];
    const uint32_t badb = slices_from_words(x, V);
    uint32_t given[3];
    planes_from_slices(B, V, given);
    clash = badb == 0 && givens_clash(B, given);
    return badb == 0;
}

// Store a SOLVED board: one byte per cell through `put(i, value)`.
template <typename Put>
PS_FN void store_values(const Board &B, Put put)
{
    uint32_t V[4][3];
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const uint32_t p0 = B.P[0][b], p1 = B.P[1][b], p2 = B.P[2][b], p3 = B.P[3][b], p4 = B.P[4][b];
        const uint32_t p5 = B.P[5][b], p6 = B.P[6][b], p7 = B.P[7][b], p8 = B.P[8][b];
        V[0][b] = p0 | p2 | p4 | p6 | p8;  // digits 1 3 5 7 9
        V[1][b] = p1 | p2 | p5 | p6;       // 2 3 6 7
        V[2][b] = p3 | p4 | p5 | p6;       // 4 5 6 7
        V[3][b] = p7 | p8;                 // 8 9
    }
#pragma unroll
    for (int i = 0; i < 81; ++i) {
        const int b = cell_band(i), p = cell_pos(i);
        const uint32_t v = ((V[0][b] >> p) & 1u) | (((V[1][b] >> p) & 1u) << 1) | (((V[2][b] >> p) & 1u) << 2) |
                           (((V[3][b] >> p) & 1u) << 3);
        put(i, v);
    }
}

// stack level: the 27 plane words + the branch entry
enum { STACK_WORDS = 28, STACK_ENTRY = 27 };
// branch entry: bits 0-4 pos, 5-6 band, 8-16 untried digits
PS_FN uint32_t make_entry(int band, int pos, uint32_t rem) { return (uint32_t)pos | ((uint32_t)band << 5) | (rem << 8); }

// ---- search modes of a board
// M_WALK: branch on the walk's next cell, digits ascending -- the first
// completion found is the walk's.  A board still searching
// after `mrv_after` passes switches to M_COUNT: back to its propagated root
// (stack level 0), branching on a fewest-candidates cell and counting
// completions to two, the first one kept on the stack's last level.  Exactly
// one completion IS the walk's answer (the walk's first completion is the
// only one); none means none for the walk too; a second one sends the board
// back to its root in M_FINAL, the walk again, with no further switch.
// Results never depend on mrv_after (0 = never switch).  Heavy-tailed sets
// gain most: 17-clue boards whose walk order is unlucky need up to ~5000
// walk passes, and at most ~1100 this way.
enum { M_WALK = 0, M_COUNT = 1, M_FINAL = 2 };

// A board's search state besides its planes: depth, and `mst` = passes on
// this board (bits 0-23) | mode << 24 | a completion kept (bit 26).
enum : uint32_t { MST_PASSES = 0xFFFFFFu, MST_FOUND = 1u << 26 };
PS_FN int mst_mode(uint32_t mst) { return (int)((mst >> 24) & 3u); }
PS_FN uint32_t mst_set_mode(uint32_t mst, int mode) { return (mst & MST_PASSES) | ((uint32_t)mode << 24); }

enum { S_CONT = 0, S_SOLVED = 1, S_NONE = 2, S_DEEP = 3 };

// A board whose propagated root still has at least SDK_PLANE_ROOT_OPEN
// undetermined cells starts in M_COUNT at once (0: never; only when the
// switch is on at all, mrv_after != 0).  Propagation that settles almost
// nothing at the root (17 clues, 60+ open cells: a quarter of the corpus)
// leaves the walk's fixed cell order nothing to lean on, and the
// fewest-candidates count is cheaper there; boards the root propagation
// opens up keep the walk's quick answers.
#ifndef SDK_PLANE_ROOT_OPEN
#define SDK_PLANE_ROOT_OPEN 58
#endif
// A backtrack that takes a level's LAST untried digit leaves the level
// exhausted: with SDK_PLANE_LASTPOP the search then continues at that
// level's depth (the next guess overwrites its line) instead of one deeper,
// so its entry is not rewritten and a later backtrack does not load it to
// find nothing there.  Level 0 is kept (it holds the propagated root the
// completion count and the final walk restart from).  The visiting order --
// and so every answer -- is the same; only the stack levels in use shrink.
#ifndef SDK_PLANE_LASTPOP
#define SDK_PLANE_LASTPOP 1
#endif
PS_FN bool root_counts(int mode, uint32_t depth, uint32_t mrv_after, uint32_t u0, uint32_t u1, uint32_t u2)
{
    return SDK_PLANE_ROOT_OPEN && mrv_after && mode == M_WALK && depth == 0 &&
           __builtin_popcount(u0) + __builtin_popcount(u1) + __builtin_popcount(u2) >= SDK_PLANE_ROOT_OPEN;
}

// One search step after a pass with result r (the lane solver's, and the
// plane kernel's lane loop: both call this).  Stack: push(level, B, entry),
// pop(level, B) -> entry (the level's planes into B, entry with them),
// put_entry(level, e).  Returns S_CONT (pass again), S_SOLVED
// (B holds the answer), S_NONE (no completion) or S_DEEP (deeper than the
// stack: the board goes to the wave kernel).  mrv_after: passes before the
// switch to the completion count (0 never).  guesses: +1 per branch node.
template <class Stack>
PS_FN int search_step(Board &B, const uint32_t (&und)[3], int r, uint32_t &depth, uint32_t &mst, const Stack &stk,
                      int node_order, uint32_t max_depth, uint32_t mrv_after, uint32_t &guesses)
{
    mst++;
    int mode = mst_mode(mst);
    if (r == STUCK && root_counts(mode, depth, mrv_after, und[0], und[1], und[2])) {
        mode = M_COUNT;  // count from the root, branching right here
        mst = mst_set_mode(mst, M_COUNT);
    }
    const uint32_t sol_level = max_depth - 1;  // M_COUNT keeps its first completion here
    // every plane load of the step at one site (the end): the level whose
    // planes replace the board's -- the next untried digit's, the root, or
    // a kept completion (one site keeps the kernel's registers in bounds)
    int reload = -1, save = -1;  // and the one plane store: a guess's level, or the kept completion
    uint32_t save_entry = 0;
    bool fix = false, fresh = false, last = false;
    int fix_band = 0, fix_pos = 0, res = S_CONT;
    uint32_t fix_d = 0;
    if (mode == M_WALK && mrv_after && r != SOLVED && (mst & MST_PASSES) >= mrv_after) {
        reload = depth ? 0 : -1;  // the propagated root (level 0's planes)
        fresh = true;
        depth = 0;
        mst = mst_set_mode(mst, M_COUNT);
        r = OPEN;
    }
    if (r == SOLVED) {
        if (mode != M_COUNT) return S_SOLVED;
        if (mst & MST_FOUND) {  // a second completion: the walk decides, from the root
            reload = 0;
            depth = 0;
            mst = mst_set_mode(mst, M_FINAL);
            r = OPEN;
        } else {
            mst |= MST_FOUND;
            save = (int)sol_level;
            r = DEAD;  // and look for another
        }
    }
    if (r == STUCK) {
        if (depth == (mode == M_COUNT ? sol_level : max_depth)) {
            if (mode != M_COUNT) return S_DEEP;
            reload = 0;  // too deep to count: the walk, from the root
            depth = 0;
            mst = mst_set_mode(mst, M_FINAL);
        } else {
            if (mode == M_COUNT) pick_mrv(B, und, fix_band, fix_pos);
            else pick_cell(und, node_order, fix_band, fix_pos);
            const uint32_t cand = cell_cand(B, fix_band, fix_pos);
            fix_d = cand & (0u - cand);
            save = (int)depth;
            save_entry = make_entry(fix_band, fix_pos, cand ^ fix_d);
            fix = true;
        }
    }
    // DEAD: back to the deepest level with an untried digit, scanning down
    // from depth - 1 (each level's planes and entry in one load)
    bool scan = false;
    if (r == DEAD) {
        if (depth) {
            scan = true;
            reload = (int)depth - 1;
        } else {
            if (mode != M_COUNT || !(mst & MST_FOUND)) return S_NONE;
            reload = (int)sol_level;  // exactly one completion
            res = S_SOLVED;
        }
    }
    if (save >= 0) stk.push((uint32_t)save, B, save_entry);
    if (reload >= 0 || fresh) B.Det[0] = B.Det[1] = B.Det[2] = 0;
    while (reload >= 0) {
        const uint32_t e = stk.pop((uint32_t)reload, B);
        if (!scan) break;
        const uint32_t rem = (e >> 8) & 0x1FFu;
        if (rem) {
            fix_d = rem & (0u - rem);
#if SDK_PLANE_LASTPOP
            last = rem == fix_d && reload > 0;  // the level's last digit: continue at its depth, entry untouched
            if (!last)
#endif
                stk.put_entry((uint32_t)reload, e & ~(fix_d << 8));
            fix_band = (int)((e >> 5) & 3u);
            fix_pos = (int)(e & 31u);
            depth = (uint32_t)reload;
            fix = true;
            break;
        }
        if (reload == 0) {  // the search is exhausted
            if (mode == M_COUNT && (mst & MST_FOUND)) {  // exactly one completion
                reload = (int)sol_level;
                scan = false;
                res = S_SOLVED;
                continue;
            }
            return S_NONE;
        }
        reload--;
    }
    // a guess and a backtrack both end by fixing one cell to one digit: one
    // set_cell for both groups of lanes (the wave runs both paths in most
    // iterations)
    if (fix) {
        depth += last ? 0u : 1u;
        guesses++;
        set_cell(B, fix_band, fix_pos, fix_d);
    }
    return res;
}

// the step's stack interface over a word stack with put(level, k, v) / get(level, k)
template <typename S>
struct WordStack {
    S &s;
    PS_MF void push(uint32_t level, const Board &B, uint32_t entry) const
    {
        save(level, B);
        s.put(level, STACK_ENTRY, entry);
    }
    PS_MF uint32_t pop(uint32_t level, Board &B) const
    {
        load(level, B);
        return s.get(level, STACK_ENTRY);
    }
    PS_MF void put_entry(uint32_t level, uint32_t e) const { s.put(level, STACK_ENTRY, e); }
    PS_MF void load(uint32_t level, Board &B) const
    {
        for (int w = 0; w < 27; ++w) B.P[w / 3][w % 3] = s.get(level, w);
    }
    PS_MF void save(uint32_t level, const Board &B) const
    {
        for (int w = 0; w < 27; ++w) s.put(level, w, B.P[w / 3][w % 3]);
    }
};

// Host / reference driver: solve one board in place with a stack of at
// least max_depth levels.  Returns 1 solved, 0 no completion, -1 depth
// overflow (board left to the wave kernel).
struct Stats {
    uint32_t guesses, passes;
};

template <typename Stack>
PS_FN int solve(Board &B, Stack &stk, int node_order, uint32_t max_depth, Stats &st, uint32_t mrv_after = 0)
{
    const WordStack<Stack> ws = {stk};
    uint32_t depth = 0, mst = 0;
    for (;;) {
        uint32_t und[3];
        const int r = pass(B, und);
        st.passes++;
        const int s = search_step(B, und, r, depth, mst, ws, node_order, max_depth, mrv_after, st.guesses);
        if (s == S_CONT) continue;
        return s == S_SOLVED ? 1 : s == S_NONE ? 0 : -1;
    }
}

}  // namespace plane

#endif  // SDK_PLANE_SOLVER_H
