// Host build of sudoku_solver_distributed_amd/csrc/plane_solver.h for the CPU
// test-suite (tests/test_plane_solver.py): the digit-plane lane solver is
// checked against the oracle before the GPU runs it.  Not a product path.
#include <stdint.h>
#include <string.h>
#include "../../sudoku_solver_distributed_amd/csrc/plane_solver.h"

struct HostStack {
    uint32_t w[82 * plane::STACK_WORDS];
    void put(uint32_t d, int k, uint32_t v) { w[d * plane::STACK_WORDS + k] = v; }
    uint32_t get(uint32_t d, int k) const { return w[d * plane::STACK_WORDS + k]; }
};

static void words_of(const uint8_t *src, uint32_t (&x)[21])
{
    uint8_t buf[84] = {0};
    memcpy(buf, src, 81);
    for (int k = 0; k < 21; ++k)
        x[k] = (uint32_t)buf[4 * k] | ((uint32_t)buf[4 * k + 1] << 8) | ((uint32_t)buf[4 * k + 2] << 16) |
               ((uint32_t)buf[4 * k + 3] << 24);
}

// the search-mode switch of plane::solve (0 = the walk only), for every
// solve below
static uint32_t g_mrv_after = 0;
extern "C" void plane_set_mrv_after(uint32_t k) { g_mrv_after = k; }

// status: 1 solved, 0 no completion, -1 invalid byte, 2 left to the wave
// kernel (clashing givens or depth overflow)
extern "C" void plane_solve_batch(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n, int node_order,
                                  uint32_t max_depth, uint64_t *guesses, uint64_t *passes)
{
    static HostStack stk;
    uint64_t g = 0, p = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t *src = in + i * 81;
        uint8_t *dst = out + i * 81;
        uint32_t x[21];
        words_of(src, x);
        plane::Board B;
        bool clash = false;
        memcpy(dst, src, 81);
        if (!plane::load_words(B, x, clash)) { status[i] = -1; continue; }
        if (clash) { status[i] = 2; continue; }
        plane::Stats st = {0, 0};
        const int r = plane::solve(B, stk, node_order, max_depth, st, g_mrv_after);
        g += st.guesses;
        p += st.passes;
        if (r == 1) plane::store_values(B, [&](int c, uint32_t v) { dst[c] = (uint8_t)v; });
        status[i] = r == 1 ? 1 : r == 0 ? 0 : 2;
    }
    *guesses = g;
    *passes = p;
}

// load_words against a plain per-byte loader; returns the number of boards
// whose planes / validity / clash flag differ.
extern "C" int64_t plane_check_load(const uint8_t *in, int64_t n)
{
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t *src = in + i * 81;
        uint32_t x[21];
        words_of(src, x);
        plane::Board B;
        bool clash = false;
        const bool ok = plane::load_words(B, x, clash);
        bool want_ok = true;
        uint32_t P[9][3] = {};
        int seen[27][10] = {};
        bool want_clash = false;
        for (int c = 0; c < 81; ++c) {
            const int v = src[c];
            if (v > 9) { want_ok = false; continue; }
            const int b = plane::cell_band(c), pos = plane::cell_pos(c);
            for (int d = 0; d < 9; ++d)
                if (v == 0 || v == d + 1) P[d][b] |= 1u << pos;
            if (v) {
                const int r = c / 9, col = c % 9, bx = (r / 3) * 3 + col / 3;
                want_clash |= seen[r][v]++ > 0;
                want_clash |= seen[9 + col][v]++ > 0;
                want_clash |= seen[18 + bx][v]++ > 0;
            }
        }
        bool diff = ok != want_ok;
        if (ok && want_ok) {
            diff |= clash != want_clash;
            for (int d = 0; d < 9; ++d)
                for (int b = 0; b < 3; ++b) diff |= B.P[d][b] != P[d][b];
        }
        bad += diff;
    }
    return bad;
}

// per-board passes / guesses / deepest stack level of the plane solver
// (scripts/make_hard_search.py filters search-heavy boards with it)
struct DepthStack {
    HostStack s;
    uint32_t max_depth = 0;
    void put(uint32_t d, int k, uint32_t v) { s.put(d, k, v); if (d + 1 > max_depth) max_depth = d + 1; }
    uint32_t get(uint32_t d, int k) const { return s.get(d, k); }
};

extern "C" void plane_solve_stats(const uint8_t *in, int64_t n, int node_order, int32_t *passes, int32_t *guesses,
                                  int32_t *depth)
{
    static DepthStack stk;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t x[21];
        words_of(in + i * 81, x);
        plane::Board B;
        bool clash = false;
        passes[i] = guesses[i] = depth[i] = -1;
        if (!plane::load_words(B, x, clash) || clash) continue;
        plane::Stats st = {0, 0};
        stk.max_depth = 0;
        plane::solve(B, stk, node_order, 81, st, g_mrv_after);
        passes[i] = (int32_t)st.passes;
        guesses[i] = (int32_t)st.guesses;
        depth[i] = (int32_t)stk.max_depth;
    }
}

// ---- the round-2 (pre-bitop3) formulation of plane::pass, restated as the
// checker of the full-rate rewrite: both must leave the same board state and
// return the same verdict after every pass (test-only).
namespace v1 {
using namespace plane;
static uint32_t spread(uint32_t c) { return c | (c << 10) | (c << 20); }
static uint32_t grows(uint32_t g) { return g - (g >> 9); }
static uint32_t rnz(uint32_t y) { return (y + ROWS) & GUARDS; }
static uint32_t fold(uint32_t y) { return (y | (y >> 10) | (y >> 20)) & 0x1FFu; }
static int pass(Board &B, uint32_t und[3])
{
    uint32_t single[3], nd[3], dead = 0;
    for (int b = 0; b < 3; ++b) {
        uint32_t o = 0, t = 0;
        for (int d = 0; d < 9; ++d) {
            t |= o & B.P[d][b];
            o |= B.P[d][b];
        }
        dead |= ROWS & ~o;
        single[b] = o & ~t;
        nd[b] = single[b] & ~B.Det[b];
        B.Det[b] = single[b];
        und[b] = ROWS & ~single[b];
    }
    const bool all_single = (single[0] & single[1] & single[2]) == ROWS;
    const bool any_nd = (nd[0] | nd[1] | nd[2]) != 0;
    uint32_t hall[3] = {0u, 0u, 0u}, hgrp[3] = {0u, 0u, 0u};
    uint32_t rowall = GUARDS, colall = 0x1FFu, boxall = BOXC;
    for (int d = 0; d < 9; ++d) {
        if (d >= SDK_PLANE_GROUP)  // the singles of the earlier groups' digits
            for (int b = 0; b < 3; ++b) B.P[d][b] &= ~hgrp[b];
        uint32_t x[3], f[3];
        for (int b = 0; b < 3; ++b) {
            x[b] = nd[b] & B.P[d][b];
            f[b] = fold(x[b]);
        }
        const uint32_t cpeer = spread(f[0] | f[1] | f[2]);
        for (int b = 0; b < 3; ++b) {
            const uint32_t g = f[b] | (f[b] >> 1) | (f[b] >> 2);
            const uint32_t peer = grows(rnz(x[b])) | cpeer | spread((g & BOXC) * 7u);
            B.P[d][b] = (peer & x[b]) | (~peer & B.P[d][b]);
        }
        uint32_t o[3], t[3], hb[3];
        for (int b = 0; b < 3; ++b) {
            const uint32_t y = B.P[d][b];
            const uint32_t nzy = rnz(y), nzm = rnz(y & (y + KDEC));
            rowall &= nzy;
            const uint32_t hr = y & grows(nzy & ~nzm);
            const uint32_t s1 = y >> 10, s2 = y >> 20;
            o[b] = (y | s1 | s2) & 0x1FFu;
            t[b] = ((y & s1) | (s2 & (y | s1))) & 0x1FFu;
            const uint32_t o1 = o[b] >> 1, o2 = o[b] >> 2;
            const uint32_t ob = o[b] | o1 | o2;
            const uint32_t tb = t[b] | (t[b] >> 1) | (t[b] >> 2) | (o[b] & o1) | (o2 & (o[b] | o1));
            boxall &= ob;
            hb[b] = hr | (y & spread((ob & ~tb & BOXC) * 7u));
        }
        const uint32_t O = o[0] | o[1] | o[2];
        const uint32_t T = t[0] | t[1] | t[2] | (o[0] & o[1]) | (o[2] & (o[0] | o[1]));
        colall &= O;
        const uint32_t hcol = spread(O & ~T);
#if SDK_PLANE_LC
        // rule D: a box whose places lie in one column takes d out of that
        // column in the other bands; one whose places lie in one row, out of
        // that row in the other boxes
        uint32_t vcol[3] = {0u, 0u, 0u};
        for (int b = 0; b < 3; ++b)
            for (int j = 0; j < 3; ++j) {
                const uint32_t c = (o[b] >> (3 * j)) & 7u;
                if (c && !(c & (c - 1))) vcol[b] |= c << (3 * j);
            }
        for (int b = 0; b < 3; ++b) {
            uint32_t cols = 0;
            for (int e = 0; e < 3; ++e)
                if (e != b) cols |= vcol[e];
            uint32_t ec = 0;
#if SDK_PLANE_LC & 1
            ec = cols & ~vcol[b];
#endif
#if SDK_PLANE_LC & 4
            // a column whose places lie in this band only: the other columns
            // of its box (all of the band's such columns kept)
            uint32_t claimed = 0;
            for (int c = 0; c < 9; ++c) {
                int bands = 0;
                for (int e = 0; e < 3; ++e)
                    if ((o[e] >> c) & 1u) bands |= 1 << e;
                if (bands == (1 << b)) claimed |= 1u << c;
            }
            for (int j = 0; j < 3; ++j)
                if ((claimed >> (3 * j)) & 7u) ec |= (7u << (3 * j)) & ~claimed;
#endif
            uint32_t m = spread(ec);
            B.P[d][b] &= ~m;
        }
#endif
        for (int b = 0; b < 3; ++b) {
            const uint32_t hd = (hb[b] | hcol) & B.P[d][b];  // (after rule D)
            B.P[d][b] = (B.P[d][b] & ~hall[b]) | hd;  // this group's lower digits' singles leave, d's own stay
            hall[b] |= hd;
        }
        if (d % SDK_PLANE_GROUP == SDK_PLANE_GROUP - 1)
            for (int b = 0; b < 3; ++b) hgrp[b] = hall[b];
    }
    for (int b = 0; b < 3; ++b) {
        uint32_t later = B.P[8][b];
        for (int e = 7; e >= 0; --e) {
            B.P[e][b] &= ~(hall[b] & later);
            if (e) later |= B.P[e][b];
        }
    }
#if SDK_PLANE_LC & 2
    // rule D, box -> row, after the digit loop: a box whose places lie in
    // one row takes the digit out of that row outside the boxes pointing
    // into it (two boxes into one row: both kept)
    for (int d = 0; d < 9; ++d)
        for (int b = 0; b < 3; ++b) {
            uint32_t into[3] = {0u, 0u, 0u}, m = 0;
            for (int j = 0; j < 3; ++j) {
                int rows = 0;
                for (int k = 0; k < 3; ++k)
                    if ((B.P[d][b] >> (10 * k + 3 * j)) & 7u) rows |= 1 << k;
                if (rows && !(rows & (rows - 1))) into[__builtin_ctz(rows)] |= 7u << (3 * j);
            }
            for (int k = 0; k < 3; ++k)
                if (into[k]) m |= (0x1FFu & ~into[k]) << (10 * k);
            B.P[d][b] &= ~m;
        }
#endif
    dead |= (rowall ^ GUARDS) | (colall ^ 0x1FFu) | ((boxall & BOXC) ^ BOXC);
    if (dead) return DEAD;
    if (all_single) return SOLVED;
    const bool newh = ((hall[0] & und[0]) | (hall[1] & und[1]) | (hall[2] & und[2])) != 0;
    return (any_nd || newh) ? OPEN : STUCK;  // (rule D alone does not count, as plane::pass)
}
}  // namespace v1

static bool same_state(const plane::Board &a, const plane::Board &b, const uint32_t (&ua)[3], const uint32_t (&ub)[3])
{
    for (int d = 0; d < 9; ++d)
        for (int k = 0; k < 3; ++k)
            if (a.P[d][k] != b.P[d][k]) return false;
    for (int k = 0; k < 3; ++k)
        if (a.Det[k] != b.Det[k] || ua[k] != ub[k]) return false;
    return true;
}

// Step plane::pass and v1::pass side by side from (a) each board's loaded
// planes, branching on the first undetermined cell at a fixpoint, and (b)
// `nrand` random plane states (any bits in the cell positions, random Det):
// returns the number of passes whose state or verdict differ.
extern "C" int64_t plane_check_pass(const uint8_t *in, int64_t n, int64_t nrand, uint64_t seed)
{
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t x[21];
        words_of(in + i * 81, x);
        plane::Board A, B;
        bool clash = false;
        if (!plane::load_words(A, x, clash)) continue;
        B = A;
        for (int step = 0; step < 400; ++step) {
            uint32_t ua[3], ub[3];
            const int ra = plane::pass(A, ua), rb = v1::pass(B, ub);
            if (ra != rb || !same_state(A, B, ua, ub)) { bad++; break; }
            if (ra == plane::DEAD || ra == plane::SOLVED) break;
            if (ra == plane::STUCK) {
                int band, pos;
                plane::pick_cell(ua, 0, band, pos);
                const uint32_t cand = plane::cell_cand(A, band, pos);
                const uint32_t d = cand & (0u - cand);
                plane::set_cell(A, band, pos, d);
                plane::set_cell(B, band, pos, d);
            }
        }
    }
    uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)(s >> 11); };
    for (int64_t i = 0; i < nrand; ++i) {
        plane::Board A;
        const int density = (int)(rnd() % 4);  // sparse to dense planes
        for (int d = 0; d < 9; ++d)
            for (int k = 0; k < 3; ++k) {
                uint32_t w = rnd();
                for (int j = 0; j < density; ++j) w |= rnd();
                A.P[d][k] = w & plane::ROWS;
            }
        for (int k = 0; k < 3; ++k) A.Det[k] = (rnd() & rnd()) & plane::ROWS;
        plane::Board B = A;
        for (int step = 0; step < 8; ++step) {
            uint32_t ua[3], ub[3];
            const int ra = plane::pass(A, ua), rb = v1::pass(B, ub);
            if (ra != rb || !same_state(A, B, ua, ub)) { bad++; break; }
        }
    }
    return bad;
}

// per-board pass and guess counts (scripts/drain_sim.py: the pass-count
// distribution the plane kernel's scheduling sees)
extern "C" void plane_board_passes(const uint8_t *in, int64_t n, int node_order, uint32_t *passes, uint32_t *guesses)
{
    static HostStack stk;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t x[21];
        words_of(in + i * 81, x);
        plane::Board B;
        bool clash = false;
        passes[i] = guesses[i] = 0;
        if (!plane::load_words(B, x, clash) || clash) continue;
        plane::Stats st = {0, 0};
        plane::solve(B, stk, node_order, 81, st, g_mrv_after);
        passes[i] = st.passes;
        guesses[i] = st.guesses;
    }
}

