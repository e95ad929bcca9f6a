// Host build of sudoku_solver_distributed_amd/csrc/plane_wide.h (the wave-wide
// tail solver of plane_kernel) for the CPU test-suite
// (tests/test_plane_solver.py): the same source, over an emulated 64-lane
// wave, is checked against the lane solver (plane_solver.h) and the oracle
// before the GPU runs it.  Not a product path.
#include <stdint.h>
#include <string.h>


#include "../../sudoku_solver_distributed_amd/csrc/plane_wide.h"

enum { LEVEL_WORDS = 32, MAX_LEVELS = 82 };

// plane_kernel's per-lane stack line layout: word 3d+b = P[d][b], word 27 = entry
struct WStack {
    uint32_t *w;
    void push(uint32_t level, const wide::V &v, const wide::Lanes &L, uint32_t entry) const
    {
        for (int i = 0; i < 64; ++i)
            if ((L.valid.m >> i) & 1) w[level * LEVEL_WORDS + L.word.x[i]] = v.x[i];
        w[level * LEVEL_WORDS + plane::STACK_ENTRY] = entry;
    }
    uint32_t entry(uint32_t level) const { return w[level * LEVEL_WORDS + plane::STACK_ENTRY]; }
    wide::V restore(uint32_t level, const wide::Lanes &L) const
    {
        wide::V r(0u);
        for (int i = 0; i < 64; ++i)
            if ((L.valid.m >> i) & 1) r.x[i] = w[level * LEVEL_WORDS + L.word.x[i]];
        return r;
    }
    void put_entry(uint32_t level, uint32_t e) const { w[level * LEVEL_WORDS + plane::STACK_ENTRY] = e; }
    uint64_t open_levels(uint32_t depth, uint32_t &first) const
    {
        uint64_t m = 0;
        first = 0;
        for (uint32_t l = depth; l-- > 0;)
            if ((entry(l) >> 8) & 0x1FFu) {
                m |= 1ull << l;
                first = entry(l);
            }
        return m;
    }
};

// the search-mode switch (plane::search_step / wide::solve; 0 = the walk only)
static uint32_t g_mrv_after = 0;
extern "C" void wide_set_mrv_after(uint32_t k) { g_mrv_after = k; }

static uint32_t stack_words[MAX_LEVELS * LEVEL_WORDS];
// the same words as plane::WordStack's put / get
struct LineStack {
    void put(uint32_t level, int k, uint32_t v) { stack_words[level * LEVEL_WORDS + k] = v; }
    uint32_t get(uint32_t level, int k) const { return stack_words[level * LEVEL_WORDS + k]; }
};
static LineStack lines;

static void words_of(const uint8_t *src, uint32_t (&x)[21])
{
    uint8_t buf[84] = {0};
    memcpy(buf, src, 81);
    for (int k = 0; k < 21; ++k)
        x[k] = (uint32_t)buf[4 * k] | ((uint32_t)buf[4 * k + 1] << 8) | ((uint32_t)buf[4 * k + 2] << 16) |
               ((uint32_t)buf[4 * k + 3] << 24);
}

static wide::V to_wave(const plane::Board &B, const wide::Lanes &L)
{
    wide::V w(0u);
    for (int i = 0; i < 64; ++i)
        if ((L.valid.m >> i) & 1) w.x[i] = B.P[L.d.x[i]][L.b.x[i]];
    return w;
}

// the store path of plane_kernel's wide tail: value slices per band -> bytes
static void store_wave(const wide::V &w, const wide::Lanes &L, uint8_t *dst)
{
    wide::V s[4];
    wide::value_slices(w, L, s);
    for (int c = 0; c < 81; ++c) {
        const int b = plane::cell_band(c), p = plane::cell_pos(c);
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) v |= ((s[k].x[16 * b] >> p) & 1u) << k;
        dst[c] = (uint8_t)v;
    }
}

// Solve each board: `lane_guesses` guesses (or the whole search, if it ends
// first) on the lane solver, stepping exactly like plane_kernel, then the
// rest of the search on the wave-wide solver from the same state and stack.
// status: 1 solved, 0 no completion, -1 invalid byte, 2 left to the wave
// kernel (clashing givens or depth overflow).  passes_wide: wide passes.
extern "C" void wide_solve_batch(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n, int node_order,
                                 uint32_t max_depth, uint32_t lane_guesses, uint64_t *guesses, uint64_t *passes_lane,
                                 uint64_t *passes_wide)
{
    const WStack stk = {stack_words};
    const wide::Lanes L = wide::lanes();
    uint64_t g = 0, pl = 0, pw = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t *src = in + i * 81;
        uint8_t *dst = out + i * 81;
        memcpy(dst, src, 81);
        uint32_t x[21];
        words_of(src, x);
        plane::Board B;
        bool clash = false;
        if (!plane::load_words(B, x, clash)) { status[i] = -1; continue; }
        if (clash) { status[i] = 2; continue; }
        // ---- lane phase (plane_kernel's loop body: pass + plane::search_step)
        uint32_t depth = 0, lg = 0, mst = 0;
        int done = -2;  // -2: hand off
        const plane::WordStack<LineStack> ls = {lines};
        while (lg < lane_guesses) {
            uint32_t und[3];
            const int r = plane::pass(B, und);
            pl++;
            const int s = plane::search_step(B, und, r, depth, mst, ls, node_order, max_depth, g_mrv_after, lg);
            if (s == plane::S_CONT) continue;
            done = s == plane::S_SOLVED ? 1 : s == plane::S_NONE ? 0 : -1;
            break;
        }
        g += lg;
        if (done == 1) {
            plane::store_values(B, [&](int c, uint32_t v) { dst[c] = (uint8_t)v; });
            status[i] = 1;
            continue;
        }
        if (done == 0) { status[i] = 0; continue; }
        if (done == -1) { status[i] = 2; continue; }
        // ---- wide phase: same planes (Det dropped), same stack and depth
        wide::V w = to_wave(B, L);
        wide::Stats st = {0, 0, 0};
        wide::NoCancel hk;
        const int r = wide::solve(w, depth, stk, L, node_order, max_depth, st, hk, mst, g_mrv_after);
        g += st.guesses;
        pw += st.passes;
        if (r == wide::W_SOLVED) {
            store_wave(w, L, dst);
            status[i] = 1;
        } else {
            status[i] = r == wide::W_UNSOLVABLE ? 0 : 2;
        }
    }
    *guesses = g;
    *passes_lane = pl;
    *passes_wide = pw;
}

// Fixpoints of the wide pass against the lane pass, from each loaded board
// and from `trials` random mid-search states per board (random cells fixed to
// a random candidate between propagations).  Both passes are iterated until
// the state stops changing (a STUCK pass may still have removed places by
// rule D, which neither pass counts as progress; the orders differ, the
// closure does not).  Returns the number of states where the two
// disagree (verdict, planes or undetermined cells) and the STUCK side holds
// no two determined cells with one digit in a unit: such a pair is a
// contradiction neither rule set flags at once, and which pass meets it
// first depends on the order singles are applied (both stay sound).
static bool determined_clash(const plane::Board &E)
{
    uint32_t det[3];
    for (int b = 0; b < 3; ++b) {
        uint32_t o = 0, t = 0;
        for (int d = 0; d < 9; ++d) {
            t |= o & E.P[d][b];
            o |= E.P[d][b];
        }
        det[b] = o & ~t;
    }
    return plane::givens_clash(E, det);
}

extern "C" int64_t wide_check_fixpoint(const uint8_t *in, int64_t n, int trials, uint32_t seed)
{
    const wide::Lanes L = wide::lanes();
    int64_t bad = 0;
    uint32_t rs = seed * 2654435761u + 1u;
    auto rnd = [&rs]() { rs ^= rs << 13; rs ^= rs >> 17; rs ^= rs << 5; return rs; };
    for (int64_t i = 0; i < n; ++i) {
        uint32_t x[21];
        words_of(in + i * 81, x);
        plane::Board B0;
        bool clash = false;
        if (!plane::load_words(B0, x, clash) || clash) continue;
        for (int trial = 0; trial <= trials; ++trial) {
            plane::Board B = B0;
            uint32_t ul[3];
            int rl = plane::STUCK;
            const int guesses = trial ? 1 + (int)(rnd() % 4) : 0;
            for (int k = 0; k < guesses; ++k) {
                while ((rl = plane::pass(B, ul)) == plane::OPEN) {}
                if (rl != plane::STUCK) break;
                int band, pos;
                plane::pick_cell(ul, (int)(rnd() & 1u), band, pos);
                uint32_t d = plane::cell_cand(B, band, pos);
                for (uint32_t j = rnd() % (uint32_t)__builtin_popcount(d); j; --j) d &= d - 1;
                plane::set_cell(B, band, pos, d & (0u - d));
            }
            if (rl != plane::STUCK) continue;
            wide::V w = to_wave(B, L), det(0u), und;
            for (int k = 0; k < 64; ++k)
                if (L.b.x[k] < 3) det.x[k] = B.Det[L.b.x[k]];
            int rw;
            for (;;) {
                const plane::Board prev = B;
                rl = plane::pass(B, ul);
                if (rl == plane::OPEN || (rl == plane::STUCK && memcmp(prev.P, B.P, sizeof B.P) != 0)) continue;
                break;
            }
            for (;;) {
                const wide::V prev = w;
                rw = wide::pass(w, det, und, L);
                bool moved = false;
                for (int k = 0; k < 64; ++k) moved |= prev.x[k] != w.x[k];
                if (rw == wide::OPEN || (rw == wide::STUCK && moved)) continue;
                break;
            }
            bool diff = rl != rw;
            if (!diff && rl == plane::STUCK) {
                const wide::V want = to_wave(B, L);
                for (int k = 0; k < 64; ++k) diff |= want.x[k] != w.x[k];
                for (int b = 0; b < 3; ++b) diff |= ul[b] != und.x[16 * b];
            }
            if (diff) {
                plane::Board E = B;  // the STUCK side's planes
                if (rw == wide::STUCK)
                    for (int k = 0; k < 64; ++k)
                        if ((L.valid.m >> k) & 1) E.P[L.d.x[k]][L.b.x[k]] = w.x[k];
                bad += !determined_clash(E);
            }
        }
    }
    return bad;
}
