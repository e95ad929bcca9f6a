// Host build of sudoku_solver_distributed_amd/csrc/plane_wide.h (the wave-wide
// tail solver of plane_kernel) for the CPU test-suite
// (tests/test_plane_solver.py): the same source, over an emulated 64-lane
// wave, is checked against the lane solver (plane_solver.h) and the oracle
// before the GPU runs it.  Not a product path.
#include <stdint.h>
#include <string.h>

#include <deque>
#include <vector>

#include "../../sudoku_solver_distributed_amd/csrc/plane_quad.h"
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
        wide::NoSplit hk;
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
// a random candidate between propagations).  Both passes are iterated to
// their first non-OPEN result.  Returns the number of states where the two
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
            while ((rl = plane::pass(B, ul)) == plane::OPEN) {}
            while ((rw = wide::pass(w, det, und, L)) == wide::OPEN) {}
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

// ---- split counting over an emulated tail pool (plane_kernel.h PoolHook /
// plane_pool_drain, the same wide::solve hooks): every board is handed to
// the pool after `lane_guesses` lane guesses; records are solved one at a
// time in FIFO order (the boards' records interleave), and a count-mode
// search deals the untried digits of its shallowest open level out as new
// records whenever the pseudo-random "a wave is hungry" signal fires (every
// chance with split_every 1).  The last subtree of a split board answers it:
// no completion / the one / the walk from the count's root.  Answers must be
// the lane solver's and the oracle's whatever the split schedule.
struct Desc {
    int out = 0, compl_ = 0;
    bool walk = false;
    int64_t board = 0;
    wide::V found, root;
};
struct Rec {
    wide::V w;
    int64_t board;
    uint32_t depth, mst, bguess;
    int desc;                       // -1: a whole board
    std::vector<uint32_t> stack;    // its stack levels (a whole board brings the lane's)
};

struct HostPool {
    std::deque<Rec> q;
    std::vector<Desc> descs;
    uint32_t rs, every;
    uint64_t splits = 0, records = 0;
    bool hungry()
    {
        rs ^= rs << 13;
        rs ^= rs >> 17;
        rs ^= rs << 5;
        return every <= 1 || rs % every == 0;
    }
};

struct HostHook {
    HostPool &pool;
    int64_t board;
    int desc;
    uint32_t sol_level;
    bool cancelled() const { return false; }
    void counting(bool) {}
    bool split() const { return desc >= 0; }
    bool completion(const wide::V &w)
    {
        Desc &D = pool.descs[desc];
        if (D.compl_++ == 0) D.found = w;
        return D.compl_ == 1;
    }
    bool abandoned() { return pool.descs[desc].compl_ >= 2 || pool.descs[desc].walk; }
    void need_walk() { pool.descs[desc].walk = true; }
    template <class Stack>
    void try_split(const wide::V &, uint32_t depth, uint32_t &mst, const Stack &stk, const wide::Lanes &L)
    {
        if (depth == 0 || !pool.hungry()) return;
        uint32_t e = 0;
        const uint64_t open = stk.open_levels(depth, e);
        if (!open) return;
        const uint32_t lvl = (uint32_t)__builtin_ctzll(open);
        const uint32_t rem = (e >> 8) & 0x1FFu;
        if (desc < 0) {
            Desc D;
            D.out = 1;
            D.board = board;
            D.root = stk.restore(0, L);
            if (mst & plane::MST_FOUND) {
                D.compl_ = 1;
                D.found = stk.restore(sol_level, L);
            }
            mst &= ~plane::MST_FOUND;
            pool.descs.push_back(D);
            desc = (int)pool.descs.size() - 1;
        }
        pool.splits++;
        const wide::V base = stk.restore(lvl, L);
        uint32_t left = rem;
        while (left) {
            const uint32_t dbit = left & (0u - left);
            left ^= dbit;
            Rec r;
            r.w = base;
            wide::set_cell(r.w, L, (int)((e >> 5) & 3u), (int)(e & 31u), dbit);
            r.board = board;
            r.depth = 0;
            r.mst = plane::mst_set_mode(0u, plane::M_COUNT);
            r.bguess = 0;
            r.desc = desc;
            r.stack.assign(MAX_LEVELS * LEVEL_WORDS, 0u);
            pool.q.push_back(std::move(r));
            pool.descs[desc].out++;
        }
        stk.put_entry(lvl, e & ~(rem << 8));
    }
};

// status: 1 solved, 0 no completion, -1 invalid byte, 2 left to the wave
// kernel; splits: split events, records: records solved
extern "C" void wide_split_solve_batch(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n, int node_order,
                                       uint32_t max_depth, uint32_t lane_guesses, uint32_t split_every, uint32_t seed,
                                       uint64_t *splits, uint64_t *records)
{
    const wide::Lanes L = wide::lanes();
    HostPool pool;
    pool.rs = seed * 2654435761u + 1u;
    pool.every = split_every;
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t *src = in + i * 81;
        uint8_t *dst = out + i * 81;
        memcpy(dst, src, 81);
        status[i] = 77;
        uint32_t x[21];
        words_of(src, x);
        plane::Board B;
        bool clash = false;
        if (!plane::load_words(B, x, clash)) { status[i] = -1; continue; }
        if (clash) { status[i] = 2; continue; }
        uint32_t depth = 0, lg = 0, mst = 0;
        int done = -2;
        const plane::WordStack<LineStack> ls = {lines};
        while (lg < lane_guesses) {
            uint32_t und[3];
            const int r = plane::pass(B, und);
            const int s = plane::search_step(B, und, r, depth, mst, ls, node_order, max_depth, g_mrv_after, lg);
            if (s == plane::S_CONT) continue;
            done = s == plane::S_SOLVED ? 1 : s == plane::S_NONE ? 0 : -1;
            break;
        }
        if (done == 1) {
            plane::store_values(B, [&](int c, uint32_t v) { dst[c] = (uint8_t)v; });
            status[i] = 1;
            continue;
        }
        if (done == 0) { status[i] = 0; continue; }
        if (done == -1) { status[i] = 2; continue; }
        Rec r;
        r.w = to_wave(B, L);
        r.board = i;
        r.depth = depth;
        r.mst = mst;
        r.bguess = lg;
        r.desc = -1;
        r.stack.assign(stack_words, stack_words + MAX_LEVELS * LEVEL_WORDS);  // the lane's stack goes along
        pool.q.push_back(std::move(r));
    }
    auto answer = [&](int r, const wide::V &w, int64_t b) {
        if (r == wide::W_SOLVED) {
            store_wave(w, L, out + b * 81);
            status[b] = 1;
        } else {
            status[b] = r == wide::W_UNSOLVABLE ? 0 : 2;
        }
    };
    while (!pool.q.empty()) {
        Rec rec = std::move(pool.q.front());
        pool.q.pop_front();
        pool.records++;
        const WStack stk = {rec.stack.data()};
        wide::Stats st = {0, 0, rec.bguess};
        HostHook hk = {pool, rec.board, rec.desc, max_depth - 1};
        wide::V w = rec.w;
        uint32_t depth = rec.depth, mst = rec.mst;
        int r = wide::solve(w, depth, stk, L, node_order, max_depth, st, hk, mst, g_mrv_after);
        if (r != wide::W_SUBTREE) {
            answer(r, w, rec.board);
            continue;
        }
        Desc &D = pool.descs[hk.desc];
        if (--D.out) continue;
        if (D.compl_ >= 2 || D.walk) {  // the walk decides, from the count's root
            std::vector<uint32_t> own(MAX_LEVELS * LEVEL_WORDS, 0u);
            const WStack os = {own.data()};
            wide::V fw = D.root;
            uint32_t d0 = 0, m0 = plane::mst_set_mode(0u, plane::M_FINAL);
            wide::Stats fs = {0, 0, 0};
            wide::NoSplit nh;
            answer(wide::solve(fw, d0, os, L, node_order, max_depth, fs, nh, m0, g_mrv_after), fw, D.board);
        } else {
            answer(D.compl_ == 1 ? wide::W_SOLVED : wide::W_UNSOLVABLE, D.found, D.board);
        }
    }
    *splits = pool.splits;
    *records = pool.records;
}

// ---- the four-board pass (plane_quad.h) against the lane pass: boards four
// at a time (row q = board 4k+q), from each loaded board and from `trials`
// random mid-search states, both passes iterated to their first non-OPEN
// result per board.  Returns the states where verdict, planes or
// undetermined cells differ, the same admitted exception as
// wide_check_fixpoint (a duplicated determined digit neither flags at once).
extern "C" int64_t quad_check_fixpoint(const uint8_t *in, int64_t n, int trials, uint32_t seed)
{
    const quad::Lanes QL = quad::lanes();
    int64_t bad = 0;
    uint32_t rs = seed * 2654435761u + 7u;
    auto rnd = [&rs]() { rs ^= rs << 13; rs ^= rs >> 17; rs ^= rs << 5; return rs; };
    for (int trial = 0; trial <= trials; ++trial) {
        for (int64_t i0 = 0; i0 < n; i0 += 4) {
            plane::Board B[4];
            bool ok[4] = {false, false, false, false};
            int rl[4] = {0, 0, 0, 0};
            uint32_t ul[4][3] = {};
            for (int q = 0; q < 4 && i0 + q < n; ++q) {
                uint32_t x[21];
                words_of(in + (i0 + q) * 81, x);
                bool clash = false;
                if (!plane::load_words(B[q], x, clash) || clash) continue;
                const int guesses = trial ? 1 + (int)(rnd() % 4) : 0;
                int r = plane::STUCK;
                for (int k = 0; k < guesses; ++k) {
                    while ((r = plane::pass(B[q], ul[q])) == plane::OPEN) {}
                    if (r != plane::STUCK) break;
                    int band, pos;
                    plane::pick_cell(ul[q], (int)(rnd() & 1u), band, pos);
                    uint32_t d = plane::cell_cand(B[q], band, pos);
                    for (uint32_t j = rnd() % (uint32_t)__builtin_popcount(d); j; --j) d &= d - 1;
                    plane::set_cell(B[q], band, pos, d & (0u - d));
                }
                ok[q] = r == plane::STUCK;
            }
            // the quad wave from the same states (Det carried over)
            wide::V w[3], det[3], und[3];
            for (int b = 0; b < 3; ++b) w[b] = det[b] = und[b] = wide::V(0u);
            for (int k = 0; k < 64; ++k) {
                const int q = k >> 4, d = k & 15;
                if (!ok[q] || d >= 9) continue;
                for (int b = 0; b < 3; ++b) {
                    w[b].x[k] = B[q].P[d][b];
                    det[b].x[k] = B[q].Det[b];
                }
            }
            for (int q = 0; q < 4; ++q)
                if (ok[q])
                    while ((rl[q] = plane::pass(B[q], ul[q])) == plane::OPEN) {}
            int rw[4] = {-1, -1, -1, -1};
            for (int it = 0; it < 200; ++it) {
                const wide::V r = quad::pass(w, det, und, QL);
                bool more = false;
                for (int q = 0; q < 4; ++q) {
                    if (!ok[q] || rw[q] >= 0) continue;
                    if (r.x[16 * q] != (uint32_t)quad::OPEN) rw[q] = (int)r.x[16 * q];
                    else more = true;
                    for (int k = 16 * q; k < 16 * q + 16; ++k)
                        if (r.x[k] != r.x[16 * q]) bad += 1000000;  // not row-uniform
                }
                if (!more) break;  // (a row past its verdict: STUCK / SOLVED are fixpoints, DEAD is not compared)
            }
            for (int q = 0; q < 4; ++q) {
                if (!ok[q]) continue;
                bool diff = rl[q] != rw[q];
                if (!diff && rl[q] == plane::STUCK) {
                    for (int d = 0; d < 9; ++d)
                        for (int b = 0; b < 3; ++b) diff |= w[b].x[16 * q + d] != B[q].P[d][b];
                    for (int b = 0; b < 3; ++b) diff |= und[b].x[16 * q] != ul[q][b];
                }
                if (diff) {
                    plane::Board E = B[q];
                    if (rw[q] == quad::STUCK)
                        for (int d = 0; d < 9; ++d)
                            for (int b = 0; b < 3; ++b) E.P[d][b] = w[b].x[16 * q + d];
                    bad += !determined_clash(E);
                }
            }
        }
    }
    return bad;
}
