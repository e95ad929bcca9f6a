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
        const int r = plane::solve(B, stk, node_order, max_depth, st);
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
        plane::solve(B, stk, node_order, 81, st);
        passes[i] = (int32_t)st.passes;
        guesses[i] = (int32_t)st.guesses;
        depth[i] = (int32_t)stk.max_depth;
    }
}
