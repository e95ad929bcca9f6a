// root_features.cpp -- per-board features of the lane solver (plane_solver.h on
// the host) for scripts/order_sim.py: can a board's pass count be predicted
// before it is solved, and would a heavy-first board order shorten the end of
// a launch?  Tooling only.
#include <stdint.h>
#include <string.h>
#include "../../sudoku_solver_distributed_amd/csrc/plane_solver.h"

struct HostStack {
    uint32_t w[82 * plane::STACK_WORDS];
    void put(uint32_t d, int k, uint32_t v) { w[d * plane::STACK_WORDS + k] = v; }
    uint32_t get(uint32_t d, int k) const { return w[d * plane::STACK_WORDS + k]; }
};

static void words_of(const uint8_t *src, uint32_t x[21])
{
    uint8_t buf[84] = {0};
    memcpy(buf, src, 81);
    for (int k = 0; k < 21; ++k)
        x[k] = buf[4 * k] | (buf[4 * k + 1] << 8) | (buf[4 * k + 2] << 16) | ((uint32_t)buf[4 * k + 3] << 24);
}

static void count_open(const plane::Board &B, const uint32_t und[3], int &U, int &cs, int &bi)
{
    U = cs = bi = 0;
    for (int b = 0; b < 3; ++b)
        for (uint32_t w = und[b]; w; w &= w - 1) {
            const int c = __builtin_popcount(plane::cell_cand(B, b, __builtin_ctz(w)));
            U++;
            cs += c;
            bi += c == 2;
        }
}

// out[18 * i + ...]: 0 passes, 1 branch nodes (the kernel's search, switch at
// mrv_after), 2 passes to the root fixpoint, 3 open cells there, 4 two-candidate
// cells there, 5 candidates there; 6 + 3k.. (k = 0..3): open cells, candidates
// and pass result after k + 1 passes
extern "C" void root_features(const uint8_t *in, int64_t n, uint32_t mrv_after, int32_t *out)
{
    static HostStack stk;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t x[21];
        words_of(in + i * 81, x);
        plane::Board B;
        bool clash = false;
        int32_t *o = out + 18 * i;
        memset(o, 0, 18 * sizeof(int32_t));
        if (!plane::load_words(B, x, clash) || clash) continue;
        plane::Board R = B;
        uint32_t und[3];
        int r = plane::OPEN, rp = 0;
        for (int k = 0; k < 4 || r == plane::OPEN; ++k) {
            const int rk = plane::pass(R, und);
            if (r == plane::OPEN) {
                r = rk;
                rp++;
            }
            if (k < 4) {
                int U, cs, bi;
                count_open(R, und, U, cs, bi);
                o[6 + 3 * k] = U;
                o[7 + 3 * k] = cs;
                o[8 + 3 * k] = r;
            }
            if (k >= 3 && r != plane::OPEN) break;
        }
        // the root fixpoint itself (R may have run past it: recompute)
        plane::Board Q = B;
        for (int k = 0; k < rp; ++k) plane::pass(Q, und);
        count_open(Q, und, o[3], o[5], o[4]);
        o[2] = rp;
        plane::Stats st = {0, 0};
        plane::solve(B, stk, 0, 32, st, mrv_after);
        o[0] = (int32_t)st.passes;
        o[1] = (int32_t)st.guesses;
    }
}
