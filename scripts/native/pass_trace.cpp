// pass_trace.cpp -- per-board pass outcome sequences of the lane solver
// (plane_solver.h on the host), for scripts/wave_events.py: how often a wave
// of 64 lanes runs the push / pop paths, refills and stores.  Tooling only.
#include <stdint.h>
#include <string.h>
#include "../../sudoku_solver_distributed_amd/csrc/plane_solver.h"

struct HostStack {
    uint32_t w[82 * plane::STACK_WORDS];
    void put(uint32_t d, int k, uint32_t v) { w[d * plane::STACK_WORDS + k] = v; }
    uint32_t get(uint32_t d, int k) const { return w[d * plane::STACK_WORDS + k]; }
};

// trace[i * maxlen + k]: outcome of board i's pass k (0 OPEN, 1 DEAD = a
// backtrack, 2 SOLVED, 3 STUCK = a guess); len[i] passes (capped at maxlen)
extern "C" void pass_trace(const uint8_t *in, int64_t n, int node_order, uint8_t *trace, int maxlen, uint32_t *len)
{
    static HostStack stk;
    for (int64_t i = 0; i < n; ++i) {
        uint8_t buf[84] = {0};
        memcpy(buf, in + i * 81, 81);
        uint32_t x[21];
        for (int k = 0; k < 21; ++k)
            x[k] = (uint32_t)buf[4 * k] | ((uint32_t)buf[4 * k + 1] << 8) | ((uint32_t)buf[4 * k + 2] << 16) |
                   ((uint32_t)buf[4 * k + 3] << 24);
        plane::Board B;
        bool clash = false;
        len[i] = 0;
        if (!plane::load_words(B, x, clash) || clash) continue;
        uint32_t depth = 0, k = 0;
        uint8_t *t = trace + i * maxlen;
        for (;;) {
            uint32_t und[3];
            const int r = plane::pass(B, und);
            if (k < (uint32_t)maxlen) t[k] = (uint8_t)r;
            k++;
            if (r == plane::SOLVED) break;
            if (r == plane::OPEN) continue;
            if (r == plane::STUCK) {
                int band, pos;
                plane::pick_cell(und, node_order, band, pos);
                const uint32_t cand = plane::cell_cand(B, band, pos);
                const uint32_t d = cand & (0u - cand);
                for (int w = 0; w < 27; ++w) stk.put(depth, w, B.P[w / 3][w % 3]);
                stk.put(depth, plane::STACK_ENTRY, plane::make_entry(band, pos, cand ^ d));
                depth++;
                plane::set_cell(B, band, pos, d);
                continue;
            }
            bool found = false;
            while (depth) {
                depth--;
                const uint32_t e = stk.get(depth, plane::STACK_ENTRY);
                const uint32_t rem = (e >> 8) & 0x1FFu;
                if (!rem) continue;
                const uint32_t d = rem & (0u - rem);
                for (int w = 0; w < 27; ++w) B.P[w / 3][w % 3] = stk.get(depth, w);
                B.Det[0] = B.Det[1] = B.Det[2] = 0;
                stk.put(depth, plane::STACK_ENTRY, e & ~(d << 8));
                depth++;
                plane::set_cell(B, (int)((e >> 5) & 3u), (int)(e & 31u), d);
                found = true;
                break;
            }
            if (!found) break;
        }
        len[i] = k < (uint32_t)maxlen ? k : (uint32_t)maxlen;
    }
}

// Experiment: fewest-candidates branching (MRV) searching the WHOLE tree up
// to a second completion.  passes / guesses per board; count = completions
// found (capped at 2).
static int mrv_pick(const plane::Board &B, const uint32_t und[3], int &band, int &pos)
{
    int best = 99;
    for (int b = 0; b < 3; ++b)
        for (uint32_t w = und[b]; w; w &= w - 1) {
            const int p = __builtin_ctz(w);
            const int n = __builtin_popcount(plane::cell_cand(B, b, p));
            if (n < best) { best = n; band = b; pos = p; if (n == 2) return n; }
        }
    return best;
}

extern "C" void mrv_count(const uint8_t *in, int64_t n, uint32_t *passes, uint32_t *guesses, int32_t *count)
{
    static HostStack stk;
    for (int64_t i = 0; i < n; ++i) {
        uint8_t buf[84] = {0};
        memcpy(buf, in + i * 81, 81);
        uint32_t x[21];
        for (int k = 0; k < 21; ++k)
            x[k] = (uint32_t)buf[4 * k] | ((uint32_t)buf[4 * k + 1] << 8) | ((uint32_t)buf[4 * k + 2] << 16) |
                   ((uint32_t)buf[4 * k + 3] << 24);
        plane::Board B;
        bool clash = false;
        passes[i] = guesses[i] = 0;
        count[i] = -1;
        if (!plane::load_words(B, x, clash) || clash) continue;
        uint32_t depth = 0, np = 0, ng = 0;
        int cnt = 0;
        for (;;) {
            uint32_t und[3];
            int r = plane::pass(B, und);
            np++;
            if (r == plane::OPEN) continue;
            if (r == plane::STUCK) {
                int band = 0, pos = 0;
                mrv_pick(B, und, band, pos);
                const uint32_t cand = plane::cell_cand(B, band, pos);
                const uint32_t d = cand & (0u - cand);
                for (int w = 0; w < 27; ++w) stk.put(depth, w, B.P[w / 3][w % 3]);
                stk.put(depth, plane::STACK_ENTRY, plane::make_entry(band, pos, cand ^ d));
                depth++;
                ng++;
                plane::set_cell(B, band, pos, d);
                continue;
            }
            if (r == plane::SOLVED && ++cnt >= 2) break;
            bool found = false;  // DEAD or a first solution: backtrack
            while (depth) {
                depth--;
                const uint32_t e = stk.get(depth, plane::STACK_ENTRY);
                const uint32_t rem = (e >> 8) & 0x1FFu;
                if (!rem) continue;
                const uint32_t d = rem & (0u - rem);
                for (int w = 0; w < 27; ++w) B.P[w / 3][w % 3] = stk.get(depth, w);
                B.Det[0] = B.Det[1] = B.Det[2] = 0;
                stk.put(depth, plane::STACK_ENTRY, e & ~(d << 8));
                depth++;
                ng++;
                plane::set_cell(B, (int)((e >> 5) & 3u), (int)(e & 31u), d);
                found = true;
                break;
            }
            if (!found) break;
        }
        passes[i] = np;
        guesses[i] = ng;
        count[i] = cnt;
    }
}
