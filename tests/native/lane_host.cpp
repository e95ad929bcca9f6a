// Host build of sudoku_solver_distributed_amd/csrc/lane_solver.h for the CPU
// test-suite (tests/test_lane_solver.py): the lane-per-board algorithm is
// checked against the oracle before the GPU runs it.  Not a product path.
#include <stdint.h>
#include <string.h>
#include <vector>
#include "../../sudoku_solver_distributed_amd/csrc/lane_solver.h"

struct HostStack {
    uint32_t w[lane::MAX_DEPTH * lane::STACK_WORDS];
    void put(uint32_t d, int k, uint32_t v) { w[d * lane::STACK_WORDS + k] = v; }
    uint32_t get(uint32_t d, int k) const { return w[d * lane::STACK_WORDS + k]; }
};

extern "C" void lane_solve_batch(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n, int node_order,
                                 uint64_t *guesses, uint64_t *passes)
{
    HostStack stk;
    uint64_t g = 0, p = 0;
    for (int64_t i = 0; i < n; ++i) {
        lane::Board b;
        lane::load(b, in + i * 81);
        lane::Stats st = {0, 0};
        const int ok = lane::solve(b, stk, node_order, st);
        if (ok) lane::store(b, out + i * 81);
        else memcpy(out + i * 81, in + i * 81, 81);
        status[i] = ok;
        g += st.guesses;
        p += st.passes;
    }
    *guesses = g;
    *passes = p;
}
