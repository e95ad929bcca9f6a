// peer_greedy.h -- the reference's HTTP /solve algorithm: node.py:534-557
// P2PNode.peer_sudoku_solve on a fresh single node (no peers: every cell
// task runs locally, node.py:443-449).  Host + device code (one thread per
// board on the GPU, sdk_peer_solve_batch; g++ for the CPU tests).
//
// It is a greedy loop, not a search: the empty cells are queued row-major
// (fill_task_queue, node.py:419-425); each popped cell takes the first digit
// is_valid_move accepts (solve_sudoku_destributed, node.py:76-80), and a cell
// with none is repaired by taking over a digit placed elsewhere in its row
// (validate_solution, node.py:477-532), or left empty.  The outer loop
// (node.py:429-464) stops once a repair fails or fewer than two cells are
// empty -- otherwise it spins forever, which is reported as PG_NO_RETURN.
// The answer is whatever board is left, valid or not; `validations` counts
// node.py's SudokuSolver.check calls (every is_valid_move and the final
// check), as node.py:87 does.
//
// A P2PNode keeps partial_solution and tried_numbers_by_position (node.py:
// 149, 167) from one /solve request to the next: peer_sudoku_solve resets
// initial_sudoku, sudoku and the task queue only (node.py:539-552), so the
// repair step of a later request can take over a digit "placed" in an
// earlier board.  That part of the state is NodeState; run() starts from it
// (a fresh node: all zero) and leaves it as node.py would.
#ifndef SDK_PEER_GREEDY_H
#define SDK_PEER_GREEDY_H

#include <stdint.h>

#ifdef __HIPCC__
#define PG_FN __host__ __device__ __forceinline__
#else
#define PG_FN static inline
#endif

namespace peer {

enum { PG_CHECK_FAILED = 0, PG_CHECKED = 1, PG_NO_RETURN = 2 };

// node.py:82-116 without the rate limiter: every row, column and box sums to 45
PG_FN bool sums45(const uint8_t *g)
{
    for (int u = 0; u < 9; ++u) {
        int r = 0, c = 0, b = 0;
        const int br = 3 * (u / 3), bc = 3 * (u % 3);
        for (int k = 0; k < 9; ++k) {
            r += g[9 * u + k];
            c += g[9 * k + u];
            b += g[9 * (br + k / 3) + bc + k % 3];
        }
        if (r != 45 || c != 45 || b != 45) return false;
    }
    return true;
}

// node.py:42-60 is_valid_move; counts the check() call it makes
PG_FN bool valid_move(const uint8_t *g, int row, int col, int num, int &checks)
{
    ++checks;
    if (sums45(g)) return true;
    const int br = 3 * (row / 3), bc = 3 * (col / 3);
    for (int k = 0; k < 9; ++k)
        if (g[9 * row + k] == num || g[9 * k + col] == num || g[9 * (br + k / 3) + bc + k % 3] == num)
            return false;
    return true;
}

// the node's state that outlives a request (the C ABI's SDK_PEER_STATE_BYTES
// record, byte for byte)
struct NodeState {
    uint8_t placed[81];      // partial_solution: digit the loop put in the cell, 0 = none
    uint8_t pad0[15];
    uint16_t tried[81][9];   // tried_numbers_by_position[(r,c)]: bit v-1 of [c'] = (r, c', v) tried
    uint8_t pad1[46];
};
static_assert(sizeof(NodeState) == 1600, "SDK_PEER_STATE_BYTES");

struct State {
    uint8_t sudoku[81], initial[81];
    NodeState node;
    uint8_t ring[128];       // task_queue: a deque of cell indices (never longer than 81)
    uint32_t head, tail;     // ring[head % 128] is the left end, ring[(tail - 1) % 128] the right
};

PG_FN void clear_node(NodeState &n)
{
    for (int k = 0; k < 81; ++k) {
        n.placed[k] = 0;
        for (int c = 0; c < 9; ++c) n.tried[k][c] = 0;
    }
}

PG_FN void push_left(State &s, int cell) { s.ring[(--s.head) & 127u] = (uint8_t)cell; }
PG_FN int pop_left(State &s) { return s.ring[(s.head++) & 127u]; }

// validate_solution for a cell with no accepted digit: node.py:487-532
PG_FN bool repair(State &s, int cell, int &checks)
{
    const int row = cell / 9, col = cell % 9;
    uint8_t temp[81];
    for (int k = 0; k < 81; ++k) temp[k] = s.sudoku[k];
    int cand[9], nc = 0;
    for (int c = 0; c < 9; ++c) {
        const int rc = 9 * row + c;
        if (c == col || !s.node.placed[rc]) continue;
        const int v = s.node.placed[rc];
        temp[rc] = 0;  // the zeros accumulate along the row, as in node.py:503
        if (valid_move(temp, row, col, v, checks) && v != s.initial[rc] && !((s.node.tried[cell][c] >> (v - 1)) & 1u))
            cand[nc++] = c;
    }
    const int br = 3 * (row / 3), bc = 3 * (col / 3);
    for (int k = 0; k < nc; ++k) {
        const int c = cand[k], rc = 9 * row + c, v = s.node.placed[rc];
        bool safe = true;
        for (int t = 0; t < 9 && safe; ++t)
            safe = temp[9 * row + t] != v && temp[9 * t + col] != v && temp[9 * (br + t / 3) + bc + t % 3] != v;
        if (safe) {
            s.sudoku[cell] = (uint8_t)v;
            s.node.placed[cell] = (uint8_t)v;
            s.node.placed[rc] = 0;
            s.node.tried[cell][c] |= (uint16_t)(1u << (v - 1));
            s.sudoku[rc] = 0;
            push_left(s, rc);
            return true;
        }
    }
    s.sudoku[cell] = 0;
    return false;
}

// The whole loop on s.sudoku (filled in by the caller) from the node state
// in s.node (clear_node() first for a fresh node); returns PG_*.
PG_FN int run(State &s, int &checks)
{
    checks = 0;
    s.head = s.tail = 64;
    for (int k = 0; k < 81; ++k) {
        s.initial[k] = s.sudoku[k];
        if (!s.sudoku[k]) s.ring[(s.tail++) & 127u] = (uint8_t)k;
    }
    bool flag = true;
    for (;;) {
        while (s.head != s.tail) {
            const int cell = pop_left(s), row = cell / 9, col = cell % 9;
            int num = 0;
            for (int d = 1; d <= 9 && !num; ++d)
                if (valid_move(s.sudoku, row, col, d, checks)) num = d;
            if (num) {
                if (valid_move(s.sudoku, row, col, num, checks)) {  // node.py:480 (same board: accepted)
                    s.sudoku[cell] = (uint8_t)num;
                    s.node.placed[cell] = (uint8_t)num;
                } else {
                    push_left(s, cell);
                }
            } else {
                flag = repair(s, cell, checks);  // flag = True on entry (node.py:490), False on failure
            }
        }
        if (!flag) break;
        int empty = 0;
        for (int k = 0; k < 81; ++k) empty += s.sudoku[k] == 0;
        if (empty < 2) break;
        return PG_NO_RETURN;  // nothing is queued and nothing changes: node.py spins forever
    }
    ++checks;  // node.py:466 self.solver.check(self.sudoku)
    return sums45(s.sudoku) ? PG_CHECKED : PG_CHECK_FAILED;
}

}  // namespace peer

#endif  // SDK_PEER_GREEDY_H
