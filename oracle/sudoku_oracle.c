/*
 * sudoku_oracle.c -- CPU restatement of the reference's Sudoku algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * solver in sudoku_solver_distributed_amd/csrc.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path never does.
 *
 * Parity pinning: the restatement is checked against golden vectors produced
 * by importing the reference's own gen.py / sudoku.py / node.py
 * (tests/golden/make_golden.py writes the JSON fixtures, see tests/test_oracle.py).
 *
 * Grid layout everywhere: 81 bytes, row-major, 0 = empty, 1..9 = digit.
 *
 * Reference functions restated (cristiano-nicolau/sudoku_solver_distributed):
 *   oracle_is_valid        <- sudoku.py:60-78   Sudoku.check_is_valid
 *   oracle_check           <- sudoku.py:80-140  Sudoku.check_row/column/square/check
 *   oracle_check_sums      <- node.py:82-116    SudokuSolver.check (sums only)
 *   oracle_is_valid_move   <- node.py:42-60     SudokuSolver.is_valid_move
 *   oracle_solve           <- gen.py:6-28       solve_sudoku; NOTE its cell scan
 *                             (gen.py:11-15) `break`s only the inner loop, so it
 *                             branches on the first empty cell of the LAST row
 *                             holding one: rows 8..0, columns 0..8 ("gen order")
 *   oracle_solve_node      <- node.py:62-74     SudokuSolver.solve_sudoku_recursive
 *                             (first empty cell row-major: "node order")
 *   oracle_first_candidate <- node.py:76-80     SudokuSolver.solve_sudoku_destributed
 *   oracle_count_solutions    (test helper: uniqueness of generated puzzles)
 */
#include <stdint.h>
#include <string.h>

/* sudoku.py:60-78 -- num not in row, not in column, not in 3x3 box. */
int oracle_is_valid(const uint8_t *g, int row, int col, int num)
{
    for (int i = 0; i < 9; i++)
        if (g[row * 9 + i] == num || g[i * 9 + col] == num)
            return 0;
    int sr = 3 * (row / 3), sc = 3 * (col / 3);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            if (g[(sr + i) * 9 + sc + j] == num)
                return 0;
    return 1;
}

/* sudoku.py:85/95-98/108-113: sum(unit) == 45 and len(set(unit)) == 9 */
static int unit_ok_sum_set(const int *v)
{
    int sum = 0;
    int seen[256];
    memset(seen, 0, sizeof seen);
    int distinct = 0;
    for (int k = 0; k < 9; k++) {
        sum += v[k];
        if (!seen[v[k] & 255]) { seen[v[k] & 255] = 1; distinct++; }
    }
    return sum == 45 && distinct == 9;
}

/* sudoku.py:119-140 -- rows, then columns, then squares. */
int oracle_check(const uint8_t *g)
{
    int v[9];
    for (int r = 0; r < 9; r++) {
        for (int k = 0; k < 9; k++) v[k] = g[r * 9 + k];
        if (!unit_ok_sum_set(v)) return 0;
    }
    for (int c = 0; c < 9; c++) {
        for (int k = 0; k < 9; k++) v[k] = g[k * 9 + c];
        if (!unit_ok_sum_set(v)) return 0;
    }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            int n = 0;
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) v[n++] = g[(i * 3 + a) * 9 + j * 3 + b];
            if (!unit_ok_sum_set(v)) return 0;
        }
    return 1;
}

/* node.py:82-116 -- only the sums are checked (no distinctness). */
int oracle_check_sums(const uint8_t *g)
{
    for (int r = 0; r < 9; r++) {
        int s = 0;
        for (int k = 0; k < 9; k++) s += g[r * 9 + k];
        if (s != 45) return 0;
    }
    for (int c = 0; c < 9; c++) {
        int s = 0;
        for (int k = 0; k < 9; k++) s += g[k * 9 + c];
        if (s != 45) return 0;
    }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            int s = 0;
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) s += g[(i * 3 + a) * 9 + j * 3 + b];
            if (s != 45) return 0;
        }
    return 1;
}

/* node.py:42-60 -- is_valid_move short-circuits to True when check() passes,
 * then scans row+column together, then the box. */
int oracle_is_valid_move(const uint8_t *g, int row, int col, int num)
{
    if (oracle_check_sums(g)) return 1;
    return oracle_is_valid(g, row, col, num);
}

typedef int (*valid_fn)(const uint8_t *, int, int, int);

static _Thread_local uint64_t g_nodes; /* candidate tests (the reference's "validations"), per thread */

/* gen.py:11-15: `for i: for j: if empty: row, col = i, j; break` -- the
 * break leaves only the column loop, so the LAST row with an empty cell wins,
 * at its first empty column. */
static int gen_order_cell(const uint8_t *g)
{
    int cell = -1;
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++)
            if (g[i * 9 + j] == 0) { cell = i * 9 + j; break; }
    return cell;
}

/* node.py:63-65: first empty cell in row-major order (the loop returns). */
static int node_order_cell(const uint8_t *g)
{
    for (int i = 0; i < 81; i++)
        if (g[i] == 0) return i;
    return -1;
}

typedef int (*cell_fn)(const uint8_t *);

/* gen.py:6-28 / node.py:62-74 -- pick the branch cell, digits 1..9 ascending,
 * recursion; the board is restored to its input on failure. */
static int solve_rec(uint8_t *g, valid_fn valid, cell_fn pick)
{
    int cell = pick(g);
    if (cell < 0) return 1;
    int row = cell / 9, col = cell % 9;
    for (int num = 1; num <= 9; num++) {
        g_nodes++;
        if (valid(g, row, col, num)) {
            g[cell] = (uint8_t)num;
            if (solve_rec(g, valid, pick)) return 1;
            g[cell] = 0;
        }
    }
    return 0;
}

int oracle_solve(uint8_t *g)
{
    return solve_rec(g, oracle_is_valid, gen_order_cell);
}

/* gen.py's test (sudoku.py:60-78) with node.py's cell order: the kernel's
 * SDK_ORDER_NODE on boards whose givens do not clash. */
int oracle_solve_rowmajor(uint8_t *g)
{
    return solve_rec(g, oracle_is_valid, node_order_cell);
}

/* node.py:62-74 (same walk, node.py's is_valid_move as the test). */
int oracle_solve_node(uint8_t *g)
{
    return solve_rec(g, oracle_is_valid_move, node_order_cell);
}

uint64_t oracle_last_nodes(void) { return g_nodes; }
void oracle_reset_nodes(void) { g_nodes = 0; }

/* node.py:76-80 -- first digit 1..9 accepted by is_valid_move, or 0 (None). */
int oracle_first_candidate(const uint8_t *g, int row, int col)
{
    for (int num = 1; num <= 9; num++)
        if (oracle_is_valid_move(g, row, col, num)) return num;
    return 0;
}

/* Batch form of oracle_solve: in -> out (81 B each), status 1 = solved,
 * 0 = no solution (out = input, as gen.py leaves the board). */
void oracle_solve_batch(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n)
{
    for (int64_t p = 0; p < n; p++) {
        memcpy(out + p * 81, in + p * 81, 81);
        status[p] = oracle_solve(out + p * 81);
    }
}

void oracle_solve_batch_rowmajor(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n)
{
    for (int64_t p = 0; p < n; p++) {
        memcpy(out + p * 81, in + p * 81, 81);
        status[p] = oracle_solve_rowmajor(out + p * 81);
    }
}

/* Batch form of oracle_solve_node (node.py:62-74 with is_valid_move). */
void oracle_solve_batch_node(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n)
{
    for (int64_t p = 0; p < n; p++) {
        memcpy(out + p * 81, in + p * 81, 81);
        status[p] = oracle_solve_node(out + p * 81);
    }
}

/* Test helper: number of completions (up to `limit`) under the reference's
 * constraint (every empty cell differs from its filled peers). */
static int count_rec(uint8_t *g, int limit, int *count)
{
    int cell = -1;
    for (int i = 0; i < 81; i++)
        if (g[i] == 0) { cell = i; break; }
    if (cell < 0) { (*count)++; return *count >= limit; }
    int row = cell / 9, col = cell % 9;
    for (int num = 1; num <= 9; num++) {
        if (oracle_is_valid(g, row, col, num)) {
            g[cell] = (uint8_t)num;
            int stop = count_rec(g, limit, count);
            g[cell] = 0;
            if (stop) return 1;
        }
    }
    return 0;
}

int oracle_count_solutions(const uint8_t *g_in, int limit)
{
    uint8_t g[81];
    memcpy(g, g_in, 81);
    int count = 0;
    count_rec(g, limit, &count);
    return count;
}

/* Test helper: the same count with row/col/box bitmasks and
 * fewest-candidates branching -- used only to certify that generated
 * benchmark puzzles have a unique solution (order does not matter for a
 * count).  Same constraint as count_rec. */
static int fast_rec(uint8_t *g, uint16_t *rm, uint16_t *cm, uint16_t *bm,
                    int limit, int *count)
{
    int best = -1, bestn = 10;
    uint16_t bestc = 0;
    for (int i = 0; i < 81; i++) {
        if (g[i]) continue;
        int r = i / 9, c = i % 9, b = (r / 3) * 3 + c / 3;
        uint16_t cand = (uint16_t)(~(rm[r] | cm[c] | bm[b]) & 0x1FF);
        int n = __builtin_popcount(cand);
        if (n < bestn) { bestn = n; best = i; bestc = cand; if (n <= 1) break; }
    }
    if (best < 0) { (*count)++; return *count >= limit; }
    if (bestn == 0) return 0;
    int r = best / 9, c = best % 9, b = (r / 3) * 3 + c / 3;
    while (bestc) {
        int d = __builtin_ctz(bestc);
        bestc &= (uint16_t)(bestc - 1);
        uint16_t bit = (uint16_t)(1u << d);
        g[best] = (uint8_t)(d + 1);
        rm[r] |= bit; cm[c] |= bit; bm[b] |= bit;
        int stop = fast_rec(g, rm, cm, bm, limit, count);
        rm[r] &= (uint16_t)~bit; cm[c] &= (uint16_t)~bit; bm[b] &= (uint16_t)~bit;
        g[best] = 0;
        if (stop) return 1;
    }
    return 0;
}

int oracle_count_solutions_fast(const uint8_t *g_in, int limit)
{
    uint8_t g[81];
    uint16_t rm[9] = {0}, cm[9] = {0}, bm[9] = {0};
    memcpy(g, g_in, 81);
    for (int i = 0; i < 81; i++) {
        if (!g[i]) continue;
        int r = i / 9, c = i % 9, b = (r / 3) * 3 + c / 3;
        uint16_t bit = (uint16_t)(1u << (g[i] - 1));
        /* a duplicated given makes the reference's walk ignore the clash
         * (only empty cells are tested), so record it without failing */
        rm[r] |= bit; cm[c] |= bit; bm[b] |= bit;
    }
    int count = 0;
    fast_rec(g, rm, cm, bm, limit, &count);
    return count;
}

/* Test helper: fewest-candidates search that also returns the first
 * completion it meets and whether it is the only one (count up to 2).  For a
 * board with exactly one completion that completion is, necessarily, the
 * walk's (gen.py:6-28) answer -- lets tests pin hard 17-clue boards at
 * scale, where the literal walk needs up to ~1e9 candidate tests. */
static int uniq_rec(uint8_t *g, uint16_t *rm, uint16_t *cm, uint16_t *bm,
                    int *count, uint8_t *first)
{
    int best = -1, bestn = 10;
    uint16_t bestc = 0;
    for (int i = 0; i < 81; i++) {
        if (g[i]) continue;
        int r = i / 9, c = i % 9, b = (r / 3) * 3 + c / 3;
        uint16_t cand = (uint16_t)(~(rm[r] | cm[c] | bm[b]) & 0x1FF);
        int n = __builtin_popcount(cand);
        if (n < bestn) { bestn = n; best = i; bestc = cand; if (n <= 1) break; }
    }
    if (best < 0) {
        if (*count == 0) memcpy(first, g, 81);
        (*count)++;
        return *count >= 2;
    }
    if (bestn == 0) return 0;
    int r = best / 9, c = best % 9, b = (r / 3) * 3 + c / 3;
    while (bestc) {
        int d = __builtin_ctz(bestc);
        bestc &= (uint16_t)(bestc - 1);
        uint16_t bit = (uint16_t)(1u << d);
        g[best] = (uint8_t)(d + 1);
        rm[r] |= bit; cm[c] |= bit; bm[b] |= bit;
        int stop = uniq_rec(g, rm, cm, bm, count, first);
        rm[r] &= (uint16_t)~bit; cm[c] &= (uint16_t)~bit; bm[b] &= (uint16_t)~bit;
        g[best] = 0;
        if (stop) return 1;
    }
    return 0;
}

/* returns the number of completions capped at 2; out = first one found */
int oracle_solve_unique(const uint8_t *g_in, uint8_t *out)
{
    uint8_t g[81];
    uint16_t rm[9] = {0}, cm[9] = {0}, bm[9] = {0};
    memcpy(g, g_in, 81);
    memcpy(out, g_in, 81);
    for (int i = 0; i < 81; i++) {
        if (!g[i]) continue;
        int r = i / 9, c = i % 9, b = (r / 3) * 3 + c / 3;
        uint16_t bit = (uint16_t)(1u << (g[i] - 1));
        rm[r] |= bit; cm[c] |= bit; bm[b] |= bit;
    }
    int count = 0;
    uniq_rec(g, rm, cm, bm, &count, out);
    return count;
}

void oracle_solve_unique_batch(const uint8_t *in, uint8_t *out, int32_t *count, int64_t n)
{
    for (int64_t p = 0; p < n; p++) count[p] = oracle_solve_unique(in + p * 81, out + p * 81);
}

/* Test helper: the same count (to 2, first completion kept) with naked and
 * hidden singles propagated before each branch on a fewest-candidates cell.
 * Propagation only removes candidates no completion can use, so the
 * completions and their count are the plain search's (checked against
 * oracle_solve_unique in tests/test_oracle.py); hard 17-clue boards need
 * ~100x fewer nodes.  Givens that clash count 0 here where the plain
 * search (which never tests givens) may find fills: callers use it only on
 * boards whose givens do not clash. */
static int prop_singles(uint16_t *c)
{
    static const int U[27][9] = {
#define R(r) {9 * r, 9 * r + 1, 9 * r + 2, 9 * r + 3, 9 * r + 4, 9 * r + 5, 9 * r + 6, 9 * r + 7, 9 * r + 8}
        R(0), R(1), R(2), R(3), R(4), R(5), R(6), R(7), R(8),
#undef R
#define C(k) {k, 9 + k, 18 + k, 27 + k, 36 + k, 45 + k, 54 + k, 63 + k, 72 + k}
        C(0), C(1), C(2), C(3), C(4), C(5), C(6), C(7), C(8),
#undef C
#define B(b) {27 * (b / 3) + 3 * (b % 3), 27 * (b / 3) + 3 * (b % 3) + 1, 27 * (b / 3) + 3 * (b % 3) + 2, \
              27 * (b / 3) + 3 * (b % 3) + 9, 27 * (b / 3) + 3 * (b % 3) + 10, 27 * (b / 3) + 3 * (b % 3) + 11, \
              27 * (b / 3) + 3 * (b % 3) + 18, 27 * (b / 3) + 3 * (b % 3) + 19, 27 * (b / 3) + 3 * (b % 3) + 20}
        B(0), B(1), B(2), B(3), B(4), B(5), B(6), B(7), B(8),
#undef B
    };
    for (int changed = 1; changed;) {
        changed = 0;
        for (int i = 0; i < 81; i++) {
            if (!c[i]) return 0;
            if (c[i] & (c[i] - 1)) continue;
            const int r = i / 9, col = i % 9, b = (r / 3) * 3 + col / 3;
            const int *us[3] = {U[r], U[9 + col], U[18 + b]};
            for (int u = 0; u < 3; u++)
                for (int k = 0; k < 9; k++) {
                    const int p = us[u][k];
                    if (p != i && (c[p] & c[i])) {
                        c[p] &= (uint16_t)~c[i];
                        if (!c[p]) return 0;
                        changed = 1;
                    }
                }
        }
        for (int u = 0; u < 27; u++) {
            uint16_t once = 0, twice = 0;
            for (int k = 0; k < 9; k++) {
                twice |= once & c[U[u][k]];
                once |= c[U[u][k]];
            }
            if (once != 0x1FF) return 0;
            const uint16_t single = once & (uint16_t)~twice;
            for (int k = 0; single && k < 9; k++) {
                const int p = U[u][k];
                const uint16_t x = c[p] & single;
                if (x && c[p] != x) {
                    if (x & (x - 1)) return 0;
                    c[p] = x;
                    changed = 1;
                }
            }
        }
    }
    return 1;
}

static int uniqp_rec(uint16_t *c, int *count, uint8_t *first)
{
    if (!prop_singles(c)) return 0;
    int best = -1, bn = 10;
    for (int i = 0; i < 81; i++) {
        const int n = __builtin_popcount(c[i]);
        if (n > 1 && n < bn) { bn = n; best = i; if (n == 2) break; }
    }
    if (best < 0) {
        if (*count == 0)
            for (int i = 0; i < 81; i++) first[i] = (uint8_t)(__builtin_ctz(c[i]) + 1);
        (*count)++;
        return *count >= 2;
    }
    for (uint16_t m = c[best]; m; m &= (uint16_t)(m - 1)) {
        uint16_t s[81];
        memcpy(s, c, sizeof s);
        s[best] = m & (uint16_t)(0u - m);
        if (uniqp_rec(s, count, first)) return 1;
    }
    return 0;
}

int oracle_solve_unique_prop(const uint8_t *g_in, uint8_t *out)
{
    uint16_t c[81];
    memcpy(out, g_in, 81);
    for (int i = 0; i < 81; i++) c[i] = g_in[i] ? (uint16_t)(1u << (g_in[i] - 1)) : 0x1FF;
    int count = 0;
    uniqp_rec(c, &count, out);
    return count;
}

void oracle_solve_unique_prop_batch(const uint8_t *in, uint8_t *out, int32_t *count, int64_t n)
{
    for (int64_t p = 0; p < n; p++) count[p] = oracle_solve_unique_prop(in + p * 81, out + p * 81);
}

/* Timed batch walk for bench.py's cpu_baseline: solves boards in order until
 * `seconds` of wall time have elapsed; returns the number of boards fully
 * solved (a board cut off by the deadline is not counted). */
#include <time.h>
static _Thread_local double g_deadline; /* per thread: bench.py runs one walk per host core */
static _Thread_local int g_abort;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int solve_rec_timed(uint8_t *g)
{
    int cell = gen_order_cell(g);
    if (cell < 0) return 1;
    int row = cell / 9, col = cell % 9;
    for (int num = 1; num <= 9; num++) {
        if ((++g_nodes & 0xFFFFF) == 0 && now_s() > g_deadline) g_abort = 1;
        if (g_abort) return 0;
        if (oracle_is_valid(g, row, col, num)) {
            g[cell] = (uint8_t)num;
            if (solve_rec_timed(g)) return 1;
            if (g_abort) return 0;
            g[cell] = 0;
        }
    }
    return 0;
}

int64_t oracle_solve_batch_timed(const uint8_t *in, uint8_t *out, int32_t *status, int64_t n, double seconds)
{
    g_deadline = now_s() + seconds;
    g_abort = 0;
    int64_t done = 0;
    for (int64_t p = 0; p < n; p++) {
        memcpy(out + p * 81, in + p * 81, 81);
        status[p] = solve_rec_timed(out + p * 81);
        if (g_abort) break;
        done++;
        if (now_s() > g_deadline) break;
    }
    return done;
}

/* ------------------------------------------------------------------------
 * node.py:534-557 P2PNode.peer_sudoku_solve on a single node (no peers,
 * handicap 0): the reference's HTTP /solve path.  The node's
 * partial_solution and tried_numbers_by_position (node.py:149, 167) live in
 * the P2PNode and survive from one request to the next (peer_sudoku_solve
 * resets initial_sudoku, sudoku and the task queue only, node.py:539-552):
 * oracle_peer_solve_node takes them in and leaves them updated;
 * oracle_peer_solve is a fresh node (both empty).
 *   fill_task_queue (node.py:419-425): the empty cells, row-major;
 *   solve_sudoku (node.py:427-475): pop a cell, take the first digit that
 *     is_valid_move accepts (solve_sudoku_destributed, node.py:76-80; with
 *     no peers it runs locally, node.py:443-449), validate_solution;
 *   validate_solution (node.py:477-532): place the digit, or repair the cell
 *     by moving a digit placed elsewhere in its row (partial_solution /
 *     tried_numbers_by_position bookkeeping), or leave it empty (flag False);
 *   the outer `while True` (node.py:429-464) ends when flag is False, or when
 *     fewer than 2 cells are empty; otherwise it spins forever.
 * Returns 1 (final check() passed), 0 (board returned, check failed) or -1
 * (the reference never returns); *validations = node.py's counter: one per
 * SudokuSolver.check call (every is_valid_move, plus the final check).
 * ------------------------------------------------------------------------ */
static int g_val;

static int peer_valid_move(const uint8_t *g, int row, int col, int num)
{
    g_val++;  /* is_valid_move -> self.check(board) (node.py:44, 87) */
    return oracle_is_valid_move(g, row, col, num);
}

/* partial[cell] = digit placed by the loop, 0 = absent (partial_solution);
 * tried[(row,col)][c*9 + v-1]: (row, c, v) in tried_numbers_by_position[(row,
 * col)] (the row is implied: node.py:523 adds (r, c, value) with r == row) */
int oracle_peer_solve_node(uint8_t *sudoku, int32_t *validations, uint8_t partial[81], uint8_t tried[81][81])
{
    uint8_t initial[81];
    int queue[1024], qh = 512, qt = 512; /* deque: popleft at qh, append at qt, appendleft at --qh */
    int flag = 1;
    memcpy(initial, sudoku, 81);
    g_val = 0;
    for (int i = 0; i < 81; i++)
        if (sudoku[i] == 0) queue[qt++] = i;
    for (;;) {
        while (qt > qh) {
            const int cell = queue[qh++], i = cell / 9, j = cell % 9;
            int num = 0;
            for (int d = 1; d <= 9 && !num; d++)
                if (peer_valid_move(sudoku, i, j, d)) num = d;
            if (num) {                       /* node.py:479-485 */
                if (peer_valid_move(sudoku, i, j, num)) {
                    sudoku[cell] = (uint8_t)num;
                    partial[cell] = (uint8_t)num;
                } else {
                    queue[--qh] = cell;
                }
                continue;
            }
            /* node.py:487-532: repair */
            flag = 1;
            uint8_t temp[81];
            memcpy(temp, sudoku, 81);
            int vn_cell[9], vn_val[9], nv = 0;
            for (int c = 0; c < 9; c++) {
                const int rc = i * 9 + c;
                if (c == j || !partial[rc]) continue;
                temp[rc] = 0;
                const int v = partial[rc];
                if (peer_valid_move(temp, i, j, v))
                    if (v != initial[rc] && !tried[cell][c * 9 + v - 1]) { vn_cell[nv] = rc; vn_val[nv] = v; nv++; }
            }
            int repaired = 0;
            for (int k = 0; k < nv && !repaired; k++) {
                const int value = vn_val[k];
                int safe = 1;
                for (int t = 0; t < 9; t++) {
                    if (temp[i * 9 + t] == value || temp[t * 9 + j] == value) { safe = 0; break; }
                    if (temp[(3 * (i / 3) + t / 3) * 9 + 3 * (j / 3) + t % 3] == value) { safe = 0; break; }
                }
                if (safe) {
                    const int rc = vn_cell[k];
                    sudoku[cell] = (uint8_t)value;
                    partial[cell] = (uint8_t)value;
                    partial[rc] = 0;
                    tried[cell][(rc % 9) * 9 + value - 1] = 1;
                    sudoku[rc] = 0;
                    queue[--qh] = rc;
                    repaired = 1;
                }
            }
            if (!repaired) {
                sudoku[cell] = 0;
                flag = 0;
            }
            if (qh < 1 || qt >= 1024) return -2; /* cannot happen: bounded by the tried sets */
        }
        if (!flag) break;                    /* node.py:453-454 */
        int empty = 0;
        for (int c = 0; c < 81; c++) empty += sudoku[c] == 0;
        if (empty < 2) break;                /* node.py:462-464 */
        *validations = g_val;
        return -1;                           /* nothing changes any more: the loop spins */
    }
    g_val++;                                 /* node.py:466 self.solver.check(self.sudoku) */
    *validations = g_val;
    return oracle_check_sums(sudoku) ? 1 : 0;
}

int oracle_peer_solve(uint8_t *sudoku, int32_t *validations)
{
    uint8_t partial[81], tried[81][81];
    memset(partial, 0, sizeof partial);
    memset(tried, 0, sizeof tried);
    return oracle_peer_solve_node(sudoku, validations, partial, tried);
}
