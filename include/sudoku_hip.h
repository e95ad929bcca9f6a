/*
 * sudoku_hip.h -- C ABI of the MI355X (gfx950) Sudoku solver library
 * (libsudoku_hip.so, built from sudoku_solver_distributed_amd/csrc/).
 *
 * Plain pointers and sizes only.  Every `d_*` pointer is DEVICE memory on the
 * calling thread's current HIP device; `stream` is a hipStream_t (NULL = the
 * default stream).  Calls are asynchronous on `stream` unless noted.
 *
 * Grid format: 81 bytes per board, row-major, 0 = empty, 1..9 = digit; a batch
 * of n boards is n*81 contiguous bytes.
 *
 * Return codes: 0 = launched / ok, <0 = error (text in sdk_last_error()).
 *
 * Each entry point replaces one reference interface
 * (cristiano-nicolau/sudoku_solver_distributed):
 */
#ifndef SUDOKU_HIP_H
#define SUDOKU_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-board status written by the solvers */
#define SDK_UNSOLVABLE 0  /* gen.py:28 `return False`; output = input board   */
#define SDK_SOLVED 1      /* gen.py:18/25 `return True`; output = filled board */
#define SDK_INVALID -1    /* a byte > 9 in the input (rejected, output = input) */
#define SDK_CANCELLED -2  /* ordered mode: a lower-indexed board already solved */
#define SDK_FAULT -3      /* internal consistency check failed (never expected) */
#define SDK_NO_RETURN -4  /* sdk_peer_solve_batch: node.py's /solve loop never returns */

/* the reference's two walks (cell choice; digits are always tried 1..9) */
#define SDK_ORDER_GEN 0   /* gen.py:6-28: first empty cell of the LAST row that
                             has one (its scan breaks only the inner loop) */
#define SDK_ORDER_NODE 1  /* node.py:62-74: first empty cell, row-major      */

/* Bytes of device workspace sdk_solve_batch needs on the current device:
 * queue heads, cancel word, statistics, and the plane kernel's per-lane DFS
 * stacks and the deferred-board list (about 1.08 GB on an MI355X).  Allocate
 * once per device, zero once;
 * the library re-arms the per-call words itself on `stream`.
 * A workspace is SINGLE-STREAM: every call that passes the same workspace
 * must be issued on the same stream (or ordered by the caller), because each
 * sdk_solve_batch re-arms the workspace's queue head before its kernels when
 * they use it (not for a small unordered batch the static hand-out covers).
 * Enqueueing is thread-safe (the library serialises its launch sequences). */
size_t sdk_workspace_bytes(void);

/* Solve n boards.  For every board the output is the FIRST solution of the
 * reference walk selected by `order`, bit-identical:
 *   SDK_ORDER_GEN  gen.py:6-28          solve_sudoku(board)
 *   SDK_ORDER_NODE node.py:31-40,62-74  SudokuSolver.solve_sudoku, including
 *                  is_valid_move's short-circuit (node.py:44-45: every unit
 *                  sums to 45 -> any digit is accepted; only boards with
 *                  clashing givens can reach it).
 * d_puzzles and d_solutions may alias.
 * `ordered` != 0 selects frontier mode: once board i is solved, boards j > i
 * are abandoned (status SDK_CANCELLED) and the lowest solved index is kept in
 * the workspace (sdk_read_stats out[4]). */
int sdk_solve_batch(const uint8_t *d_puzzles, uint8_t *d_solutions, int32_t *d_status,
                    int64_t n, void *d_workspace, int order, int ordered, void *stream);

/* sdk_solve_batch with the lane-per-board kernel's grid capped at
 * `grid_waves` waves per SIMD (0: as many as fit, sdk_solve_batch's choice).
 * For launches kept in flight on several streams, each with its own
 * workspace (BatchSolver.solve_inflight): with a grid of 2 waves per SIMD two
 * launches are resident together, so one launch's drain (its last boards,
 * most lanes idle) runs beside the next one's start.  Results never depend on
 * it; a negative value is a bad argument (-2).  Replaces the same reference
 * walks as sdk_solve_batch (gen.py:6-28, node.py:62-74).
 * grid_waves | SDK_GRID_PIPELINED: another launch is queued behind this one
 * on the device.  Its drained waves then finish only their own last boards
 * and exit, so the next launch's waves take their slots; without the flag
 * (the launch's end is the caller's wait) they share their last boards
 * across the XCD through the tail pool (tail mode 2). */
#define SDK_GRID_PIPELINED 0x10000
int sdk_solve_batch_grid(const uint8_t *d_puzzles, uint8_t *d_solutions, int32_t *d_status,
                         int64_t n, void *d_workspace, int order, int ordered, void *stream,
                         int grid_waves);

/* Several independent batches solved by ONE launch sequence on one
 * workspace (unordered): batch i is d_puzzles[i] -> d_solutions[i],
 * d_status[i], n[i] boards, exactly as sdk_solve_batch_grid would solve it
 * alone (same bytes, same statuses).  The lane-per-board kernel's queue runs
 * over the batches laid end to end, so the lanes that finish one batch's
 * boards take the next batch's and the grid drains once per call instead of
 * once per batch: a multi-step persistent launch (bench.py's strong-scaling
 * steps, where one GPU's share of a step is too small to fill the chip).
 * 1 <= count <= SDK_MAX_BATCHES; a batch may be empty; batches must not
 * overlap each other's outputs.  Returns 0 / -1 (HIP error) / -2 (bad
 * arguments).  Replaces the same reference walks as sdk_solve_batch
 * (gen.py:6-28, node.py:62-74), once per board. */
#define SDK_MAX_BATCHES 32
int sdk_solve_batches(const uint8_t *const *d_puzzles, uint8_t *const *d_solutions, int32_t *const *d_status,
                      const int64_t *n, int count, void *d_workspace, int order, void *stream, int grid_waves);

/* Batch Sudoku.check (mode 0, sudoku.py:119-140: every row, column and box
 * sums to 45 and holds 9 distinct values) or node.py's SudokuSolver.check
 * (mode 1, node.py:82-116: sums only).  d_ok[i] = 1/0. */
int sdk_check_batch(const uint8_t *d_grids, int32_t *d_ok, int64_t n, int mode, void *stream);

/* Batch of node.py "solve" tasks (node.py:384-406 -> 76-80,
 * SudokuSolver.solve_sudoku_destributed): d_num[i] = first digit 1..9 that
 * is_valid_move (node.py:42-60) accepts at cell d_cells[i] (= row*9+col) of
 * board i, or 0 for None. */
int sdk_first_candidate_batch(const uint8_t *d_grids, const int32_t *d_cells,
                              int32_t *d_num, int64_t n, void *stream);

/* The reference's HTTP /solve algorithm, node.py:534-557
 * P2PNode.peer_sudoku_solve, one FRESH single node per board (handicap 0, no
 * peers; sdk_peer_solve_seq below carries one node's state across requests):
 * a greedy row-major cell loop with node.py's repair step (node.py:419-532),
 * not a search.  d_out[i] = the board it leaves (valid or not), d_status[i] =
 * SDK_SOLVED (its final check passed), SDK_UNSOLVABLE (returned, check
 * failed), SDK_NO_RETURN (node.py loops forever on this board; d_out = the
 * board at that point) or SDK_INVALID (a byte > 9); d_validations[i] =
 * node.py's `validations` counter after the call (one per
 * SudokuSolver.check: every is_valid_move plus the final check). */
int sdk_peer_solve_batch(const uint8_t *d_boards, uint8_t *d_out, int32_t *d_status, int32_t *d_validations,
                         int64_t n, void *stream);

/* The same /solve loop on ONE P2PNode serving n requests in order
 * (node.py:534-557, requests 0..n-1 as the reference's single-threaded
 * HTTPServer would take them).  The node keeps partial_solution and
 * tried_numbers_by_position (node.py:149, 167) across requests, and a later
 * request's repair step (node.py:501-506) reads what earlier ones left, so
 * request i starts from the state request i-1 left.  d_node_state: one
 * SDK_PEER_STATE_BYTES record in device memory, in/out (all zero = a new
 * node).  Outputs per request as sdk_peer_solve_batch; d_validations[i] is
 * the counter's increase during request i.  A request with a byte > 9 gets
 * SDK_INVALID and leaves the node as it was.  After SDK_NO_RETURN the
 * reference node spins forever and serves nothing more; this call goes on
 * from the state the loop spun in. */
#define SDK_PEER_STATE_BYTES 1600
int sdk_peer_solve_seq(const uint8_t *d_boards, uint8_t *d_out, int32_t *d_status, int32_t *d_validations,
                       int64_t n, void *d_node_state, void *stream);

/* One level of the reference walk's search tree, for splitting a single hard
 * board over waves / GPUs (node.py's per-cell peer task split, node.py:419-449,
 * re-designed as a frontier split).  Every input node is propagated; then
 *   dead   -> no child,
 *   solved -> one child: the solved grid,
 *   open   -> one child per candidate of the walk's next cell (`order`),
 *             digits ascending.
 * Children of all nodes, concatenated in input order, are therefore in the
 * walk's (lexicographic) order, and the first SOLVED child of the frontier
 * carries the walk's first solution.
 *   d_tmp:      scratch, n*81 bytes
 *   d_offsets:  n+1 int64; d_offsets[n] = total children (read it back)
 *   d_children: capacity cap*81 bytes; children past cap are not written.
 * Caller checks d_offsets[n] <= cap. */
int sdk_expand_frontier(const uint8_t *d_nodes, int64_t n, uint8_t *d_tmp, int64_t *d_offsets,
                        uint8_t *d_children, int64_t cap, int order, void *stream);

/* Copy statistics to host (synchronous on `stream`):
 * out[0] boards finished, out[1] boards solved, out[2] guesses (branch
 * nodes of the searches that gave each board its answer), out[3]
 * propagation passes / sweeps executed (all work, including searches the
 * plane kernel abandoned when it handed a board over), out[4] lowest solved
 * index in ordered mode (INT64_MAX if none), out[5] boards the plane kernel
 * handed to the wave-per-board pass (clashing givens, searches deeper than
 * its stack, the last few boards of a wave once the queue is empty).
 * reset != 0 zeroes them afterwards (and the boards-assigned count of
 * sdk_verify_workspace; never its error word). */
int sdk_read_stats(void *d_workspace, int64_t out[6], int reset, void *stream);

/* Every board answered?  (Synchronous on `stream`; library extension, the
 * reference's walk answers every board it is given, gen.py:6-28.)  Each
 * solve launch adds its board count to the workspace, each board's answer
 * (any status) counts once as finished, and a kernel that could not finish a
 * board it had taken sets an error word (SDK_ERR_* bits: 1 = a tail-pool
 * record it had claimed was never published).  out (may be
 * NULL): out[0] boards assigned, out[1] boards finished, out[2] error bits,
 * all since the last sdk_read_stats(reset) / report; out[3] reserved (0).
 * Returns 0 when
 * assigned == finished and no error bit is set; -3 otherwise (text in
 * sdk_last_error(); the error word is then cleared and the counts re-synced,
 * so each fault is reported once); -1 HIP error; -2 bad arguments. */
int sdk_verify_workspace(void *d_workspace, int64_t out[4], void *stream);

/* The same six counters as sdk_read_stats, copied to DEVICE memory d_out[6]
 * asynchronously on `stream` (stream-ordered with the solves on that
 * workspace: two snapshots around a solve give that solve's own counts
 * without a host synchronisation). */
int sdk_snapshot_stats(const void *d_workspace, int64_t *d_out, void *stream);

/* Solve-kernel selection (library extension, no reference counterpart):
 * SDK_KERNEL_AUTO (default) SDK_KERNEL_PLANE for batches of 8192 boards or
 * more, SDK_KERNEL_PACKED below; SDK_KERNEL_PLANE one lane per board on
 * digit-plane bitboards (boards with clashing givens or very deep searches
 * go to a wave-per-board pass); SDK_KERNEL_PACKED one wavefront per board,
 * both cells of a lane packed in one word.  Both give the same results.
 * 0 restores the default (or $SDK_SOLVE_KERNEL = auto|plane|packed).
 * Returns the previous selection, -1 for an unknown value. */
#define SDK_KERNEL_AUTO 1
#define SDK_KERNEL_PACKED 5
#define SDK_KERNEL_PLANE 6
int sdk_set_solve_kernel(int kernel);

/* Plane-kernel tuning (library extension, no reference counterpart; the
 * defaults are the measured optimum).  refill: idle lanes
 * before a wave refills; tail: active lanes at or below which a drained wave
 * hands its last boards to the tail solver (0 off, at most 40); tail_mode: 1
 * the wave-wide solver continues each search on the wave itself, 2 the same
 * through a per-XCD pool that every exiting wave of the XCD drains; chunk:
 * most boards a wave claims from the queue at once (at
 * most 64: a claim is staged and converted in one go; 0 one claim per refill).  A
 * negative value keeps that knob; all four negative restore the defaults
 * ($SDK_PLANE_REFILL / _TAIL / _TAIL_MODE / _CHUNK).  Results never depend on
 * them.  Returns 0, or -1 for an out-of-range value (nothing changed). */
int sdk_set_plane_tuning(int refill, int tail, int tail_mode, int chunk);

/* Plane-kernel search (library extension, no reference counterpart): a
 * board still searching after `mrv_after` propagation passes goes back to
 * its propagated root and counts its completions (to two) branching on
 * fewest-candidates cells: exactly one completion is the walk's answer, none
 * means none for the walk too, two send the board back to the walk's own
 * branch order.  With the switch on, a board whose
 * propagated root keeps >= 58 open cells counts from the root at once.  0
 * keeps every board on the walk's order; -1
 * restores the default ($SDK_PLANE_MRV, built-in 128).  Results never
 * depend on it.  Returns the setting in effect before the call (the
 * default's value when no override was set), -2 for an out-of-range value
 * (nothing changed). */
int sdk_set_plane_search(int mrv_after);

/* Library / device info. */
const char *sdk_last_error(void);
const char *sdk_version(void);
int sdk_device_cu_count(void);

#ifdef __cplusplus
}
#endif
#endif /* SUDOKU_HIP_H */
