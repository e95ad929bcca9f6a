// packed_solver.h -- wave-per-board solver: one board per wavefront, both
// cells of a lane packed into one 32-bit word.  Device code only: the
// kernels built on it (solvep_kernel, solvep_deferred_kernel) live in
// sudoku_kernels.hip, and plane_kernel runs it for a wave's last boards.
//
// Propagation rules: naked singles; hidden singles when no naked single is
// left; clash and empty-unit detection; branching on the walk's next cell,
// digits ascending -- so the walk's first completion.
// Node order additionally reproduces node.py's is_valid_move short-circuit
// (node.py:44-45) exactly: see "literal mode" below.  The arithmetic:
//   * lane l owns cell l in the low half and, for l < 17, cell 64+l in the
//     high half of every per-lane word.  Lanes >= 17 carry a phantom high
//     cell that is always filled and whose units are the dummy word 27;
//   * digits are one-hot (bit d-1 of a half), so a placement ORs straight
//     into the unit masks, and the unit masks in LDS hold every digit bit in
//     BOTH halves: one 3-input OR per half and a bit-field select give the
//     two cells' used digits in one word;
//   * emptiness, naked-single and hidden-single tests run on both halves at
//     once with packed 16-bit adds/subtracts (v_pk_add_u16 / v_pk_sub_u16:
//     x + 0x7FFF sets bit 15 iff a half is non-zero; x & (x - 1) clears the
//     lowest bit of each half) and a packed arithmetic shift turns bit 15
//     into a whole-half select mask;
//   * per-lane state is five words (digit, empty key, fill depth, givens,
//     new placements) instead of v2's eleven per-slot registers.
#ifndef SDK_PACKED_SOLVER_H
#define SDK_PACKED_SOLVER_H

enum { PROP_OPEN = 0, PROP_DEAD = 1, PROP_SOLVED = 2 };

typedef unsigned short sdk_u16x2 __attribute__((ext_vector_type(2)));
typedef short sdk_i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(sdk_u16x2, a) + __builtin_bit_cast(sdk_u16x2, b));
}
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(sdk_u16x2, a) - __builtin_bit_cast(sdk_u16x2, b));
}
// bit 15 of each half -> 0xFFFF / 0 for that half
__device__ __forceinline__ uint32_t pk_spread15(uint32_t a)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(sdk_i16x2, a) >> (sdk_i16x2){15, 15});
}
// low half from lo, high half from hi (v_bfi_b32 / v_perm_b32)
__device__ __forceinline__ uint32_t halves(uint32_t lo, uint32_t hi)
{
    return (lo & 0x0000FFFFu) | (hi & 0xFFFF0000u);
}

#define PK_EMPTY 0x81FFu        // key of an empty half: bit 15 flag + nine candidate bits
#define PK_C9 0x01FF01FFu       // candidate bits of both halves
#define PK_B15 0x80008000u      // flag bit of both halves
#define PK_NZ 0x7FFF7FFFu       // + this: bit 15 set iff the half is non-zero
#define PK_ONE 0x00010001u

struct __attribute__((aligned(16))) PackLds {
    uint32_t M[28];   // unit masks of filled cells, digit bits in both halves; M[27] = 0 (phantom units)
    uint32_t T[28];   // per unit: digits that are candidates of >= 2 empty cells, both halves
    uint32_t C[128];  // per cell: candidates published for the unit gather (81.. padding)
    uint32_t bad;     // units whose GIVENS repeat a digit (hidden-single rules off there)
    uint32_t pad[3];
};

struct PCells {
    uint32_t D;   // one-hot digit per half (0 = empty)
    uint32_t EK;  // PK_EMPTY per empty half, 0 per filled (or phantom) half
    uint32_t LV;  // depth at which each half was filled (givens / phantom: 0)
    uint32_t G;   // one-hot given per half (the input board: written back on failure)
    uint32_t GS;  // one-hot "given" of the current propagation root (= G except below a
                  // literal-mode node, where every cell filled there counts as given)
    uint32_t NW;  // one-hot placements since the last sweep (not yet in the unit masks)
    int u0, u1, u2, u3, u4, u5;  // units (rows 0-8, columns 9-17, boxes 18-26) of the low / high cell
    int ub, us1, us2;            // unit gather (lanes < 27): cells ub + k*us1 + (k/3)*us2
};

__device__ __forceinline__ void pinit_lane(PCells &s, int lane)
{
    int r, c, b;
    cell_units(lane, r, c, b);
    s.u0 = r; s.u1 = 9 + c; s.u2 = 18 + b;
    if (lane < 17) {
        cell_units(64 + lane, r, c, b);
        s.u3 = r; s.u4 = 9 + c; s.u5 = 18 + b;
    } else {
        s.u3 = s.u4 = s.u5 = 27;
    }
    if (lane < 9) { s.ub = 9 * lane; s.us1 = 1; s.us2 = 0; }
    else if (lane < 18) { s.ub = lane - 9; s.us1 = 9; s.us2 = 0; }
    else { const int bx = lane < 27 ? lane - 18 : 0;
           s.ub = (bx / 3) * 27 + (bx % 3) * 3; s.us1 = 1; s.us2 = 6; }
}

__device__ __forceinline__ uint32_t onehot(uint32_t v) { return v ? 1u << ((v - 1) & 31) : 0u; }
__device__ __forceinline__ uint32_t digit_of(uint32_t oh) { return oh ? (uint32_t)__builtin_ctz(oh) + 1 : 0u; }

// Load one board; raw bytes stay in a / b for the invalid-board write-back.
// Returns false (wave-uniform) if any byte is > 9.
__device__ __forceinline__ bool pload_board(const uint8_t *__restrict__ src, int lane, PCells &s, uint32_t &a,
                                            uint32_t &b)
{
    a = src[lane];
    b = lane < 17 ? (uint32_t)src[64 + lane] : 0u;
    s.D = onehot(a) | (onehot(b) << 16);
    s.G = s.D;
    s.GS = s.D;
    s.EK = (a == 0 ? PK_EMPTY : 0u) | ((lane < 17 && b == 0) ? (PK_EMPTY << 16) : 0u);
    s.LV = 0;
    s.NW = 0;
    return !wany(a > 9 || b > 9);
}

// Root givens' (s.GS) unit masks (both halves; returned in lanes 0..26, W.M
// holds them) and the bad-unit mask.
__device__ __forceinline__ uint32_t pbuild_given_masks(PackLds &W, int lane, const PCells &s, uint32_t &bad)
{
    if (lane < 28) W.M[lane] = 0;
    if (lane == 0) W.bad = 0;
    wave_lds_sync();
    const uint32_t g0 = s.GS & 0xFFFFu, g1 = s.GS >> 16;
    uint32_t d = 0;
    if (g0) {
        const uint32_t bd = g0 | (g0 << 16);
        if (atomicOr(&W.M[s.u0], bd) & bd) d |= 1u << s.u0;
        if (atomicOr(&W.M[s.u1], bd) & bd) d |= 1u << s.u1;
        if (atomicOr(&W.M[s.u2], bd) & bd) d |= 1u << s.u2;
    }
    if (g1) {
        const uint32_t bd = g1 | (g1 << 16);
        if (atomicOr(&W.M[s.u3], bd) & bd) d |= 1u << s.u3;
        if (atomicOr(&W.M[s.u4], bd) & bd) d |= 1u << s.u4;
        if (atomicOr(&W.M[s.u5], bd) & bd) d |= 1u << s.u5;
    }
    if (d) atomicOr(&W.bad, d);
    wave_lds_sync();
    bad = __builtin_amdgcn_readfirstlane(W.bad);
    return lane < 27 ? W.M[lane] : 0u;
}

// One propagation sweep (v2's sweep() on packed cells; same rules, same
// return contract).  c9 receives both halves' candidates (0 for filled).
__device__ __forceinline__ int psweep(PackLds &W, int lane, PCells &s, uint32_t gmask, uint32_t bad,
                                      uint32_t depth2, bool &rebuild, uint32_t &c9, bool &placed)
{
    placed = false;
    // ---- phase A: bring the unit masks up to date; clash detection
    uint32_t f;
    if (rebuild) {
        if (lane < 27) W.M[lane] = gmask;
        f = s.D & ~s.GS;
    } else {
        f = s.NW;
    }
    s.NW = 0;
    uint32_t clash = 0;
    if (rebuild || wany(f != 0)) {
        wave_lds_sync();
        const uint32_t f0 = f & 0xFFFFu, f1 = f >> 16;
        if (f0) {
            const uint32_t bd = f0 | (f0 << 16);
            clash |= (atomicOr(&W.M[s.u0], bd) | atomicOr(&W.M[s.u1], bd) | atomicOr(&W.M[s.u2], bd)) & bd;
        }
        if (f1) {
            const uint32_t bd = f1 | (f1 << 16);
            clash |= (atomicOr(&W.M[s.u3], bd) | atomicOr(&W.M[s.u4], bd) | atomicOr(&W.M[s.u5], bd)) & bd;
        }
        wave_lds_sync();
    }
    rebuild = false;
    const uint32_t mlo = W.M[s.u0] | W.M[s.u1] | W.M[s.u2];
    const uint32_t mhi = W.M[s.u3] | W.M[s.u4] | W.M[s.u5];
    const uint32_t cand = s.EK & ~halves(mlo, mhi);  // bit 15 per half: empty
    c9 = cand & PK_C9;
    const uint32_t nz = pk_add(c9, PK_NZ);           // bit 15: some candidate left
    if (wany(((cand & ~nz & PK_B15) | clash) != 0)) return PROP_DEAD;
    if (!wany(s.EK != 0)) return PROP_SOLVED;

    // ---- naked singles: non-zero and x & (x - 1) == 0
    const uint32_t naked = nz & ~pk_add(c9 & pk_sub(c9, PK_ONE), PK_NZ) & PK_B15;
    if (wany(naked != 0)) {
        const uint32_t nm = pk_spread15(naked);
        const uint32_t p = c9 & nm;
        s.D |= p;
        s.EK &= ~nm;
        s.LV = (s.LV & ~nm) | (depth2 & nm);
        s.NW = p;
        placed = true;
        return PROP_OPEN;
    }

    // ---- phase B: hidden singles and digits with no place in a unit
    // (v2's publish / gather; a unit whose givens clash publishes T = all)
    W.C[lane] = c9 & 0x1FFu;
    W.C[64 + lane] = c9 >> 16;  // lanes >= 17 land in padding
    wave_lds_sync();
    bool udead = false;
    if (lane < 27) {
        uint32_t once = 0, twice = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t x = W.C[s.ub + k * s.us1 + (k / 3) * s.us2];
            twice |= once & x;
            once |= x;
        }
        const bool ok = !((bad >> lane) & 1u);
        const uint32_t tv = ok ? twice : 0x1FFu;
        W.T[lane] = tv | (tv << 16);
        udead = ok && ((once | W.M[lane]) & 0x1FFu) != 0x1FFu;
    }
    wave_lds_sync();
    const uint32_t tlo = W.T[s.u0] & W.T[s.u1] & W.T[s.u2];
    const uint32_t thi = W.T[s.u3] & W.T[s.u4] & W.T[s.u5];
    const uint32_t h = c9 & ~halves(tlo, thi);
    if (wany(udead || (h & pk_sub(h, PK_ONE)) != 0)) return PROP_DEAD;
    if (wany(h != 0)) {
        const uint32_t hm = pk_spread15(pk_add(h, PK_NZ));
        s.D |= h;
        s.EK &= ~hm;
        s.LV = (s.LV & ~hm) | (depth2 & hm);
        s.NW = h;
        placed = true;
    }
    return PROP_OPEN;
}

__device__ __forceinline__ int ppropagate(PackLds &W, int lane, PCells &s, uint32_t gmask, uint32_t bad,
                                          uint32_t depth, bool &rebuild, uint32_t &c9, uint32_t &sweeps)
{
    const uint32_t depth2 = depth | (depth << 16);
    for (;;) {
        bool placed;
        const int st = psweep(W, lane, s, gmask, bad, depth2, rebuild, c9, placed);
        sweeps++;
        if (st != PROP_OPEN || !placed) return st;
    }
}

__device__ __forceinline__ void pplace(PCells &s, int lane, int cell, uint32_t dbit, uint32_t level)
{
    if (lane == (cell & 63)) {
        const int sh = cell >= 64 ? 16 : 0;
        const uint32_t hm = 0xFFFFu << sh;
        s.D |= dbit << sh;
        s.EK &= ~hm;
        s.LV = (s.LV & ~hm) | (level << sh);
        s.NW |= dbit << sh;
    }
}

// clear every cell filled at depth >= `depth` (givens and phantoms have depth 0)
__device__ __forceinline__ void pundo(PCells &s, uint32_t depth)
{
    if ((s.LV & 0xFFFFu) >= depth) { s.D &= 0xFFFF0000u; s.EK |= PK_EMPTY; }
    if ((s.LV >> 16) >= depth) { s.D &= 0x0000FFFFu; s.EK |= PK_EMPTY << 16; }
}

__device__ __forceinline__ void pstore_board(uint8_t *__restrict__ dst, int lane, const PCells &s, bool original)
{
    const uint32_t x = original ? s.G : s.D;
    dst[lane] = (uint8_t)digit_of(x & 0xFFFFu);
    if (lane < 17) dst[64 + lane] = (uint8_t)digit_of(x >> 16);
}

// ------------------------------------------------------------ literal mode
// node.py's walk tests a digit with is_valid_move (node.py:42-60), which
// answers True whenever every row, column and box already sums to 45
// (node.py:44-45, SudokuSolver.check).  With an empty cell on the board that
// needs repeated digits, so only boards whose givens clash can get there --
// and then the walk may put ANY digit in the cell.  Propagation (naked /
// hidden singles, dead-cell tests) presumes the plain rule below such a
// node, so in node order the search runs "literally" (no propagation, branch
// on the first empty cell, candidates = the digits is_valid_move accepts)
// while such a node is still reachable:
//
//   R(N) = every unit u has  s_u <= 45 <= s_u + 9 e_u  (sum / empty cells)
//          and some empty cell has a repeated digit in its row, its column
//          AND its box.
//
// Along a path s_u only grows, s_u + 9 e_u only shrinks, and plain moves
// create no repeated digit, so R is monotone: once R(N) is false the whole
// subtree is the plain walk, rooted at N (every cell filled at N counts as a
// given there: GS).  A node where the short-circuit fires has R true (its
// cell's units sum to 45 with a hole, so they repeat a digit).
struct LitEval {
    bool R;        // a short-circuit node is reachable below (and at) this node
    bool s45;      // every unit sums to 45 here: is_valid_move accepts 1..9
    uint32_t cand; // lane: candidates of its low (bits 0-8) / high (16-24) cell
};

__device__ __forceinline__ LitEval lit_eval(PackLds &W, int lane, const PCells &s)
{
    // T[u]: sum | filled count << 8; C[u]: digits present; pad[0]: units
    // with a repeated digit.  (T and C are psweep phase-B scratch.)
    if (lane < 28) { W.T[lane] = 0; W.C[lane] = 0; }
    if (lane == 0) W.pad[0] = 0;
    wave_lds_sync();
    const uint32_t dlo = digit_of(s.D & 0xFFFFu), dhi = digit_of(s.D >> 16);
    uint32_t dup = 0;
    if (dlo) {
        const uint32_t add = dlo | (1u << 8), bit = 1u << (dlo - 1);
        atomicAdd(&W.T[s.u0], add); atomicAdd(&W.T[s.u1], add); atomicAdd(&W.T[s.u2], add);
        if (atomicOr(&W.C[s.u0], bit) & bit) dup |= 1u << s.u0;
        if (atomicOr(&W.C[s.u1], bit) & bit) dup |= 1u << s.u1;
        if (atomicOr(&W.C[s.u2], bit) & bit) dup |= 1u << s.u2;
    }
    if (dhi) {  // phantom halves (lanes >= 17) hold no digit
        const uint32_t add = dhi | (1u << 8), bit = 1u << (dhi - 1);
        atomicAdd(&W.T[s.u3], add); atomicAdd(&W.T[s.u4], add); atomicAdd(&W.T[s.u5], add);
        if (atomicOr(&W.C[s.u3], bit) & bit) dup |= 1u << s.u3;
        if (atomicOr(&W.C[s.u4], bit) & bit) dup |= 1u << s.u4;
        if (atomicOr(&W.C[s.u5], bit) & bit) dup |= 1u << s.u5;
    }
    if (dup) atomicOr(&W.pad[0], dup);
    wave_lds_sync();
    const uint32_t dups = __builtin_amdgcn_readfirstlane(W.pad[0]);
    bool unit_ok = true, is45 = true;
    if (lane < 27) {
        const uint32_t t = W.T[lane], sum = t & 0xFFu, empty = 9u - (t >> 8);
        unit_ok = sum <= 45u && sum + 9u * empty >= 45u;
        is45 = sum == 45u;
    }
    const bool clo = (s.EK & 0x8000u) && ((dups >> s.u0) & (dups >> s.u1) & (dups >> s.u2) & 1u);
    const bool chi = (s.EK & 0x80000000u) && ((dups >> s.u3) & (dups >> s.u4) & (dups >> s.u5) & 1u);
    LitEval r;
    r.R = !wany(!unit_ok) && wany(clo || chi);
    r.s45 = !wany(!is45);
    const uint32_t ulo = W.C[s.u0] | W.C[s.u1] | W.C[s.u2], uhi = W.C[s.u3] | W.C[s.u4] | W.C[s.u5];
    r.cand = (~ulo & 0x1FFu) | ((~uhi & 0x1FFu) << 16);
    return r;
}

// Full search of one board.
__device__ __forceinline__ int psearch(PackLds &W, int lane, PCells &s, int64_t idx, int order, const int64_t *best,
                                       uint32_t &guesses, uint32_t &sweeps)
{
    uint32_t bad;
    uint32_t gmask = pbuild_given_masks(W, lane, s, bad);
    // literal mode is possible only in node order, with repeated givens
    bool lit = order == SDK_ORDER_NODE && bad != 0;
    uint32_t lit_top = 0;  // literal mode: depth at which the plain walk took over
    bool rebuild = false;  // W.M already holds exactly the givens
    uint32_t depth = 0;
    uint32_t stk0 = 0, stk1 = 0;  // DFS stack: level k lives in lane k&63 of stk(k>>6)
    uint32_t c9;
    bool in_lit = lit;
    int result;
    for (;;) {
        bool dead = false;
        if (in_lit) {
            const LitEval e = lit_eval(W, lane, s);
            if (e.R) {
                // node.py:63-72 literally: first empty cell, digits is_valid_move accepts
                const uint64_t eb0 = __builtin_amdgcn_ballot_w64((s.EK & 0x8000u) != 0);
                const uint64_t eb1 = __builtin_amdgcn_ballot_w64((s.EK & 0x80000000u) != 0);
                const int cell = order_cell(eb0, eb1, SDK_ORDER_NODE);  // R => an empty cell exists
                const uint32_t cand = e.s45 ? 0x1FFu
                                    : cell < 64 ? rdlane(e.cand, cell) & 0x1FFu : rdlane(e.cand, cell - 64) >> 16;
                if (cand == 0) {
                    dead = true;
                } else {
                    const uint32_t d = lowbit(cand);
                    const uint32_t entry = ((uint32_t)cell << 9) | (cand ^ d);
                    if (depth < 64) { if (lane == (int)depth) stk0 = entry; }
                    else if (lane == (int)depth - 64) stk1 = entry;
                    depth++;
                    pplace(s, lane, cell, d, depth);
                    guesses++;
                    continue;
                }
            } else {
                // the plain walk from here: every filled cell is a given below
                in_lit = false;
                lit_top = depth;
                s.GS = s.D;
                s.NW = 0;
                gmask = pbuild_given_masks(W, lane, s, bad);
                rebuild = false;
            }
        }
        if (!dead) {
            const int st = ppropagate(W, lane, s, gmask, bad, depth, rebuild, c9, sweeps);
            if (st == PROP_SOLVED) { result = SDK_SOLVED; break; }
            if (st == PROP_OPEN) {
                // branch on the walk's next cell, smallest digit first
                const uint64_t eb0 = __builtin_amdgcn_ballot_w64((s.EK & 0x8000u) != 0);
                const uint64_t eb1 = __builtin_amdgcn_ballot_w64((s.EK & 0x80000000u) != 0);
                const int cell = order_cell(eb0, eb1, order);
                const uint32_t cand = cell < 64 ? rdlane(c9, cell) & 0x1FFu : rdlane(c9, cell - 64) >> 16;
                if (cand == 0) { result = SDK_FAULT; break; }  // unreachable: a fixpoint has no empty cell without candidates
                const uint32_t d = lowbit(cand);
                const uint32_t entry = ((uint32_t)cell << 9) | (cand ^ d);
                if (depth < 64) { if (lane == (int)depth) stk0 = entry; }
                else if (lane == (int)depth - 64) stk1 = entry;
                depth++;
                pplace(s, lane, cell, d, depth);
                guesses++;
                if (best && (guesses & 63u) == 0) {
                    const int64_t b = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (__builtin_amdgcn_readfirstlane((int)(b < idx))) { result = SDK_CANCELLED; break; }
                }
                continue;
            }
        }
        // dead: backtrack to the deepest level with an untried digit
        rebuild = true;
        s.NW = 0;
        bool exhausted = false;
        for (;;) {
            if (depth == 0) { exhausted = true; break; }
            const uint32_t top = depth - 1;
            const uint32_t entry = top < 64 ? rdlane(stk0, top) : rdlane(stk1, top - 64);
            pundo(s, depth);
            depth = top;
            if (lit && !in_lit && top < lit_top) {
                // back above the node where the plain walk took over: literal again
                in_lit = true;
                s.GS = s.G;
            }
            const uint32_t rem = entry & 0x1FFu;
            if (rem == 0) continue;
            const int cell = (int)(entry >> 9);
            const uint32_t d = lowbit(rem);
            const uint32_t ne = ((uint32_t)cell << 9) | (rem ^ d);
            if (depth < 64) { if (lane == (int)depth) stk0 = ne; }
            else if (lane == (int)depth - 64) stk1 = ne;
            depth++;
            pplace(s, lane, cell, d, depth);
            guesses++;
            break;
        }
        if (exhausted) { result = SDK_UNSOLVABLE; break; }
    }
    s.GS = s.G;
    return result;
}

// One board (index p) by the whole wave: load, search, store, status.
__device__ __forceinline__ void psolve_board(PackLds &W, int lane, PCells &s, const uint8_t *__restrict__ puzzles,
                                             uint8_t *__restrict__ sols, int32_t *__restrict__ status, int64_t p,
                                             unsigned long long *__restrict__ ws, const int64_t *best, int order,
                                             uint32_t &solved, uint32_t &guesses, uint32_t &sweeps)
{
    const uint8_t *src = puzzles + p * 81;
    uint8_t *dst = sols + p * 81;
    uint32_t a, b;
    int st;
    if (!pload_board(src, lane, s, a, b)) {
        st = SDK_INVALID;
        dst[lane] = (uint8_t)a;  // raw input back
        if (lane < 17) dst[64 + lane] = (uint8_t)b;
    } else if (best && __builtin_amdgcn_readfirstlane((int)(
                   __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p))) {
        st = SDK_CANCELLED;
        pstore_board(dst, lane, s, true);
    } else {
        st = psearch(W, lane, s, p, order, best, guesses, sweeps);
        pstore_board(dst, lane, s, st != SDK_SOLVED);
        if (st == SDK_SOLVED) {
            solved++;
            if (best && lane == 0)
                __hip_atomic_fetch_min((int64_t *)&ws[WS_BEST], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (lane == 0) status[p] = st;
}

__device__ __forceinline__ void pflush_stats(int lane, unsigned long long *__restrict__ ws, uint32_t fin,
                                             uint32_t solved, uint32_t guesses, uint32_t sweeps)
{
    if (lane == 0 && fin) {
        atomicAdd(&ws[WS_FINISHED], (unsigned long long)fin);
        atomicAdd(&ws[WS_SOLVED], (unsigned long long)solved);
        atomicAdd(&ws[WS_GUESSES], (unsigned long long)guesses);
        atomicAdd(&ws[WS_SWEEPS], (unsigned long long)sweeps);
    }
}

#endif  // SDK_PACKED_SOLVER_H
