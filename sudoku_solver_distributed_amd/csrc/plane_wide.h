// plane_wide.h -- one board over a whole WAVE, on the digit planes of
// plane_solver.h.  The drained-wave tail of plane_kernel (plane_kernel.h).
//
// Why: once the board queue is empty a wave of plane_kernel holds its last
// boards one per lane, and a lane pass costs the whole wave ~1300 issue slots
// whatever its active lanes, so the wave idles on its slowest board for tens
// of passes.  Here the 27 plane words of ONE board are spread
// over the wave, lane 16*b + d holding P[d][b] (rows of 16 lanes = bands,
// lanes 9..15 of a row and row 3 hold 0), and a pass is ~150 wave
// instructions: the nine digits and three bands run in parallel,
// cross-digit sums are DPP row rotations, cross-band ones ds_bpermute.  The
// search continues from the lane's state -- same planes, same per-lane stack
// lines (plane_kernel.h PlaneStack), same branch rule -- so nothing is redone.
//
// Propagation is the same rule set as plane::pass (A naked singles, B peer
// elimination, C hidden singles, dead units, D box -> column locked
// candidates), with C's hidden singles applied
// Jacobi-style (all digits at once; a cell forced for two digits is dead)
// instead of Gauss-Seidel, and B run a second time for the cells forced this
// pass.  Both passes are sound and reach the same fixpoints (up to when a
// duplicated determined digit -- a contradiction neither flags at once -- is
// met), so the branch cells and the first completion in walk order are the
// lane solver's.  The host build (tests/native/wide_host.cpp)
// checks fixpoints, answers and guess counts against plane_solver.h.
//
// The code is written once over a lane-value type V: on the device V is this
// lane's uint32_t and the cross-lane helpers are DPP / ds_bpermute / ballot;
// on the host V holds all 64 lanes and the helpers emulate them.
#ifndef SDK_PLANE_WIDE_H
#define SDK_PLANE_WIDE_H

#include "plane_solver.h"

namespace wide {

using plane::BOXC;
using plane::GUARDS;
using plane::ROWS;

#if defined(__HIPCC__)
#define WD_FN __device__ __forceinline__
#define WD_MF __device__ __forceinline__
typedef uint32_t V;  // this lane's word
typedef bool M;      // this lane's flag
WD_FN V lane_id() { return __lane_id(); }
WD_FN uint64_t ballot(M m) { return __builtin_amdgcn_ballot_w64(m); }
WD_FN uint32_t rdl(V v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
// DPP row_ror:N -- lane j of a 16-lane row reads lane (j + N) mod 16 of it
template <int N>
WD_FN V ror(V v)
{
    return (V)__builtin_amdgcn_update_dpp(0, (int)v, 0x120 + N, 0xF, 0xF, false);
}
// value of lane byteaddr / 4
WD_FN V bperm(V v, V byteaddr) { return (V)__builtin_amdgcn_ds_bpermute((int)byteaddr, (int)v); }
WD_FN M eq(V a, V b) { return a == b; }
WD_FN M ne(V a, V b) { return a != b; }
WD_FN M lt(V a, V b) { return a < b; }
WD_FN M mand(M a, M b) { return a && b; }
WD_FN M mor(M a, M b) { return a || b; }
WD_FN V pick(M m, V a, V b) { return m ? a : b; }
WD_FN V or3(V a, V b, V c) { return plane::or3(a, b, c); }
WD_FN V maj3(V a, V b, V c) { return plane::maj3(a, b, c); }
WD_FN V xor3(V a, V b, V c) { return plane::xor3(a, b, c); }
WD_FN V point_rows(V y) { return plane::point_rows(y); }
WD_FN V andn(V a, V b) { return plane::andn(a, b); }
WD_FN V andn2(V a, V b, V c) { return plane::andn2(a, b, c); }
WD_FN V sel(V m, V a, V b) { return plane::sel(m, a, b); }
WD_FN V bop3_nor(V a, V b, V c) { return plane::bop3_nor(a, b, c); }
WD_FN V mul24(V c, uint32_t k) { return plane::mul24(c, k); }
#else
#define WD_FN static inline
#define WD_MF inline
struct V {
    uint32_t x[64];
    V() {}
    V(uint32_t c)
    {
        for (int i = 0; i < 64; ++i) x[i] = c;
    }
};
struct M {
    uint64_t m;
};
#define WD_BIN(op)                                                 \
    WD_FN V operator op(const V &a, const V &b)                    \
    {                                                              \
        V r;                                                       \
        for (int i = 0; i < 64; ++i) r.x[i] = a.x[i] op b.x[i];    \
        return r;                                                  \
    }
WD_BIN(&)
WD_BIN(|)
WD_BIN(^)
WD_BIN(+)
WD_BIN(-)
WD_BIN(>>)
WD_BIN(<<)
#undef WD_BIN
WD_FN V operator>>(const V &a, int s) { return a >> V((uint32_t)s); }
WD_FN V operator~(const V &a)
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = ~a.x[i];
    return r;
}
WD_FN M mand(M a, M b) { return M{a.m & b.m}; }
WD_FN M mor(M a, M b) { return M{a.m | b.m}; }
#define WD_CMP(name, op)                                                      \
    WD_FN M name(const V &a, const V &b)                                      \
    {                                                                         \
        uint64_t m = 0;                                                       \
        for (int i = 0; i < 64; ++i) m |= (uint64_t)(a.x[i] op b.x[i]) << i;  \
        return M{m};                                                          \
    }
WD_CMP(eq, ==)
WD_CMP(ne, !=)
WD_CMP(lt, <)
#undef WD_CMP
WD_FN V lane_id()
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = (uint32_t)i;
    return r;
}
WD_FN uint64_t ballot(M m) { return m.m; }
WD_FN uint32_t rdl(const V &v, int l) { return v.x[l]; }
template <int N>
WD_FN V ror(const V &v)
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = v.x[(i & ~15) | ((i + N) & 15)];
    return r;
}
WD_FN V bperm(const V &v, const V &a)
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = v.x[(a.x[i] >> 2) & 63];
    return r;
}
WD_FN V pick(M m, const V &a, const V &b)
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = ((m.m >> i) & 1) ? a.x[i] : b.x[i];
    return r;
}
#define WD_F3(name)                                                             \
    WD_FN V name(const V &a, const V &b, const V &c)                            \
    {                                                                           \
        V r;                                                                    \
        for (int i = 0; i < 64; ++i) r.x[i] = plane::name(a.x[i], b.x[i], c.x[i]); \
        return r;                                                               \
    }
WD_F3(or3)
WD_F3(maj3)
WD_F3(xor3)
WD_F3(andn2)
WD_F3(sel)
WD_F3(bop3_nor)
#undef WD_F3
WD_FN V andn(const V &a, const V &b) { return a & ~b; }
WD_FN V point_rows(const V &y)
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = plane::point_rows(y.x[i]);
    return r;
}
WD_FN V mul24(const V &c, uint32_t k)
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = plane::mul24(c.x[i], k);
    return r;
}
#endif

enum { OPEN = plane::OPEN, DEAD = plane::DEAD, SOLVED = plane::SOLVED, STUCK = plane::STUCK };

// lane roles: lane 16*b + d holds P[d][b]
struct Lanes {
    V d, b;        // digit (0..15; 9..15 pad), band (0..3; 3 pad)
    M valid;       // b < 3 && d < 9
    V word;        // 3d + b: the plane's word in a stack line
    V src1, src2;  // byte addresses (ds_bpermute) of digit d in bands (b+1)%3, (b+2)%3
};
WD_FN Lanes lanes()
{
    Lanes L;
    const V l = lane_id();
    L.d = l & 15u;
    L.b = l >> 4;
    L.valid = mand(lt(L.b, V(3u)), lt(L.d, V(9u)));
    L.word = L.d + L.d + L.d + L.b;
    // nibble b of 0x3021 / 0x3102: (b+1)%3 / (b+2)%3, the pad row itself
    const V sh = L.b << 2;
    L.src1 = ((((V(0x3021u) >> sh) & 15u) << 4) + L.d) << 2;
    L.src2 = ((((V(0x3102u) >> sh) & 15u) << 4) + L.d) << 2;
    return L;
}

// (o, t) = (>= 1, >= 2) over the 16 lanes of each row.  Step N joins the
// window [j, j+N) with [j+N, j+2N): disjoint, so "two" is counted exactly.
WD_FN void row_or_ge2(V &o, V &t)
{
#define WD_STEP(N)                          \
    {                                       \
        const V o2 = ror<N>(o), t2 = ror<N>(t); \
        t = or3(t, t2, o & o2);             \
        o = o | o2;                         \
    }
    WD_STEP(1)
    WD_STEP(2)
    WD_STEP(4)
    WD_STEP(8)
#undef WD_STEP
}
// candidate counts over the row's nine digit lanes, saturating: t >= 2,
// th >= 3, f >= 4 (row-uniform; o = the lane's word, pad lanes 0)
WD_FN void row_count234(V o, V &t, V &th, V &f)
{
    t = V(0u);
    th = V(0u);
    f = V(0u);
#define WD_STEP(N)                                                            \
    {                                                                         \
        const V o2 = ror<N>(o), t2 = ror<N>(t), h2 = ror<N>(th), f2 = ror<N>(f); \
        f = or3(or3(f, f2, th & o2), t & t2, o & h2);                         \
        th = or3(or3(th, h2, t & o2), o & t2, V(0u));                         \
        t = or3(t, t2, o & o2);                                               \
        o = o | o2;                                                           \
    }
    WD_STEP(1)
    WD_STEP(2)
    WD_STEP(4)
    WD_STEP(8)
#undef WD_STEP
}

WD_FN V row_or(V v)
{
    v = v | ror<1>(v);
    v = v | ror<2>(v);
    v = v | ror<4>(v);
    v = v | ror<8>(v);
    return v;
}

// One pass over the board (rules A, B, C; plane::pass's contract).  det: the
// band's cells already eliminated from their peers (row-uniform); und: the
// band's undetermined cells (row-uniform, rows 0-2).
WD_FN int pass(V &w, V &det, V &und, const Lanes &L)
{
    // ---- A: determined cells of each band (over the row's nine digits)
    V o = w, t = V(0u);
    row_or_ge2(o, t);
    const V single = andn(o, t);
    M dead = mand(L.valid, ne(o, V(ROWS)));  // a cell with no candidate
    const V nd = andn(single, det);
    det = single;
    und = andn(V(ROWS), single);
    const bool all_single = ballot(mand(L.valid, ne(single, V(ROWS)))) == 0;
    const bool any_nd = ballot(ne(nd, V(0u))) != 0;

    // ---- B: digit d leaves the peers of the newly determined cells holding d
    const V x = nd & w;
    const V f = or3(x, x >> 10, x >> 20) & 0x1FFu;  // columns holding x in this band
    const V cpeer = mul24(or3(f, bperm(f, L.src1), bperm(f, L.src2)), 0x100401u);
    const V g = or3(f, f >> 1, f >> 2);  // box bits 0/3/6
    const V rn = (x + ROWS) & GUARDS;    // rows holding x
    const V peer = or3(rn - (rn >> 9), cpeer, mul24(g & BOXC, 0x701C07u));
    w = sel(peer, x, w);

    // ---- C: places of d per row / box of the band, per column over the bands
    const V y = w;
    const V y1 = y + ROWS;  // row guard set iff the row has a place
    dead = mor(dead, mand(L.valid, ne(y1 & GUARDS, V(GUARDS))));
    const V z = y & y1;  // y without its lowest place per row
    const V nz = (z + ROWS) & GUARDS;
    const V gr = nz - (nz >> 9);  // rows with >= 2 places
    const V s1 = y >> 10, s2 = y >> 20;
    const V oc = or3(y, s1, s2) & 0x1FFu;   // columns with >= 1 place in the band
    const V tc = maj3(y, s1, s2) & 0x1FFu;  //              >= 2
    const V o1 = oc >> 1, o2 = oc >> 2;
    const V ob = or3(oc, o1, o2);
    dead = mor(dead, mand(L.valid, ne(ob & BOXC, V(BOXC))));  // a box with no place
    const V tb = or3(tc, tc >> 1, tc >> 2);
    const V mo = maj3(oc, o1, o2);  // box bits: >= 2 columns with a place
    const V hb = mul24(andn2(ob, tb, mo) & BOXC, 0x701C07u);  // boxes with one
    const V oA = bperm(oc, L.src1), oB = bperm(oc, L.src2);
    const V tA = bperm(tc, L.src1), tB = bperm(tc, L.src2);
    const V O = or3(oc, oA, oB);
    dead = mor(dead, mand(L.valid, ne(O, V(0x1FFu))));  // a column with no place
    const V hcol = mul24(andn2(O, or3(tc, tA, tB), maj3(oc, oA, oB)) & 0x1FFu, 0x100401u);
    const V hall = y & bop3_nor(gr, hb, hcol);  // d's hidden singles (and d's determined cells)

    // ---- Jacobi: a cell forced for another digit leaves d's plane; forced
    // for two digits it is dead
    V H = hall, H2 = V(0u);
    row_or_ge2(H, H2);
    dead = mor(dead, ne(H2, V(0u)));
    w = andn(w, andn(H, hall));
#ifndef SDK_WIDE_B2
#define SDK_WIDE_B2 1
#endif
#if SDK_WIDE_B2
    {
        // ---- B again, for the cells forced this pass: their digits leave
        // their peers now, not next pass (the lane pass gets the same effect
        // from its Gauss-Seidel order)
        const V x2 = andn(H, det) & w;
        det = det | H;
        const V f2 = or3(x2, x2 >> 10, x2 >> 20) & 0x1FFu;
        const V cp2 = mul24(or3(f2, bperm(f2, L.src1), bperm(f2, L.src2)), 0x100401u);
        const V g2 = or3(f2, f2 >> 1, f2 >> 2);
        const V rn2 = (x2 + ROWS) & GUARDS;
        w = sel(or3(rn2 - (rn2 >> 9), cp2, mul24(g2 & BOXC, 0x701C07u)), x2, w);
    }
#endif
#if SDK_WIDE_LC
    {
        // ---- D (plane::pass rule D): a box whose places lie in one column
        // takes d out of that column in the other bands (columns from this
        // pass's y: a superset of the places now, so still sound); likewise
        // for a row.
        const V vp = oc & mul24(andn(xor3(oc, o1, o2), mo) & BOXC, 7u);
        V ec = V(0u);
#if SDK_WIDE_LC & 1
        ec = andn(or3(vp, bperm(vp, L.src1), bperm(vp, L.src2)), vp);
#endif
#if SDK_WIDE_LC & 4
        {
            const V cc = oc & (andn(xor3(oc, oA, oB), maj3(oc, oA, oB)) & 0x1FFu);  // columns only in this band
            ec = ec | andn(mul24(or3(cc, cc >> 1, cc >> 2) & BOXC, 7u), cc);
        }
#endif
        V e = mul24(ec, 0x100401u);
#if SDK_WIDE_LC & 2
        e = e | point_rows(w);
#endif
        w = andn(w, e);
    }
#endif

    if (ballot(dead)) return DEAD;
    if (all_single) return SOLVED;
    const bool newh = ballot(ne(H & und, V(0u))) != 0;
    return (any_nd || newh) ? OPEN : STUCK;  // (rule D alone: not OPEN, as plane::pass)
}

// fix the cell (band, pos) to digit bit dbit
WD_FN void set_cell(V &w, const Lanes &L, int band, int pos, uint32_t dbit)
{
    const M clr = mand(mand(L.valid, eq(L.b, V((uint32_t)band))), eq((V(dbit) >> L.d) & 1u, V(0u)));
    w = pick(clr, andn(w, V(1u << pos)), w);
}

enum { W_UNSOLVABLE = 0, W_SOLVED = 1, W_OVERFLOW = -1, W_CANCELLED = 2 };

struct Stats {
    uint32_t passes, guesses, bguess;  // bguess: this board's guesses (lane + wide)
};

// the search's hook: cancelled() -- ordered mode, a lower board has a completion
struct NoCancel {
    WD_MF bool cancelled() const { return false; }
};

// Continue the search of the board in w at `depth` (levels below it on the
// stack) to its first completion in walk order.  Stack: push(level, w, L,
// entry), entry(level), restore(level, L), put_entry(level, e) over the
// plane_kernel stack line layout.  hk: the hook above.  mst / mrv_after:
// the board's search mode, as the lane solver's (plane::search_step, the
// same transitions).  Returns W_*; on W_SOLVED w holds the completion.
template <class Stack, class Hook>
WD_FN int solve(V &w, uint32_t &depth, const Stack &stk, const Lanes &L, int node_order, uint32_t max_depth,
                Stats &st, Hook &hk, uint32_t &mst, uint32_t mrv_after)
{
    V det = V(0u);
    const uint32_t sol_level = max_depth - 1;
    for (;;) {
        V und;
        st.passes++;
        int r = pass(w, det, und, L);
        mst++;
        int mode = plane::mst_mode(mst);
        if (r == STUCK && plane::root_counts(mode, depth, mrv_after, rdl(und, 0), rdl(und, 16), rdl(und, 32))) {
            mode = plane::M_COUNT;  // a wide-open root: count at once (plane::search_step)
            mst = plane::mst_set_mode(mst, plane::M_COUNT);
        }
        if (mode == plane::M_WALK && mrv_after && r != SOLVED && (mst & plane::MST_PASSES) >= mrv_after) {
            if (depth) w = stk.restore(0, L);  // the propagated root
            det = V(0u);
            depth = 0;
            mst = plane::mst_set_mode(mst, plane::M_COUNT);
            continue;
        }
        if (r == OPEN) continue;
        if (r == SOLVED) {
            if (mode != plane::M_COUNT) return W_SOLVED;
            if (mst & plane::MST_FOUND) {  // a second completion: the walk, from the root
                w = stk.restore(0, L);
                det = V(0u);
                depth = 0;
                mst = plane::mst_set_mode(mst, plane::M_FINAL);
                continue;
            } else {
                mst |= plane::MST_FOUND;
                stk.push(sol_level, w, L, 0u);
                r = DEAD;
            }
        }
        if (r == STUCK) {
            if (depth == (mode == plane::M_COUNT ? sol_level : max_depth)) {
                if (mode != plane::M_COUNT) return W_OVERFLOW;
                w = stk.restore(0, L);  // too deep to count: the walk, from the root
                det = V(0u);
                depth = 0;
                mst = plane::mst_set_mode(mst, plane::M_FINAL);
                continue;
            }
            if (hk.cancelled()) return W_CANCELLED;
            const uint32_t u[3] = {rdl(und, 0), rdl(und, 16), rdl(und, 32)};
            int band, pos;
            if (mode == plane::M_COUNT) {
                V t, th, f;
                row_count234(pick(L.valid, w, V(0u)), t, th, f);
                const V e2 = und & andn(t, th), e3 = und & andn(th, f);
                const uint32_t m2[3] = {rdl(e2, 0), rdl(e2, 16), rdl(e2, 32)};
                const uint32_t m3[3] = {rdl(e3, 0), rdl(e3, 16), rdl(e3, 32)};
                plane::pick_mrv_masks(m2, m3, u, band, pos);
            } else {
                plane::pick_cell(u, node_order, band, pos);
            }
            const uint64_t cm = ballot(mand(mand(L.valid, eq(L.b, V((uint32_t)band))), ne((w >> pos) & 1u, V(0u))));
            const uint32_t cand = (uint32_t)(cm >> (16 * band)) & 0x1FFu;
            const uint32_t dbit = cand & (0u - cand);
            stk.push(depth, w, L, plane::make_entry(band, pos, cand ^ dbit));
            depth++;
            st.guesses++;
            st.bguess++;
            set_cell(w, L, band, pos, dbit);
            continue;
        }
        // DEAD: back to the deepest level with an untried digit
        for (;;) {
            if (depth == 0) {
                if (mode == plane::M_COUNT && (mst & plane::MST_FOUND)) {  // exactly one completion
                    w = stk.restore(sol_level, L);
                    return W_SOLVED;
                }
                return W_UNSOLVABLE;
            }
            depth--;
            const uint32_t e = stk.entry(depth);
            const uint32_t rem = (e >> 8) & 0x1FFu;
            if (!rem) continue;
            const uint32_t dbit = rem & (0u - rem);
            w = stk.restore(depth, L);
            det = V(0u);
#if SDK_PLANE_LASTPOP
            if (rem != dbit || depth == 0) {  // (a level's last digit: continue at its depth, plane_solver.h)
                stk.put_entry(depth, e & ~(dbit << 8));
                depth++;
            }
#else
            stk.put_entry(depth, e & ~(dbit << 8));
            depth++;
#endif
            st.guesses++;
            st.bguess++;
            set_cell(w, L, (int)((e >> 5) & 3u), (int)(e & 31u), dbit);
            break;
        }
    }
}

// Value bit-slices of a solved board: slice k (k = 0..3) of band b, in every
// lane of row b (bit pos = bit k of the value at pos)
WD_FN void value_slices(const V &w, const Lanes &L, V (&s)[4])
{
    const V dv = L.d + 1u;
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = row_or(pick(ne((dv >> k) & 1u, V(0u)), w, V(0u)));
}

}  // namespace wide

#endif  // SDK_PLANE_WIDE_H
