// plane_quad.h -- FOUR boards over one wave, on the digit planes of
// plane_solver.h: the tail pool's solver (plane_kernel.h).
//
// Why: at the end of a launch the XCD tail pool holds ~12 boards per wave,
// the heaviest residual searches of the launch, and the one-board-per-wave
// solver (plane_wide.h: lane 16b+d holds P[d][b], ~200 wave instructions
// per pass, latency-bound on its DPP / ds_bpermute chains) spends ~200 wave
// instructions per board-pass there -- ten times a lane pass's share.  Here
// row q of the wave (lanes 16q..16q+15) holds board q, lane 16q+d the three
// band words of digit d (d < 9; lanes 9..15 of a row hold 0): cross-digit
// sums are DPP row rotations within the row, exactly as in plane_wide.h,
// and cross-band sums (columns) stay inside a lane, so there is no
// ds_bpermute at all.  One pass over four boards is ~300 wave instructions
// (~75 per board-pass), and the four rows' searches step independently
// (plane_kernel.h plane_quad_drain).
//
// The pass is plane_wide.h's rule set and order (A naked singles, B peer
// elimination, C hidden singles per digit, Jacobi over digits with a cell
// forced twice dead, B again for the cells forced this pass), so it reaches
// the same fixpoints, branch cells and first completions;
// tests/native/wide_host.cpp checks it against the lane pass.
#ifndef SDK_PLANE_QUAD_H
#define SDK_PLANE_QUAD_H

#include "plane_wide.h"

namespace quad {

using plane::BOXC;
using plane::GUARDS;
using plane::ROWS;
using wide::M;
using wide::V;

enum { OPEN = plane::OPEN, DEAD = plane::DEAD, SOLVED = plane::SOLVED, STUCK = plane::STUCK };

// lane roles: lane 16q + d holds digit d of board q (row q)
struct Lanes {
    V d, q;     // digit (0..15; 9..15 pad), row / board slot (0..3)
    M valid;    // d < 9
    V rowsh;    // 16 q: the row's bit offset in a ballot
};
WD_FN Lanes lanes()
{
    Lanes L;
    const V l = wide::lane_id();
    L.d = l & 15u;
    L.q = l >> 4;
    L.valid = wide::lt(L.d, V(9u));
    L.rowsh = L.q << 4;
    return L;
}

// this lane's row's 16 bits of a ballot
#if defined(__HIPCC__)
WD_FN V row_bits(uint64_t m, const Lanes &L) { return (V)(m >> L.rowsh) & 0xFFFFu; }
#else
WD_FN V row_bits(uint64_t m, const Lanes &L)
{
    V r;
    for (int i = 0; i < 64; ++i) r.x[i] = (uint32_t)(m >> L.rowsh.x[i]) & 0xFFFFu;
    return r;
}
#endif
// "some lane of my row": a row-uniform flag
WD_FN M row_any(M f, const Lanes &L) { return wide::ne(row_bits(wide::ballot(f), L), V(0u)); }

// B: digit d (this lane's) leaves the peers of the newly determined cells
// x[b] (cells of d's plane that just became determined)
WD_FN void eliminate(V (&w)[3], const V (&x)[3])
{
    V f[3];
#pragma unroll
    for (int b = 0; b < 3; ++b) f[b] = wide::or3(x[b], x[b] >> 10, x[b] >> 20) & 0x1FFu;  // columns holding x
    const V cpeer = wide::mul24(wide::or3(f[0], f[1], f[2]), 0x100401u);
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const V g = wide::or3(f[b], f[b] >> 1, f[b] >> 2);  // box bits 0/3/6
        const V rn = (x[b] + ROWS) & GUARDS;                // rows holding x
        const V peer = wide::or3(rn - (rn >> 9), cpeer, wide::mul24(g & BOXC, 0x701C07u));
        w[b] = wide::sel(peer, x[b], w[b]);
    }
}

// One pass over the four boards (rules A, B, C; plane::pass's contract, per
// row).  det: each band's cells already eliminated from their peers; und:
// the undetermined cells (both row-uniform).  Returns the row's result
// (row-uniform).  Pad lanes (d >= 9) must hold 0 in w and stay 0.
WD_FN V pass(V (&w)[3], V (&det)[3], V (&und)[3], const Lanes &L)
{
    // ---- A: determined cells of each band (over the row's nine digits)
    V nd[3], single[3];
    M dead = M{};
    V any_nd = V(0u), all = V(ROWS);
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        V o = w[b], t = V(0u);
        wide::row_or_ge2(o, t);
        single[b] = wide::andn(o, t);
        dead = wide::mor(dead, wide::ne(o, V(ROWS)));  // a cell with no candidate (row-uniform)
        nd[b] = wide::andn(single[b], det[b]);
        det[b] = single[b];
        und[b] = wide::andn(V(ROWS), single[b]);
        any_nd = any_nd | nd[b];
        all = all & single[b];
    }

    // ---- B: this lane's digit leaves the peers of the newly determined cells holding it
    {
        V x[3];
#pragma unroll
        for (int b = 0; b < 3; ++b) x[b] = nd[b] & w[b];
        eliminate(w, x);
    }

    // ---- C: places of this lane's digit per row / box of each band, per column over the bands
    V oc[3], tc[3], gr[3], hb[3];
#if SDK_WIDE_LC
    V vp[3];
#endif
    V rowall = V(GUARDS), boxall = V(BOXC);
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const V y = w[b];
        const V y1 = y + ROWS;  // row guard set iff the row has a place
        rowall = rowall & y1;
        const V z = y & y1;  // y without its lowest place per row
        const V nz = (z + ROWS) & GUARDS;
        gr[b] = nz - (nz >> 9);  // rows with >= 2 places
        const V s1 = y >> 10, s2 = y >> 20;
        oc[b] = wide::or3(y, s1, s2) & 0x1FFu;   // columns with >= 1 place in the band
        tc[b] = wide::maj3(y, s1, s2) & 0x1FFu;  //              >= 2
        const V o1 = oc[b] >> 1, o2 = oc[b] >> 2;
        const V ob = wide::or3(oc[b], o1, o2);
        boxall = boxall & ob;
        const V tb = wide::or3(tc[b], tc[b] >> 1, tc[b] >> 2);
        const V mo = wide::maj3(oc[b], o1, o2);  // box bits: >= 2 columns with a place
        hb[b] = wide::mul24(wide::andn2(ob, tb, mo) & BOXC, 0x701C07u);  // boxes with one
#if SDK_WIDE_LC
        vp[b] = oc[b] & wide::mul24(wide::andn(wide::xor3(oc[b], o1, o2), mo) & BOXC, 7u);  // rule D
#endif
    }
    const V O = wide::or3(oc[0], oc[1], oc[2]);
    const V hcol = wide::mul24(wide::andn2(O, wide::or3(tc[0], tc[1], tc[2]), wide::maj3(oc[0], oc[1], oc[2])) & 0x1FFu,
                               0x100401u);
    // a unit with no place for this digit (pad lanes have none: masked)
    const M unit_dead = wide::mor(wide::mor(wide::ne(rowall & GUARDS, V(GUARDS)), wide::ne(O, V(0x1FFu))),
                                  wide::ne(boxall & BOXC, V(BOXC)));
    dead = wide::mor(dead, row_any(wide::mand(L.valid, unit_dead), L));
    V hall[3];
#pragma unroll
    for (int b = 0; b < 3; ++b) hall[b] = w[b] & wide::bop3_nor(gr[b], hb[b], hcol);  // the digit's hidden singles

    // ---- Jacobi: a cell forced for another digit leaves this digit's plane;
    // forced for two digits it is dead
    V H[3], newh = V(0u);
    M twice = M{};
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        V h2 = V(0u);
        H[b] = hall[b];
        wide::row_or_ge2(H[b], h2);
        twice = wide::mor(twice, wide::ne(h2, V(0u)));
        w[b] = wide::andn(w[b], wide::andn(H[b], hall[b]));
        newh = newh | (H[b] & und[b]);
    }
    dead = wide::mor(dead, twice);
    // ---- B again, for the cells forced this pass
    {
        V x2[3];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            x2[b] = wide::andn(H[b], det[b]) & w[b];
            det[b] = det[b] | H[b];
        }
        eliminate(w, x2);
    }
#if SDK_WIDE_LC
    {
        // ---- D (plane::pass rule D): a box whose places lie in one column
        // takes the digit out of that column in the other bands; likewise
        // for a row
        const V vpa = wide::or3(vp[0], vp[1], vp[2]);
        const V one_band = wide::andn(wide::xor3(oc[0], oc[1], oc[2]), wide::maj3(oc[0], oc[1], oc[2])) & 0x1FFu;
        (void)vpa;
        (void)one_band;
        V lc = V(0u);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            V ec = V(0u);
#if SDK_WIDE_LC & 1
            ec = wide::andn(vpa, vp[b]);
#endif
#if SDK_WIDE_LC & 4
            {
                const V cc = oc[b] & one_band;
                ec = ec | wide::andn(wide::mul24(wide::or3(cc, cc >> 1, cc >> 2) & BOXC, 7u), cc);
            }
#endif
            V e = wide::mul24(ec, 0x100401u);
#if SDK_WIDE_LC & 2
            e = e | wide::point_rows(w[b]);
#endif
            lc = lc | (w[b] & e);
            w[b] = wide::andn(w[b], e);
        }
        newh = newh | wide::row_or(lc);
    }
#endif
    const M solved = wide::eq(all, V(ROWS));
    const M open = wide::ne(any_nd | newh, V(0u));
    return wide::pick(dead, V((uint32_t)DEAD), wide::pick(solved, V((uint32_t)SOLVED),
                                                           wide::pick(open, V((uint32_t)OPEN), V((uint32_t)STUCK))));
}

}  // namespace quad

#endif  // SDK_PLANE_QUAD_H
