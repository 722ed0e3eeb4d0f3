// trellis_dense.h -- the deletion trellises of one segment without guard-band ones, in dense edge
// slots (host + device).  Same stages, same values and orders as trellis_body.h's Trel (round 5).
//
// Status: not on the shipped path.  As a lane-serial drop-in for Trel in DelBase / DelNode it
// decoded bit-exactly (the whole GPU suite) at half the rate -- n = 12 (n0 = 4) 34.6 k -> 16.4 k
// cw/s: its creation-order scans cost more private-memory reads than Trel's index saves, and
// halving the private segment did not raise residency.  It is the validated representation for
// the 16-lane-group kernel of DESIGN.md section 9 (slots a lane each, ranks by first contribution).
//
// Restates, for the n0 >= 3 path without guard-band ones (as DelBase / DelNode do with Trel):
//   BinaryTrellis.__miusPlusTransform                 VectorDistributions/BinaryTrellis.py:206-258
//   BinaryTrellis.calcNormalizationVector / normalize VectorDistributions/BinaryTrellis.py:280-306
//   the collection collapse                           VectorDistributions/CollectionOfBinaryTrellises.py:68-82
//
// Why a second representation.  A Trel keeps each edge layer as creation-ordered arrays plus
// direct-mapped lookups (vertex index per vpos, edge index per vertex pair and label) and a
// counting-sort index by from- and to-vertex, all at worst-case capacity: 22.6 KB a lane at
// n0 = 4, most of it touched by every transform.  Here an edge lives at a fixed slot of its
// layer, indexed by (from position - the layer's window start, advance - the least advance,
// label): the slot is the lookup.  Every vertex of a depth-d trellis's layer j lies in the base
// layer's window [max(0, j 2^d - dd), min(j 2^d, m)] (dd = L - m deletions; trellis_body.h's
// capacity note), and an edge spans 2^d base steps, each advancing vpos by 0 or 1 with at most dd
// deletions in all, so its advance is in [max(0, 2^d - dd), 2^d]: V = L/2 + 1 window positions
// and min(2^d, L/2) + 1 advances a layer.
//
// Orders.  The reference's sums run over insertion-ordered dicts; as in Trel, a layer keeps its
// edges' creation order (eord: slot of the r-th created edge; crank: the rank of a slot) and its
// vertices' insertion order (vord / vrank), and every loop walks them in that order: "vertices in
// order, then that vertex's out-edges in creation order" is a scan of the creation order filtered
// by from-vertex, so no index is built.  tests/emu/dtrel_check.cpp compares every stage with
// Trel's on random segments and decision histories: the same edges, the same creation and
// insertion orders, bit-identical probabilities and collapsed values.
#pragma once
#include "trellis_body.h"

namespace pcub {

// A depth-D trellis of the base length L (LEN = L >> D layers).
template <int L, int D>
struct DTrel {
    static constexpr int LEN = L >> D;
    static constexpr int V = L / 2 + 1;                        // window positions a layer
    static constexpr int NA = ((1 << D) < L / 2 ? (1 << D) : L / 2) + 1;  // advances an edge layer
    static constexpr int S = V * NA * 2;                      // slots an edge layer
    static_assert(S <= 255, "slot ids and ranks in bytes");
    int m, dd;                    // received symbols, deletions (L - m)
    // vrank / crank are validated on use (present iff rank < count and the order array points back),
    // so a clear touches only the counts, as Trel's direct-mapped lookups
    uint8_t nv[LEN + 1];
    uint8_t vord[LEN + 1][V];     // window offsets in insertion order
    uint8_t vrank[LEN + 1][V];    // insertion rank of a window offset
    uint8_t ne[LEN];
    uint8_t eord[LEN][S];         // slots in creation order
    uint8_t crank[LEN][S];        // creation rank of a slot
    double p[LEN][S];

    PCUB_HD int lo(int l) const {
        const int b = l << D;
        return b - dd > 0 ? b - dd : 0;
    }
    PCUB_HD int amin() const { return (1 << D) - dd > 0 ? (1 << D) - dd : 0; }
    PCUB_HD int slot(int l, int u, int v, int x) const { return ((u - lo(l)) * NA + (v - u - amin())) * 2 + x; }
    PCUB_HD int s_from(int l, int s) const { return lo(l) + (s >> 1) / NA; }
    PCUB_HD int s_to(int l, int s) const { return s_from(l, s) + ((s >> 1) % NA) + amin(); }
    static PCUB_HD int s_lbl(int s) { return s & 1; }

    PCUB_HD void clear(int m_) {
        m = m_;
        dd = L - m_;
        for (int l = 0; l <= LEN; ++l) nv[l] = 0;
        for (int l = 0; l < LEN; ++l) ne[l] = 0;
    }
    // __getVertexAndAddIfNeeded (BinaryTrellis.py:155-162)
    PCUB_HD void vertex(int l, int vpos) {
        const int o = vpos - lo(l);
        const int r = vrank[l][o];
        if (r < nv[l] && vord[l][r] == o) return;
        vrank[l][o] = nv[l];
        vord[l][nv[l]] = (uint8_t)o;
        ++nv[l];
    }
    // the interface trellis_transform_base drives (vertex probabilities are 1.0 without ones)
    PCUB_HD void clear() {}
    PCUB_HD void set_prob(int l, int vpos, double) {
        if (m <= L) vertex(l, vpos);
    }
    PCUB_HD void index() {}
    // addToEdgeProb (BinaryTrellis.py:128-136)
    PCUB_HD void add(int l, int u, int v, int x, double prob) {
        vertex(l, u);
        vertex(l + 1, v);
        const int s = slot(l, u, v, x);
        const int r = crank[l][s];
        if (r < ne[l] && eord[l][r] == s) {
            p[l][s] += prob;
            return;
        }
        crank[l][s] = ne[l];
        eord[l][ne[l]] = (uint8_t)s;
        ++ne[l];
        p[l][s] = 0.0 + prob;
    }
};

// trellis_transform_base into a dense child (m > L: no edges, only the two end vertices, as Trel)
template <int L, int D>
PCUB_HD void dtrellis_transform_base(const BaseT<L>& b, DTrel<L, D>& ct, const uint32_t* dec) {
    ct.clear(b.m);
    if (b.m > L) {
        // Trel: set_prob(0, 0), set_prob(H, m) -- vertices outside any window; no edge reads them
        ct.nv[0] = 1;
        ct.nv[DTrel<L, D>::LEN] = 1;
        return;
    }
    trellis_transform_base<L>(b, ct, dec);
}

// __miusPlusTransform of a dense parent (trellis_transform's iteration: middle vertices in
// insertion order, their in-edges in creation order, for each their out-edges in creation order)
template <int L, int D>
PCUB_HD void dtrellis_transform(const DTrel<L, D>& pt, DTrel<L, D + 1>& ct, const uint32_t* dec) {
    constexpr int H = DTrel<L, D + 1>::LEN;
    ct.clear(pt.m);
    if (pt.m > L) {
        ct.nv[0] = 1;
        ct.nv[H] = 1;
        return;
    }
    ct.vertex(0, 0);
    ct.vertex(H, pt.m);
    for (int j = 0; j < H; ++j) {
        const int mid = 2 * j + 1;
        const int dj = dec ? (int)((*dec >> j) & 1u) : 0;
        const int lm = pt.lo(mid);
        for (int wi = 0; wi < pt.nv[mid]; ++wi) {
            const int w = lm + pt.vord[mid][wi];
            for (int ia = 0; ia < pt.ne[mid - 1]; ++ia) {
                const int a = pt.eord[mid - 1][ia];
                if (pt.s_to(mid - 1, a) != w) continue;
                const int u = pt.s_from(mid - 1, a), la = DTrel<L, D>::s_lbl(a);
                const double pa = pt.p[mid - 1][a];
                for (int ib = 0; ib < pt.ne[mid]; ++ib) {
                    const int bs = pt.eord[mid][ib];
                    if (pt.s_from(mid, bs) != w) continue;
                    const int v = pt.s_to(mid, bs), lb = DTrel<L, D>::s_lbl(bs);
                    const double prob = pa * pt.p[mid][bs];
                    const int ml = la ^ lb;
                    if (!dec) ct.add(j, u, v, ml, prob);
                    else if (ml == dj) ct.add(j, u, v, lb, prob);
                }
            }
        }
    }
}

// calcNormalizationVector + normalize (trellis_normalize's order: vertices in insertion order, then
// their out-edges in creation order)
template <int L, int D>
PCUB_HD void dtrellis_normalize(DTrel<L, D>& t) {
    constexpr int LEN = DTrel<L, D>::LEN;
    for (int i = 0; i < LEN; ++i) {
        double s0 = 0.0, s1 = 0.0;
        const int li = t.lo(i);
        for (int vi = 0; vi < t.nv[i]; ++vi) {
            const int vp = li + t.vord[i][vi];
            for (int ie = 0; ie < t.ne[i]; ++ie) {
                const int s = t.eord[i][ie];
                if (t.s_from(i, s) != vp) continue;
                if (DTrel<L, D>::s_lbl(s)) s1 += t.p[i][s];
                else s0 += t.p[i][s];
            }
        }
        double d = s0 >= s1 ? s0 : s1;
        if (d == 0.0) d = 1.0;
        for (int ie = 0; ie < t.ne[i]; ++ie) t.p[i][t.eord[i][ie]] /= d;
    }
}

// trellis_collapse of a dense length-2 trellis (no ones: the child's marginal is the per-label sum of
// the transform's contributions in its iteration order)
template <int L, int D>
PCUB_HD void dtrellis_collapse(const DTrel<L, D>& pt, const uint32_t* dec, double& m0, double& m1) {
    static_assert(DTrel<L, D>::LEN == 2, "length-2 trellis");
    m0 = 0.0;
    m1 = 0.0;
    if (pt.m > L) return;
    const int dj = dec ? (int)(*dec & 1u) : 0;
    const int l1 = pt.lo(1);
    for (int wi = 0; wi < pt.nv[1]; ++wi) {
        const int w = l1 + pt.vord[1][wi];
        for (int ia = 0; ia < pt.ne[0]; ++ia) {
            const int a = pt.eord[0][ia];
            if (pt.s_to(0, a) != w) continue;
            const int la = DTrel<L, D>::s_lbl(a);
            for (int ib = 0; ib < pt.ne[1]; ++ib) {
                const int bs = pt.eord[1][ib];
                if (pt.s_from(1, bs) != w) continue;
                const int lb = DTrel<L, D>::s_lbl(bs);
                const double prob = pt.p[0][a] * pt.p[1][bs];
                const int ml = la ^ lb;
                int x = ml;
                if (dec) {
                    if (ml != dj) continue;
                    x = lb;
                }
                if (x) m1 += prob;
                else m0 += prob;
            }
        }
    }
}

}  // namespace pcub
