// trellis_body.h -- deletion-channel trellis stages of the SC decoder (host + device).
//
// Replaces, per (codeword, trellis) lane:
//   Guardbands.removeDeletionGuardBands / trimZerosAtEdges    Guardbands.py:47-93
//   BinaryTrellis.buildTrellis_uniformInput_deletion          VectorDistributions/BinaryTrellis.py:309-438
//   BinaryTrellis.__miusPlusTransform                         VectorDistributions/BinaryTrellis.py:206-258
//   BinaryTrellis.calcNormalizationVector / normalize         VectorDistributions/BinaryTrellis.py:280-306
//   BinaryTrellis.calcMarginalizedProbabilities(normalize=False), as called by the
//   collection collapse                                      VectorDistributions/CollectionOfBinaryTrellises.py:68-82
// for a single-state, uniform-input trellis, with or without guard-band ones
// (numberOfOnesToAddAtBothEndsOfGuardbands; main_deletion.py's default is 0).
//
// Order of floating-point sums.  The reference keeps vertices and edges in
// insertion-ordered dicts and every sum (edge accumulation in a transform, the
// per-layer normaliser, the marginal) runs in that order.  A vertex's out-edges
// (in-edges) in dict order are exactly the edges leaving (entering) it in
// CREATION order, so each edge layer is stored as an append-only array in
// creation order, and each vertex layer as an append-only list of vpos values
// in insertion order.  Iterating "vertices of layer i in order, then the edge
// array filtered by from-vertex" is then the reference's iteration, and all
// sums are formed in the same order (tests/test_trellis_* pin this bit-exactly).
// The layers are indexed (Trel::index) so that iteration touches only the vertex's own edges.
// Vertex probabilities matter only on the first and last layer (the marginal of a
// length-1 trellis, :260-278); they are kept for those two layers.
//
// Capacities (OC = the most guard-band ones the instantiation accepts).  Base layer
// l of a trellis of length L with m received symbols and `ones` ones holds vpos in
// [max(0, l + ones - dc), min(l + ones, m)], dc = L + 2 ones - m: at most
// V = L/2 + 1 + ones vertices.  A transformed trellis's layer j is a subset of base
// layer j*2^d, so every layer of every depth has at most V vertices; a base edge
// layer has at most 3V edges (one insertion, two deletions per vertex) and an edge of
// a depth-d trellis spans 2^d base layers, so it advances vpos by 0 .. 2^d: at most
// 2V(2^d + 1) edges (one per from-vertex, advance, label), and never more than 2V^2.
#pragma once
#include <type_traits>

#include "sc_common.h"

namespace pcub {

// edge key: from vpos (15 bits) | to vpos (15 bits) | label
PCUB_HD uint32_t ekey(int u, int v, int x) { return ((uint32_t)u << 16) | ((uint32_t)v << 1) | (uint32_t)x; }
PCUB_HD int ek_from(uint32_t k) { return (int)(k >> 16); }
PCUB_HD int ek_to(uint32_t k) { return (int)((k >> 1) & 0x7fffu); }
PCUB_HD int ek_lbl(uint32_t k) { return (int)(k & 1u); }

template <int LEN, int V, int E>
struct Trel {
    // edge indices and counts in the narrowest type that holds E (private memory is the
    // deletion kernel's working set: every byte here is per trellis lane)
    using EI = typename std::conditional<(E <= 127), int8_t, int16_t>::type;
    // direct-mapped lookups (validated on use, so they are never cleared): vertex index of a
    // vpos per layer, edge index of (from vertex, to vertex, label) per edge layer.  Without
    // them every addToEdgeProb is a linear search of the layer's edges, a chain of dependent
    // private-memory loads on the GPU.  vpos >= VPM (only when a guard-band parse hands a
    // segment longer than its trellis) falls back to the search.
    static constexpr int VPM = 2 * V + 2;
    int8_t nv[LEN + 1];     // vertices per layer
    int16_t vp[LEN + 1][V]; // vpos in insertion order
    double pr0[V];          // vertex probabilities of layer 0 (insertion order)
    double prL[V];          // ... and of layer LEN
    EI ne[LEN];             // edges per edge layer
    uint32_t key[LEN][E];   // creation order
    double p[LEN][E];
    int8_t vidx[LEN + 1][VPM];
    EI lut[LEN][V][V][2];
    // per edge: from / to vertex index; after index(): the edges of each layer grouped by
    // from-vertex and by to-vertex, each group in creation order (a stable counting sort), so
    // "vertices in order, then that vertex's edges in creation order" -- the reference's
    // iteration -- touches only those edges
    int8_t efv[LEN][E], etv[LEN][E];
    EI byfrom[LEN][E], byto[LEN][E];
    EI fstart[LEN][V + 1], tstart[LEN][V + 1];

    PCUB_HD void clear() {
        for (int l = 0; l <= LEN; ++l) nv[l] = 0;
        for (int l = 0; l < LEN; ++l) ne[l] = 0;
    }
    // __getVertexAndAddIfNeeded (BinaryTrellis.py:155-162); returns the vertex's index
    PCUB_HD int vertex(int l, int vpos) {
        const int c = nv[l];
        if (vpos >= 0 && vpos < VPM) {
            const int i = vidx[l][vpos];
            if (i >= 0 && i < c && vp[l][i] == vpos) return i;
        } else {
            for (int i = 0; i < c; ++i)
                if (vp[l][i] == vpos) return i;
        }
        vp[l][c] = (int16_t)vpos;
        if (vpos >= 0 && vpos < VPM) vidx[l][vpos] = (int8_t)c;
        nv[l] = (int8_t)(c + 1);
        return c;
    }
    // setVertexProb (BinaryTrellis.py:123-125), first / last layer
    PCUB_HD void set_prob(int l, int vpos, double prob) {
        const int i = vertex(l, vpos);
        if (l == 0) pr0[i] = prob;
        else prL[i] = prob;
    }
    PCUB_HD double prob_last(int vpos) const {
        for (int i = 0; i < nv[LEN]; ++i)
            if (vp[LEN][i] == vpos) return prL[i];
        return 1.0;
    }
    // addToEdgeProb (BinaryTrellis.py:128-136): from-vertex, to-vertex, then the edge (+= p)
    PCUB_HD void add(int l, int u, int v, int x, double prob) {
        const int ui = vertex(l, u);
        const int vi = vertex(l + 1, v);
        const uint32_t k = ekey(u, v, x);
        const int c = ne[l];
        const int e = lut[l][ui][vi][x];
        if (e >= 0 && e < c && key[l][e] == k) {
            p[l][e] += prob;
            return;
        }
        key[l][c] = k;
        p[l][c] = 0.0 + prob;
        efv[l][c] = (int8_t)ui;
        etv[l][c] = (int8_t)vi;
        lut[l][ui][vi][x] = (EI)c;
        ne[l] = (EI)(c + 1);
    }
    // group every edge layer by from-vertex and by to-vertex (structure only: p may change later)
    PCUB_HD void index() {
        for (int l = 0; l < LEN; ++l) {
            const int n = ne[l];
            for (int v = 0; v <= V; ++v) fstart[l][v] = tstart[l][v] = 0;
            for (int e = 0; e < n; ++e) {
                ++fstart[l][efv[l][e] + 1];
                ++tstart[l][etv[l][e] + 1];
            }
            for (int v = 0; v < V; ++v) {
                fstart[l][v + 1] += fstart[l][v];
                tstart[l][v + 1] += tstart[l][v];
            }
            EI fp[V], tp[V];
            for (int v = 0; v < V; ++v) {
                fp[v] = fstart[l][v];
                tp[v] = tstart[l][v];
            }
            for (int e = 0; e < n; ++e) {
                byfrom[l][fp[efv[l][e]]++] = (EI)e;
                byto[l][tp[etv[l][e]]++] = (EI)e;
            }
        }
    }
};

// capacities of the trellises of base length L accepting up to OC guard-band ones
template <int L, int OC = 0>
struct DelCap {
    static constexpr int V = L / 2 + 1 + OC;
    static constexpr int E0 = 3 * V;  // base edge layer
    // edge layer of a depth-d trellis (d >= 1)
    static constexpr int E(int d) { return 2 * V * V < 2 * V * ((1 << d) + 1) ? 2 * V * V : 2 * V * ((1 << d) + 1); }
};

// Guard-band vertex probabilities, comb(ones, i) (1-pd)^i pd^(ones-i) for i = 0 .. ones
// (buildTrellis_uniformInput_deletion, BinaryTrellis.py:343-345, 371-373), computed on the
// host with libm pow -- the function CPython's float ** int calls -- so they are the
// reference's values bit for bit.
struct OnesProbs {
    int ones;
    double pr[4];
};

// The base trellis of one segment, word[s .. s+m) (buildTrellis_uniformInput_deletion,
// trimmed edges, op.ones guard-band ones).  `bit(i)` returns received symbol i of the codeword.
template <int L, class T, class BitF>
PCUB_HD void trellis_build(T& t, const BitF& bit, int s, int m, double pd, const OnesProbs& op = OnesProbs{0, {1.0}}) {
    t.clear();
    const int ones = op.ones;
    const int dcount = L + 2 * ones - m;
    if (ones > 0) {
        const int k = ones < m ? ones : m;
        for (int i = 0; i <= k; ++i) t.set_prob(0, i, op.pr[i]);
        for (int i = m; i >= m - k; --i) t.set_prob(L, i, op.pr[m - i]);
    } else {
        t.set_prob(0, 0, 1.0);  // setVertexProb: start vertex, prob 1.0
        t.set_prob(L, m, 1.0);  // end vertex, prob 1.0
    }
    const double p_ins = 0.5 * (1.0 - pd);
    const double p_del = 0.5 * pd;
    for (int l = 0; l < L; ++l) {
        const int lo = l + ones - dcount > 0 ? l + ones - dcount : 0;
        const int hi = l + ones < m ? l + ones : m;
        for (int vp = lo; vp <= hi; ++vp) {
            if (vp < m) t.add(l, vp, vp + 1, bit(s + vp), p_ins);
            if (l + 1 + ones - dcount <= vp) {
                // label 0 then 1; a deletion of a 0 at either trimmed edge is certain
                t.add(l, vp, vp, 0, (vp > 0 && vp < m) ? p_del : 0.5);
                t.add(l, vp, vp, 1, p_del);
            }
        }
    }
    t.index();
}

// __miusPlusTransform (BinaryTrellis.py:206-258).  dec = nullptr: minus; else bit j
// of *dec is decisionVector[j] (plus).
template <int LEN, class P, class C>
PCUB_HD void trellis_transform(const P& pt, C& ct, const uint32_t* dec) {
    constexpr int H = LEN / 2;
    ct.clear();
    for (int i = 0; i < pt.nv[0]; ++i) ct.set_prob(0, pt.vp[0][i], pt.pr0[i]);
    for (int i = 0; i < pt.nv[LEN]; ++i) ct.set_prob(H, pt.vp[LEN][i], pt.prL[i]);
    for (int j = 0; j < H; ++j) {
        const int mid = 2 * j + 1;
        const int dj = dec ? (int)((*dec >> j) & 1u) : 0;
        for (int wi = 0; wi < pt.nv[mid]; ++wi) {
            // in-edges of w (layer mid-1, creation order) x out-edges of w (layer mid)
            for (int ia = pt.tstart[mid - 1][wi]; ia < pt.tstart[mid - 1][wi + 1]; ++ia) {
                const int a = pt.byto[mid - 1][ia];
                const uint32_t ka = pt.key[mid - 1][a];
                const double pa = pt.p[mid - 1][a];
                for (int ib = pt.fstart[mid][wi]; ib < pt.fstart[mid][wi + 1]; ++ib) {
                    const int b = pt.byfrom[mid][ib];
                    const uint32_t kb = pt.key[mid][b];
                    const double prob = pa * pt.p[mid][b];
                    const int ml = ek_lbl(ka) ^ ek_lbl(kb);
                    if (!dec) {
                        ct.add(j, ek_from(ka), ek_to(kb), ml, prob);
                    } else if (ml == dj) {
                        ct.add(j, ek_from(ka), ek_to(kb), ek_lbl(kb), prob);
                    }
                }
            }
        }
    }
    ct.index();
}

// The base trellis of one segment without guard-band ones, never stored (trellis_n02.h's
// Base02 for any length L): buildTrellis_uniformInput_deletion (BinaryTrellis.py:384-436)
// walks the layers in order and, inside layer l, the from-positions vp in [lo(l), hi(l)]
// ascending, creating the insertion edge vp -> vp+1 (label y[vp]) and then the deletion
// edges vp -> vp (labels 0, 1).  So a vertex's out-edges in dict order are [insertion,
// deletion 0, deletion 1], its in-edges [insertion from vp-1, deletion 0, deletion 1 from
// vp], and the vertices of a middle layer are inserted in the order the previous layer's
// edges first reach them.  Its only layer-0 / layer-L vertices are vpos 0 and m (vertex
// probability 1.0), and edges exist only when m <= L.
template <int L>
struct BaseT {
    static constexpr int V = L / 2 + 1;  // vertices per layer, at most (DelCap<L, 0>::V)
    int m;
    int d;        // deletions: L - m
    uint32_t y;   // received bits of the segment (m <= L)
    double pins;  // 0.5 (1 - pd)
    double pdel;  // 0.5 pd
    PCUB_HD int lo(int l) const { return l - d > 0 ? l - d : 0; }
    PCUB_HD int hi(int l) const { return l < m ? l : m; }
    PCUB_HD bool from_ok(int l, int vp) const { return vp >= lo(l) && vp <= hi(l); }
    // edge leaving (l, vp) of kind 0 = insertion, 1 = deletion 0, 2 = deletion 1
    PCUB_HD bool out_edge(int l, int vp, int kind, int& to, int& lbl, double& p) const {
        if (!from_ok(l, vp)) return false;
        if (kind == 0) {
            if (vp >= m) return false;
            to = vp + 1;
            lbl = (int)((y >> vp) & 1u);
            p = pins;
            return true;
        }
        if (l + 1 - d > vp) return false;
        to = vp;
        lbl = kind - 1;
        p = (kind == 1 && !(vp > 0 && vp < m)) ? 0.5 : pdel;
        return true;
    }
    // Vertices of middle layer l (1 <= l < L) that have in-edges, in insertion order.  The
    // edges of layer l-1 reach, in creation order: lo+1 (insertion from lo), lo (deletion
    // from lo), then vp+1 for every later from-position vp (its deletion target vp was
    // already reached by the insertion from vp-1), with lo = lo(l-1).
    PCUB_HD int nreached(int l) const {
        const int a = lo(l - 1);
        if (a > hi(l - 1)) return 0;  // m > L: no edges
        const int last = hi(l - 1) < m - 1 ? hi(l - 1) : m - 1;  // last from-position with an insertion
        return (a < m ? 1 : 0) + (l - d <= a ? 1 : 0) + (last > a ? last - a : 0);
    }
    PCUB_HD int reached(int l, int i) const {
        const int a = lo(l - 1);
        const int c0 = a < m ? 1 : 0;
        const int c1 = l - d <= a ? 1 : 0;
        if (i < c0) return a + 1;
        if (i < c0 + c1) return a;
        return a + 2 + (i - c0 - c1);
    }
};

template <int L, class BitF>
PCUB_HD BaseT<L> base_segment(const BitF& bit, int s, int m, double pd) {
    BaseT<L> b;
    b.m = m;
    b.d = L - m;
    b.y = 0;
    if (m <= L)
        for (int i = 0; i < m; ++i) b.y |= (uint32_t)(bit(s + i) & 1) << i;
    b.pins = 0.5 * (1.0 - pd);
    b.pdel = 0.5 * pd;
    return b;
}

// trellis_transform with the base trellis as the parent (same iteration: middle vertices
// in insertion order, in-edges x out-edges in creation order, products pa * pb).
template <int L, class C>
PCUB_HD void trellis_transform_base(const BaseT<L>& b, C& ct, const uint32_t* dec) {
    constexpr int H = L / 2;
    ct.clear();
    ct.set_prob(0, 0, 1.0);
    ct.set_prob(H, b.m, 1.0);
    for (int j = 0; j < H; ++j) {
        const int mid = 2 * j + 1;
        const int dj = dec ? (int)((*dec >> j) & 1u) : 0;
        const int nw = b.nreached(mid);
        for (int wi = 0; wi < nw; ++wi) {
            const int w = b.reached(mid, wi);
            for (int a = 0; a < 3; ++a) {
                const int u = a == 0 ? w - 1 : w;
                int tu, lu;
                double pu;
                if (!b.out_edge(mid - 1, u, a, tu, lu, pu) || tu != w) continue;
                for (int o = 0; o < 3; ++o) {
                    int tv, lv;
                    double pv;
                    if (!b.out_edge(mid, w, o, tv, lv, pv)) continue;
                    const double prob = pu * pv;
                    const int ml = lu ^ lv;
                    if (!dec) {
                        ct.add(j, u, tv, ml, prob);
                    } else if (ml == dj) {
                        ct.add(j, u, tv, lv, prob);
                    }
                }
            }
        }
    }
    ct.index();
}

// calcNormalizationVector + normalize (BinaryTrellis.py:280-306), as the decoder
// applies them to every freshly transformed child.
template <int LEN, class T>
PCUB_HD void trellis_normalize(T& t) {
    for (int i = 0; i < LEN; ++i) {
        double s0 = 0.0, s1 = 0.0;
        for (int vi = 0; vi < t.nv[i]; ++vi) {
            for (int ie = t.fstart[i][vi]; ie < t.fstart[i][vi + 1]; ++ie) {
                const int e = t.byfrom[i][ie];
                if (ek_lbl(t.key[i][e])) s1 += t.p[i][e];
                else s0 += t.p[i][e];
            }
        }
        double d = s0 >= s1 ? s0 : s1;  // np.maximum of two non-negative finite sums
        if (d == 0.0) d = 1.0;
        for (int e = 0; e < t.ne[i]; ++e) t.p[i][e] /= d;
    }
}

// calcMarginalizedProbabilities(normalize=False) of a length-1 trellis
// (BinaryTrellis.py:260-278): vertexProb * edgeProb * toVertex.vertexProb / 1.0 summed
// per label, vertices in order, out-edges in creation order.
template <class T>
PCUB_HD void trellis_marginal(const T& t, double& m0, double& m1) {
    m0 = 0.0;
    m1 = 0.0;
    for (int vi = 0; vi < t.nv[0]; ++vi) {
        const double pv = t.pr0[vi];
        for (int ie = t.fstart[0][vi]; ie < t.fstart[0][vi + 1]; ++ie) {
            const int e = t.byfrom[0][ie];
            const uint32_t k = t.key[0][e];
            const double term = pv * t.p[0][e] * t.prob_last(ek_to(k));
            if (ek_lbl(k)) m1 += term;
            else m0 += term;
        }
    }
}

// The collapse of a length-2 trellis (CollectionOfBinaryTrellises.py:68-82) with no
// guard-band ones (every vertex probability 1.0): its minus/plus child has length 1,
// and its only vertices are
// the start (vpos 0) and the end (vpos m), so the child has at most two edges,
// start -> end with label 0 and with label 1.  The child's marginal (normalize=False)
// is therefore 0.0 + the accumulated probability of each of those edges, i.e. the
// sum of the transform's contributions per label in the transform's iteration
// order -- accumulated here directly, without materialising the child.
template <class P>
PCUB_HD void trellis_collapse(const P& pt, const uint32_t* dec, double& m0, double& m1) {
    m0 = 0.0;
    m1 = 0.0;
    const int dj = dec ? (int)(*dec & 1u) : 0;
    for (int wi = 0; wi < pt.nv[1]; ++wi) {
        for (int ia = pt.tstart[0][wi]; ia < pt.tstart[0][wi + 1]; ++ia) {
            const int a = pt.byto[0][ia];
            const uint32_t ka = pt.key[0][a];
            for (int ib = pt.fstart[1][wi]; ib < pt.fstart[1][wi + 1]; ++ib) {
                const int b = pt.byfrom[1][ib];
                const uint32_t kb = pt.key[1][b];
                const double prob = pt.p[0][a] * pt.p[1][b];
                const int ml = ek_lbl(ka) ^ ek_lbl(kb);
                int x = ml;
                if (dec) {
                    if (ml != dj) continue;
                    x = ek_lbl(kb);
                }
                if (x) m1 += prob;
                else m0 += prob;
            }
        }
    }
}

// trimZerosAtEdges on word[s .. e): the first and last 1 (Guardbands.py:66-93).
template <class BitF>
PCUB_HD void trim_range(const BitF& bit, int& s, int& e) {
    int a = s;
    while (a < e && bit(a) != 1) ++a;
    if (a == e) {
        s = e = a;
        return;
    }
    int b = e - 1;
    while (bit(b) != 1) --b;
    s = a;
    e = b + 1;
}

// removeDeletionGuardBands (Guardbands.py:47-63) for one trellis: trim, halve
// (left = first len/2), descend toward trellis index t (levels = n - n0 halvings,
// most significant bit of t first), trim again at the end.
template <class BitF>
PCUB_HD void segment_of(const BitF& bit, int len, int levels, int t, int& s, int& m) {
    int a = 0, e = len;
    trim_range(bit, a, e);
    for (int k = levels - 1; k >= 0; --k) {
        const int h = (e - a) / 2;
        if ((t >> k) & 1) a += h;
        else e = a + h;
        trim_range(bit, a, e);
    }
    s = a;
    m = e - a;
}

// The same parse on a bit-packed received word (bit i of word i >> 5 = symbol i == 1,
// bits past the word's length 0): each probe covers 32 symbols, so a guard band of
// zeros is crossed in a few LDS reads instead of one dependent byte load per symbol.
// first symbol 1 in [a, e), or e (a word a step)
PCUB_HD int first_one(const uint32_t* w, int a, int e) {
    while (a < e) {
        const uint32_t x = w[a >> 5] >> (a & 31);
        if (x) {
            const int i = a + __builtin_ctz(x);
            return i < e ? i : e;
        }
        a = (a | 31) + 1;
    }
    return e;
}

// last symbol 1 in [a, e); one must exist
PCUB_HD int last_one(const uint32_t* w, int e) {
    int b = e - 1;
    for (;;) {
        const uint32_t x = w[b >> 5] << (31 - (b & 31));
        if (x) return b - __builtin_clz(x);
        b = (b & ~31) - 1;
    }
}

// The same scans for long guard bands (round 6): the first word alone, then four words a probe
// (independent loads, clamped to the range's words and masked), so a zero run of up to ~100 symbols
// past the first word costs one round trip instead of one per word.  The table-driven kernel uses them
// at 128 trellises (n = 10: 85 -> 95 M cw/s); at n = 8 (C5), where a trim nearly always finds its one
// in the first word, the larger inlined scans cost 17 %, and at n = 11 3 %, so the plain ones stay.
PCUB_HD int first_one_p4(const uint32_t* w, int a, int e) {
    if (a >= e) return e;
    int wi = a >> 5;
    const uint32_t x = w[wi] >> (a & 31);
    if (x) {
        const int i = a + __builtin_ctz(x);
        return i < e ? i : e;
    }
    const int last = (e - 1) >> 5;  // the last word the range touches
    for (++wi; wi <= last; wi += 4) {
        const int i1 = wi + 1 <= last ? wi + 1 : last, i2 = wi + 2 <= last ? wi + 2 : last,
                  i3 = wi + 3 <= last ? wi + 3 : last;
        const uint32_t x0 = w[wi];
        const uint32_t x1 = wi + 1 <= last ? w[i1] : 0u;
        const uint32_t x2 = wi + 2 <= last ? w[i2] : 0u;
        const uint32_t x3 = wi + 3 <= last ? w[i3] : 0u;
        const int i = x0   ? (wi << 5) + __builtin_ctz(x0)
                      : x1 ? ((wi + 1) << 5) + __builtin_ctz(x1)
                      : x2 ? ((wi + 2) << 5) + __builtin_ctz(x2)
                      : x3 ? ((wi + 3) << 5) + __builtin_ctz(x3)
                           : -1;
        if (i >= 0) return i < e ? i : e;
    }
    return e;
}

PCUB_HD int last_one_p4(const uint32_t* w, int e) {
    const int b = e - 1;
    int wi = b >> 5;
    const uint32_t x = w[wi] << (31 - (b & 31));
    if (x) return b - __builtin_clz(x);
    for (--wi;; wi -= 4) {
        const int i1 = wi >= 1 ? wi - 1 : 0, i2 = wi >= 2 ? wi - 2 : 0, i3 = wi >= 3 ? wi - 3 : 0;
        const uint32_t x0 = w[wi];
        const uint32_t x1 = wi >= 1 ? w[i1] : 0u;
        const uint32_t x2 = wi >= 2 ? w[i2] : 0u;
        const uint32_t x3 = wi >= 3 ? w[i3] : 0u;
        const int i = x0   ? (wi << 5) + 31 - __builtin_clz(x0)
                      : x1 ? ((wi - 1) << 5) + 31 - __builtin_clz(x1)
                      : x2 ? ((wi - 2) << 5) + 31 - __builtin_clz(x2)
                      : x3 ? ((wi - 3) << 5) + 31 - __builtin_clz(x3)
                           : -1;
        if (i >= 0) return i;
    }
}

template <bool P4 = false>
PCUB_HD void trim_range_packed(const uint32_t* w, int& s, int& e) {
    const int a = P4 ? first_one_p4(w, s, e) : first_one(w, s, e);
    if (a == e) {
        s = e = a;
        return;
    }
    e = (P4 ? last_one_p4(w, e) : last_one(w, e)) + 1;
    s = a;
}

PCUB_HD void segment_of_packed(const uint32_t* w, int len, int levels, int t, int& s, int& m) {
    int a = 0, e = len;
    trim_range_packed(w, a, e);
    for (int k = levels - 1; k >= 0; --k) {
        const int h = (e - a) / 2;
        if ((t >> k) & 1) a += h;
        else e = a + h;
        trim_range_packed(w, a, e);
    }
    s = a;
    m = e - a;
}

}  // namespace pcub
