// trellis_n02.h -- register-resident trellis stages for n0 = 2 (4-input trellises,
// the main_deletion.py configuration), host + device.
//
// Same computation as trellis_body.h (build -> minus/plus -> normalise -> collapse,
// VectorDistributions/BinaryTrellis.py:206-438, CollectionOfBinaryTrellises.py:55-82),
// with no per-lane memory:
//   * the base trellis is never stored: its vertices, its edges and their creation
//     order follow from (m, received bits, pd) -- buildTrellis_uniformInput_deletion
//     (:384-436) walks layers in order and, inside a layer, the from-positions vp in
//     ascending order, creating the insertion edge vp -> vp+1 (label y[vp]) and then the
//     deletion edges vp -> vp (labels 0, 1).  So the out-edges of a vertex in dict
//     order are [insertion, deletion 0, deletion 1], its in-edges [insertion from
//     vp-1, deletion 0, deletion 1 from vp], and a layer's vertices are inserted in the
//     order the previous layer's edges reach them;
//   * the depth-1 trellis (2 inputs) has layers {0}, W (the vertices of base layer 2
//     it reaches, at most 3) and {m}: at most 6 edges start -> w and 6 edges w -> end.
//     It is kept in fixed-size arrays appended in creation order, accessed only with
//     compile-time indices (fully unrolled, predicated), so it stays in VGPRs.
// Sums keep the reference's iteration order exactly (tests/test_emulated_deletion.py
// checks this path against the general one and the golden vectors).
#pragma once
#include "sc_common.h"

namespace pcub {

constexpr int kN02L = 4;  // inputs per base trellis
constexpr int kN02V = 3;  // vertices per layer, at most
constexpr int kN02E = 6;  // edges per depth-1 edge layer, at most

// The base trellis of one segment (length m, received bits y: bit i = symbol s+i;
// edges exist only when m <= 4).
struct Base02 {
    int m;
    int d;        // deletions: 4 - m
    uint32_t y;   // received bits (m <= 4)
    double pins;  // 0.5 (1 - pd)
    double pdel;  // 0.5 pd
    PCUB_HD int lo(int l) const { return l - d > 0 ? l - d : 0; }
    PCUB_HD int hi(int l) const { return l < m ? l : m; }
    PCUB_HD bool from_ok(int l, int vp) const { return vp >= lo(l) && vp <= hi(l); }
    // edges leaving (l, vp), creation order: kind 0 = insertion, 1 = deletion 0, 2 = deletion 1
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
    // vertex order of base layer l (1 <= l <= 3): the previous layer's edges reach them
    // in creation order, then any from-position of layer l not reached yet
    PCUB_HD int layer(int l, int* vs) const {
        int c = 0;
        auto add = [&](int v) {
            bool have = false;
#pragma unroll
            for (int i = 0; i < kN02V; ++i) have = have || (i < c && vs[i] == v);
            if (!have) {
#pragma unroll
                for (int i = 0; i < kN02V; ++i)
                    if (i == c) vs[i] = v;
                ++c;
            }
        };
#pragma unroll
        for (int s = 0; s < kN02V; ++s) {
            const int vp = lo(l - 1) + s;
            if (vp > hi(l - 1)) continue;
            if (vp < m) add(vp + 1);
            if (l - d <= vp) add(vp);
        }
#pragma unroll
        for (int s = 0; s < kN02V; ++s) {
            const int vp = lo(l) + s;
            if (vp > hi(l)) continue;
            if (vp < m || l + 1 - d <= vp) add(vp);
        }
        return c;
    }
};

// depth-1 trellis: layers {0}, W, {m}
struct Child02 {
    int nw;
    int w[kN02V];        // layer-1 vertices in insertion order
    int n0;              // edges 0 -> w (creation order): key = w*2 + label
    int k0[kN02E];
    double p0[kN02E];
    int n1;              // edges w -> m: key = w*2 + label
    int k1[kN02E];
    double p1[kN02E];

    PCUB_HD void vertex(int v) {
        bool have = false;
#pragma unroll
        for (int i = 0; i < kN02V; ++i) have = have || (i < nw && w[i] == v);
        if (!have) {
#pragma unroll
            for (int i = 0; i < kN02V; ++i)
                if (i == nw) w[i] = v;
            ++nw;
        }
    }
    // addToEdgeProb on edge layer J (BinaryTrellis.py:128-136): from-vertex, to-vertex, edge
    template <int J>
    PCUB_HD void add(int key, double p) {
        int(&k)[kN02E] = J ? k1 : k0;
        double(&pp)[kN02E] = J ? p1 : p0;
        int& n = J ? n1 : n0;
        bool found = false;
#pragma unroll
        for (int i = 0; i < kN02E; ++i)
            if (i < n && k[i] == key) {
                pp[i] += p;
                found = true;
            }
        if (!found) {
#pragma unroll
            for (int i = 0; i < kN02E; ++i)
                if (i == n) {
                    k[i] = key;
                    pp[i] = 0.0 + p;
                }
            ++n;
        }
    }
};

// minus (dec == nullptr) or plus (bits 0, 1 of *dec) transform of the base trellis
// (BinaryTrellis.py:206-258) into the depth-1 trellis.
PCUB_HD void n02_transform(const Base02& b, const uint32_t* dec, Child02& c) {
    c.nw = c.n0 = c.n1 = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int mid = 2 * j + 1;
        const int dj = dec ? (int)((*dec >> j) & 1u) : 0;
        int ws[kN02V];
        const int nws = b.layer(mid, ws);
#pragma unroll
        for (int wi = 0; wi < kN02V; ++wi) {
            if (wi >= nws) continue;
            const int w = ws[wi];
            // in-edges of w: insertion from w-1, then deletions 0, 1 from w (creation order)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const int u = a == 0 ? w - 1 : w;
                int tu, lu;
                double pu;
                if (!b.out_edge(mid - 1, u, a, tu, lu, pu) || tu != w) continue;
#pragma unroll
                for (int o = 0; o < 3; ++o) {
                    int tv, lv;
                    double pv;
                    if (!b.out_edge(mid, w, o, tv, lv, pv)) continue;
                    const double prob = pu * pv;
                    const int ml = lu ^ lv;
                    int x = ml;
                    if (dec) {
                        if (ml != dj) continue;
                        x = lv;
                    }
                    // new edge (u_layer_j, v_layer_j+1): j = 0 -> 0 -> tv; j = 1 -> u -> m
                    if (j == 0) {
                        c.vertex(tv);  // the from-vertex is the start (always present)
                        c.template add<0>(tv * 2 + x, prob);
                    } else {
                        c.vertex(u);   // the to-vertex is the end (always present)
                        c.template add<1>(u * 2 + x, prob);
                    }
                }
            }
        }
    }
}

// calcNormalizationVector + normalize of the depth-1 trellis (BinaryTrellis.py:280-306)
PCUB_HD void n02_normalize(Child02& c) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int i = 0; i < kN02E; ++i)
        if (i < c.n0) {
            if (c.k0[i] & 1) s1 += c.p0[i];
            else s0 += c.p0[i];
        }
    double t = s0 >= s1 ? s0 : s1;
    if (t == 0.0) t = 1.0;
#pragma unroll
    for (int i = 0; i < kN02E; ++i) c.p0[i] /= t;
    s0 = 0.0;
    s1 = 0.0;
#pragma unroll
    for (int wi = 0; wi < kN02V; ++wi) {
        if (wi >= c.nw) continue;
#pragma unroll
        for (int i = 0; i < kN02E; ++i)
            if (i < c.n1 && (c.k1[i] >> 1) == c.w[wi]) {
                if (c.k1[i] & 1) s1 += c.p1[i];
                else s0 += c.p1[i];
            }
    }
    t = s0 >= s1 ? s0 : s1;
    if (t == 0.0) t = 1.0;
#pragma unroll
    for (int i = 0; i < kN02E; ++i) c.p1[i] /= t;
}

// minus / plus (bit 0 of *dec) child of the depth-1 trellis collapsed to its
// un-normalised marginal (trellis_collapse in trellis_body.h)
PCUB_HD void n02_collapse(const Child02& c, const uint32_t* dec, double& m0, double& m1) {
    m0 = 0.0;
    m1 = 0.0;
    const int dj = dec ? (int)(*dec & 1u) : 0;
#pragma unroll
    for (int wi = 0; wi < kN02V; ++wi) {
        if (wi >= c.nw) continue;
        const int w = c.w[wi];
#pragma unroll
        for (int a = 0; a < kN02E; ++a) {
            if (a >= c.n0 || (c.k0[a] >> 1) != w) continue;
#pragma unroll
            for (int o = 0; o < kN02E; ++o) {
                if (o >= c.n1 || (c.k1[o] >> 1) != w) continue;
                const double prob = c.p0[a] * c.p1[o];
                const int ml = (c.k0[a] ^ c.k1[o]) & 1;
                int x = ml;
                if (dec) {
                    if (ml != dj) continue;
                    x = c.k1[o] & 1;
                }
                if (x) m1 += prob;
                else m0 += prob;
            }
        }
    }
}

// The collapse's paths through each middle vertex, gathered once per (normalised) child: a
// layer-1 vertex w has at most two edges start -> w (labels 0, 1; the start is the only
// from-vertex) and two edges w -> end, so n02_collapse's 3 x 6 x 6 predicated scan becomes
// 3 x 2 x 2.  Lists keep creation order, so the sums run in the same order.
struct Paths02 {
    int nin[kN02V], nout[kN02V];
    double ip[kN02V][2], op[kN02V][2];
    int il[kN02V][2], ol[kN02V][2];
};

PCUB_HD void n02_paths(const Child02& c, Paths02& q) {
#pragma unroll
    for (int wi = 0; wi < kN02V; ++wi) {
        q.nin[wi] = 0;
        q.nout[wi] = 0;
        q.ip[wi][0] = q.ip[wi][1] = q.op[wi][0] = q.op[wi][1] = 0.0;
        q.il[wi][0] = q.il[wi][1] = q.ol[wi][0] = q.ol[wi][1] = 0;
        if (wi >= c.nw) continue;
        const int w = c.w[wi];
#pragma unroll
        for (int a = 0; a < kN02E; ++a) {
            if (a < c.n0 && (c.k0[a] >> 1) == w) {
                if (q.nin[wi] == 0) {
                    q.ip[wi][0] = c.p0[a];
                    q.il[wi][0] = c.k0[a] & 1;
                } else {
                    q.ip[wi][1] = c.p0[a];
                    q.il[wi][1] = c.k0[a] & 1;
                }
                ++q.nin[wi];
            }
            if (a < c.n1 && (c.k1[a] >> 1) == w) {
                if (q.nout[wi] == 0) {
                    q.op[wi][0] = c.p1[a];
                    q.ol[wi][0] = c.k1[a] & 1;
                } else {
                    q.op[wi][1] = c.p1[a];
                    q.ol[wi][1] = c.k1[a] & 1;
                }
                ++q.nout[wi];
            }
        }
    }
}

// n02_collapse over the gathered paths (same terms, same order)
PCUB_HD void n02_collapse_paths(const Paths02& q, const uint32_t* dec, double& m0, double& m1) {
    m0 = 0.0;
    m1 = 0.0;
    const int dj = dec ? (int)(*dec & 1u) : 0;
#pragma unroll
    for (int wi = 0; wi < kN02V; ++wi) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            if (a >= q.nin[wi]) continue;
#pragma unroll
            for (int o = 0; o < 2; ++o) {
                if (o >= q.nout[wi]) continue;
                const double prob = q.ip[wi][a] * q.op[wi][o];
                const int ml = q.il[wi][a] ^ q.ol[wi][o];
                int x = ml;
                if (dec) {
                    if (ml != dj) continue;
                    x = q.ol[wi][o];
                }
                if (x) m1 += prob;
                else m0 += prob;
            }
        }
    }
}

// The whole n0 = 2 trellis stage of one lane is a function of its segment alone: the base
// trellis follows from (m, y, pd), and every value the lane hands to the memoryless subtree
// is a collapse of a child built from it under the decisions made so far.  So the four values
// a lane produces per codeword -- v1 = collapse(minus child), v2[xm] = collapse(minus child,
// xm), v3[ym] = collapse(plus child under ym), v4[ym][xm'] -- take one of 15 values per segment
// state, and there are 32 states: (m, y) for m <= 4 (index 2^m - 1 + y) and "no edges" (m > 4,
// index 31).  n02_table_entry computes one (state, child) row of that table with the same
// functions, in the same order, as the per-lane path (so the values are identical).
constexpr int kN02States = 32;
constexpr int kN02Row = 16;  // 15 values per state, padded

PCUB_HD int n02_state(int m, uint32_t y) { return (m >= 0 && m <= kN02L) ? (1 << m) - 1 + (int)y : kN02States - 1; }

// child cv of state st (cv 0: the minus child; cv 1..4: the plus child under ym = cv - 1) into
// row[0..14]: [0] = v1, [1 + xm] = v2, [3 + ym] = v3, [7 + 2 ym + xm'] = v4
PCUB_HD void n02_table_entry(int st, int cv, double pd, double* row) {
    Base02 b;
    if (st == kN02States - 1) {
        b.m = kN02L + 1;
        b.y = 0;
    } else {
        int m = 0;
        while ((2 << m) <= st + 1) ++m;
        b.m = m;
        b.y = (uint32_t)(st + 1 - (1 << m));
    }
    b.d = kN02L - b.m;
    b.pins = 0.5 * (1.0 - pd);
    b.pdel = 0.5 * pd;
    const uint32_t ym = (uint32_t)(cv - 1);
    Child02 c;
    n02_transform(b, cv ? &ym : nullptr, c);
    n02_normalize(c);
    Paths02 q;
    n02_paths(c, q);
    double m0, m1;
    n02_collapse_paths(q, nullptr, m0, m1);
    row[cv ? 3 + (int)ym : 0] = norm_pack(m0, m1);
#pragma unroll
    for (uint32_t xb = 0; xb < 2; ++xb) {
        n02_collapse_paths(q, &xb, m0, m1);
        row[cv ? 7 + 2 * (int)ym + (int)xb : 1 + (int)xb] = norm_pack(m0, m1);
    }
}

}  // namespace pcub
