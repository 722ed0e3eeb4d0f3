// trellis_wave.h -- the n0 = 4 deletion trellises computed by a whole wave (host + device).
//
// Restates, for 16-input trellises without guard-band ones (main_deletion.py's n0 = n // 3 at
// n = 12 .. 14, :100):
//   BinaryTrellis.__miusPlusTransform                 VectorDistributions/BinaryTrellis.py:206-258
//   BinaryTrellis.calcNormalizationVector / normalize VectorDistributions/BinaryTrellis.py:280-306
//   the collection collapse                           VectorDistributions/CollectionOfBinaryTrellises.py:68-82
// with the same values and the same order of every floating-point sum as trellis_body.h's Trel walk
// (DelBase / DelNode, sc_del_kern.h), which tests/emu/w4_check.cpp compares bit for bit.
//
// Task.  A trellis's SC walk visits 8 depth-3 nodes; node k's length-2 trellis is a function of the
// segment (m <= 16 received bits) and of the decisions returned before it (the re-encodings that
// select the plus transforms on its path).  One task = (trellis, k): build the depth-1, depth-2 and
// depth-3 trellises on node k's path from the implicit base (BaseT), then its three collapsed rows:
// the minus row, and the plus row for either decision of the minus subtree.  Nothing persists between
// tasks but the 16 decision bits, so a codeword's 2^(n-4) trellises need no per-trellis storage
// (the lane-serial Trel kernel kept 22.6 KB of private memory a trellis).
//
// Layout.  One wave a task, its trellises in the wave's LDS region (W4Buf), lanes over edge slots.
// A depth-d trellis's edge (layer j, from u, advance a, label x) sits at a fixed slot: u's offset in
// the layer's window [lo, hi] (lo = max(0, j 2^d - dd), hi = min(j 2^d, m), dd = 16 - m deletions),
// a - amin(d) with a in [amin(d), amin(d) + na(d)) (amin = max(0, 2^d - dd), na = min(2^d, dd) + 1),
// and x: pw * na(d) * 2 slots a layer, pw = min(dd, m) + 1 window positions (trellis_dense.h's
// capacity argument).  A child edge's sum is a gather: its contributions come from middle vertices w
// (u -> w -> v), and the reference adds them in its iteration order -- middle vertices in insertion
// order, then in-edges of w in creation order, then out-edges in creation order -- so a slot walks
// the middle layer's vertices by insertion rank and, per w, its (at most two) in-edges by creation
// rank.  The orders themselves are ranks:
//   * an edge is created by its first contribution, so its creation rank is the rank of the key
//     (rank of w, creation rank of the in-edge, creation rank of the out-edge) of that contribution
//     among the layer's edges;
//   * a vertex of a middle layer l is inserted by its first reference: as the to-vertex of an edge of
//     layer l - 1 (all of layer l - 1's adds come first), else as the from-vertex of one of layer l;
//     its insertion rank is the rank of (phase, least creation rank);
//   * the normaliser of a layer sums, per label, the edges in (from-vertex rank, creation rank) order.
// Sums whose order matters are taken by one lane in that order; zero terms padded after a sum's last
// term (x + 0.0 == x for the non-negative sums here) keep their trip counts regular.
#pragma once
#include "trellis_body.h"

namespace pcub {

constexpr int kW4L = 16;      // base trellis length
constexpr int kW4PW = 9;      // window positions a layer, at most (min(dd, m) + 1)
constexpr int kW4SA = 432;    // region A: depth 1 (8 x 9 x 3 x 2) or depth 3 (2 x 9 x 9 x 2)
constexpr int kW4SB = 360;    // region B: depth 2 (4 x 9 x 5 x 2)
constexpr uint32_t kW4None = 0xffffffffu;
constexpr uint8_t kW4NoC = 0xffu;
constexpr uint32_t kW4NoV = 0xffffffffu;

// n / d for n < 2^16, 0 < d < 512 by one multiply (exhaustively checked on the host): the phases
// decode their flat item indices without integer division
PCUB_HD uint32_t w4_magic(int d) { return (1u << 25) / (uint32_t)d + 1u; }
PCUB_HD int w4_div(int n, uint32_t mg) { return (int)(((uint64_t)(uint32_t)n * mg) >> 25); }

// a segment: m received symbols (m <= 16), bits y, the channel's edge probabilities
struct W4Dims {
    int m, dd, pw;
    uint32_t y;
    double pins, pdel;
    PCUB_HD void set(int m_, uint32_t y_, double pd) {
        m = m_;
        dd = kW4L - m_;
        pw = (dd < m_ ? dd : m_) + 1;
        y = y_;
        pins = 0.5 * (1.0 - pd);
        pdel = 0.5 * pd;
    }
    PCUB_HD int lo(int b) const { return b - dd > 0 ? b - dd : 0; }
    PCUB_HD int hi(int b) const { return b < m ? b : m; }
    PCUB_HD int na(int d) const { return ((1 << d) < dd ? (1 << d) : dd) + 1; }
    PCUB_HD int amin(int d) const { return (1 << d) - dd > 0 ? (1 << d) - dd : 0; }
    PCUB_HD int sl(int d) const { return pw * na(d) * 2; }
    // the base trellis (buildTrellis_uniformInput_deletion, BinaryTrellis.py:384-436; BaseT)
    PCUB_HD bool b_in(int l, int vp) const { return vp >= lo(l) && vp <= hi(l); }
    PCUB_HD bool b_ins(int l, int vp) const { return b_in(l, vp) && vp < m; }
    PCUB_HD bool b_del(int l, int vp) const { return b_in(l, vp) && vp >= lo(l + 1); }
    PCUB_HD int ybit(int vp) const { return (int)((y >> vp) & 1u); }
    PCUB_HD double p_del(int vp, int lbl) const { return (lbl == 0 && !(vp > 0 && vp < m)) ? 0.5 : pdel; }
    // creation rank of base edge (l, vp, kind): kind 0 insertion, 1 deletion of a 0, 2 of a 1; the
    // layer creates, for vp ascending, the insertion and then the two deletions
    PCUB_HD int b_crank(int l, int vp, int kind) const {
        const int a = lo(l), a1 = lo(l + 1);
        const int mi = vp < m ? vp : m;
        const int nins = mi - a > 0 ? mi - a : 0;
        const int ds = a > a1 ? a : a1;
        const int ndel = vp - ds > 0 ? 2 * (vp - ds) : 0;
        return nins + ndel + (kind == 0 ? 0 : (vp < m ? 1 : 0) + (kind - 1));
    }
    // insertion rank of vertex w of base layer l (1 <= l < 16) among those with in-edges (BaseT::reached)
    PCUB_HD int b_vrank(int l, int w) const {
        const int a = lo(l - 1);
        const int c0 = a < m ? 1 : 0;
        const int c1 = l - dd <= a ? 1 : 0;
        const int last = hi(l - 1) < m - 1 ? hi(l - 1) : m - 1;
        if (c0 && w == a + 1) return 0;
        if (c1 && w == a) return c0;
        if (w >= a + 2 && w <= last + 1) return c0 + c1 + (w - a - 2);
        return -1;
    }
};

// one wave's trellises (LDS on the device)
struct alignas(16) W4Buf {
    double pA[kW4SA];        // region A: depth 1, later depth 3 (probabilities)
    uint32_t kA[kW4SA];      // ... first-contribution keys
    double pB[kW4SB];        // region B: depth 2
    uint32_t kB[kW4SB];
    uint8_t cA[kW4SA];       // creation ranks (kW4NoC: no edge)
    uint8_t cB[kW4SB];
    uint8_t vrA[9][kW4PW];   // vertex insertion rank per window offset (kW4NoC: absent), layers 0..8
    uint8_t voA[9][kW4PW];   // window offset of the vertex of each rank
    uint8_t nvA[9];
    uint8_t vrB[5][kW4PW];
    uint8_t voB[5][kW4PW];
    uint8_t nvB[5];
    uint32_t vkey[8][kW4PW];  // vertex keys of the layer being ranked (phase << 31 | least edge key)
    uint32_t ncnt[8][2];      // edges a (layer, label) of the layer being normalised
    double sums[8][2];        // normalisation sums
    double out[3];            // the task's rows: minus, plus after 0, plus after 1
};

// a depth-d trellis in one of the regions
struct W4View {
    double* p;
    uint32_t* k;
    uint8_t* c;
    uint8_t (*vr)[kW4PW];
    uint8_t (*vo)[kW4PW];
    uint8_t* nv;
    double* tmp;  // normalisation scratch: the other region (>= this trellis's slot count doubles)
};

PCUB_HD W4View w4_view_a(W4Buf& b) { return W4View{b.pA, b.kA, b.cA, b.vrA, b.voA, b.nvA, b.pB}; }
PCUB_HD W4View w4_view_b(W4Buf& b) { return W4View{b.pB, b.kB, b.cB, b.vrB, b.voB, b.nvB, b.pA}; }

// ---- phase 1 of a transform: child edges (values and first-contribution keys) ----

// depth-1 child (layer j, window offset uo, advance offset ao) from the implicit base: the middle
// vertices are w = u (in-edges: the deletions) and w = u + 1 (the insertion), by base insertion rank
PCUB_HD void w4_base_item(const W4Dims& D, const W4View& C, int j, int uo, int ao, int dj, bool plus) {
    const int NA = D.na(1), SL = D.sl(1);
    const int s = j * SL + (uo * NA + ao) * 2;
    double acc[2] = {0.0, 0.0};
    uint32_t key[2] = {kW4None, kW4None};
    const int l0 = 2 * j, l1 = 2 * j + 1;
    const int u = D.lo(l0) + uo;
    if (u <= D.hi(l0)) {
        const int v = u + D.amin(1) + ao;
        int wv[2], rk[2], nw = 0;
        for (int a1 = 0; a1 < 2; ++a1) {
            const int w = u + a1, a2 = v - w;
            if (a2 < 0 || a2 > 1) continue;
            const int r = D.b_vrank(l1, w);
            if (r < 0) continue;
            wv[nw] = w;
            rk[nw] = r;
            ++nw;
        }
        if (nw == 2 && rk[1] < rk[0]) {
            const int t = wv[0]; wv[0] = wv[1]; wv[1] = t;
            const int q = rk[0]; rk[0] = rk[1]; rk[1] = q;
        }
        for (int i = 0; i < nw; ++i) {
            const int w = wv[i], a1 = w - u, a2 = v - w;
            // in-edges u -> w in creation order
            int na = 0, la[2], ca[2];
            double pa[2];
            if (a1 == 0) {
                if (D.b_del(l0, u)) {
                    for (int x = 0; x < 2; ++x) {
                        la[na] = x;
                        pa[na] = D.p_del(u, x);
                        ca[na] = D.b_crank(l0, u, 1 + x);
                        ++na;
                    }
                }
            } else if (D.b_ins(l0, u)) {
                la[0] = D.ybit(u);
                pa[0] = D.pins;
                ca[0] = D.b_crank(l0, u, 0);
                na = 1;
            }
            // out-edges w -> v, by label
            bool eb[2] = {false, false};
            double pb[2] = {0.0, 0.0};
            int cb[2] = {0, 0};
            if (a2 == 0) {
                if (D.b_del(l1, w))
                    for (int x = 0; x < 2; ++x) {
                        eb[x] = true;
                        pb[x] = D.p_del(w, x);
                        cb[x] = D.b_crank(l1, w, 1 + x);
                    }
            } else if (D.b_ins(l1, w)) {
                const int yb = D.ybit(w);
                eb[yb] = true;
                pb[yb] = D.pins;
                cb[yb] = D.b_crank(l1, w, 0);
            }
            for (int ia = 0; ia < na; ++ia)
                for (int x = 0; x < 2; ++x) {
                    int lb;
                    if (plus) {
                        lb = x;
                        if ((la[ia] ^ lb) != dj) continue;
                    } else {
                        lb = la[ia] ^ x;
                    }
                    if (!eb[lb]) continue;
                    acc[x] += pa[ia] * pb[lb];
                    if (key[x] == kW4None) key[x] = ((uint32_t)rk[i] << 16) | ((uint32_t)ca[ia] << 8) | (uint32_t)cb[lb];
                }
        }
    }
    for (int x = 0; x < 2; ++x) {
        C.p[s + x] = acc[x];
        C.k[s + x] = key[x];
    }
}

// depth-(d+1) child (layer j, uo, ao) of the depth-d parent P: walk P's middle layer 2j + 1 by
// insertion rank; per w, the in-edges (u, w - u) by creation rank, each with its out-edge to v
PCUB_HD void w4_item(const W4Dims& D, int d, const W4View& P, const W4View& C, int j, int uo, int ao, int dj,
                     bool plus) {
    const int NAc = D.na(d + 1), SLc = D.sl(d + 1);
    const int NAp = D.na(d), SLp = D.sl(d), AMp = D.amin(d);
    const int s = j * SLc + (uo * NAc + ao) * 2;
    double acc[2] = {0.0, 0.0};
    uint32_t key[2] = {kW4None, kW4None};
    const int u = D.lo((2 * j) << d) + uo;
    if (u <= D.hi((2 * j) << d)) {
        const int v = u + D.amin(d + 1) + ao;
        const int mv = 2 * j + 1;
        const int wlo = D.lo(mv << d);
        const int nvm = P.nv[mv];
        for (int r = 0; r < nvm; ++r) {
            const int wo = P.vo[mv][r];
            const int w = wlo + wo;
            const int a1 = w - u - AMp, a2 = v - w - AMp;
            if (a1 < 0 || a1 >= NAp || a2 < 0 || a2 >= NAp) continue;
            const int ia = (2 * j) * SLp + (uo * NAp + a1) * 2;
            const int ib = (2 * j + 1) * SLp + (wo * NAp + a2) * 2;
            // both labels of a slot pair in one read each (pairs start at even slots: 2- and 16-byte aligned)
            const uint32_t cap = *reinterpret_cast<const uint16_t*>(P.c + ia);
            const uint32_t cbp = *reinterpret_cast<const uint16_t*>(P.c + ib);
            const double2 pap = *reinterpret_cast<const double2*>(P.p + ia);
            const double2 pbp = *reinterpret_cast<const double2*>(P.p + ib);
            const int ca0 = (int)(cap & 0xffu), ca1 = (int)(cap >> 8);
            const int cb0 = (int)(cbp & 0xffu), cb1 = (int)(cbp >> 8);
            const int f = (ca1 < ca0) ? 1 : 0;  // the in-edge created first (kW4NoC sorts last)
            for (int t = 0; t < 2; ++t) {
                const int la = f ^ t;
                const int ca = la ? ca1 : ca0;
                if (ca == kW4NoC) continue;
                const double pa = la ? pap.y : pap.x;
                for (int x = 0; x < 2; ++x) {
                    int lb;
                    if (plus) {
                        lb = x;
                        if ((la ^ lb) != dj) continue;
                    } else {
                        lb = la ^ x;
                    }
                    const int cb = lb ? cb1 : cb0;
                    if (cb == kW4NoC) continue;
                    acc[x] += pa * (lb ? pbp.y : pbp.x);
                    if (key[x] == kW4None) key[x] = ((uint32_t)r << 16) | ((uint32_t)ca << 8) | (uint32_t)cb;
                }
            }
        }
    }
    for (int x = 0; x < 2; ++x) {
        C.p[s + x] = acc[x];
        C.k[s + x] = key[x];
    }
}

// ---- the phases (lane-strided loops; a wave barrier between consecutive phases) ----
//
// Enumeration.  Of a depth-d layer j's pw x na(d) (from, advance) slot pairs only those with the
// from-position in the layer's window [lo(j 2^d), hi(j 2^d)] (nu of them) and the to-position in the
// next layer's window can hold an edge: w4_arange gives each from-position's advance offsets, at most
// K = min(na, nu(next)) of them.  Every phase walks only these pairs (the other slots are never
// written, so never read): the end layers, whose windows are single positions, hold ~1/9 of their
// dense slots at n0 = 4.

// advance offsets [a0, a1] of window offset uo in depth-d layer j
PCUB_HD void w4_arange(const W4Dims& D, int d, int j, int uo, int& a0, int& a1) {
    const int u = D.lo(j << d) + uo, AM = D.amin(d), NA = D.na(d);
    const int b1 = (j + 1) << d;
    a0 = D.lo(b1) - u - AM;
    a0 = a0 > 0 ? a0 : 0;
    a1 = D.hi(b1) - u - AM;
    a1 = a1 < NA - 1 ? a1 : NA - 1;
}

PCUB_HD int w4_nu(const W4Dims& D, int b) { return D.hi(b) - D.lo(b) + 1; }

// Lanes.  A depth-d trellis has LEN = 16 >> d layers; each layer gets LPL = 64 / LEN lanes (8, 16,
// 32), lane = j * LPL + q, and its q-th, (q + LPL)-th, .. item: no lane decodes a flat index.
PCUB_HD int w4_lpl_log(int d) { return 2 + d; }

// layer j's enumerated pairs: item r -> (uo, ao); false past the from-position's advance range
struct W4Layer {
    int j, nu, K;
    uint32_t mk;
    PCUB_HD void set(const W4Dims& D, int d, int j_) {
        j = j_;
        nu = w4_nu(D, j << d);
        const int nn = w4_nu(D, (j + 1) << d), NA = D.na(d);
        K = NA < nn ? NA : nn;
        mk = w4_magic(K);
    }
    PCUB_HD bool item(const W4Dims& D, int d, int r, int& uo, int& ao) const {
        uo = w4_div(r, mk);
        int a0, a1;
        w4_arange(D, d, j, uo, a0, a1);
        ao = a0 + (r - uo * K);
        return ao <= a1;
    }
};

// child edges of the transform into depth d + 1 (d = 0: from the base)
PCUB_HD void w4_ph_edges(const W4Dims& D, int d, const W4View& P, const W4View& C, uint32_t dec, bool plus,
                         int lane) {
    const int dc = d + 1, lg = w4_lpl_log(dc);
    W4Layer Ly;
    Ly.set(D, dc, lane >> lg);
    const int dj = (int)((dec >> Ly.j) & 1u);
    for (int r = lane & ((1 << lg) - 1); r < Ly.nu * Ly.K; r += 1 << lg) {
        int uo, ao;
        if (!Ly.item(D, dc, r, uo, ao)) continue;
        if (d == 0) w4_base_item(D, C, Ly.j, uo, ao, dj, plus);
        else w4_item(D, d, P, C, Ly.j, uo, ao, dj, plus);
    }
}

// creation ranks of the child's edges (both labels of a pair against the layer's enumerated keys);
// zero the normalisation counters
PCUB_HD void w4_ph_rank(const W4Dims& D, int dc, const W4View& C, W4Buf& b, int lane) {
    const int SL = D.sl(dc), NA = D.na(dc), lg = w4_lpl_log(dc);
    W4Layer Ly;
    Ly.set(D, dc, lane >> lg);
    const int j = Ly.j;
    for (int r = lane & ((1 << lg) - 1); r < Ly.nu * Ly.K; r += 1 << lg) {
        int uo, ao;
        if (!Ly.item(D, dc, r, uo, ao)) continue;
        const int s = j * SL + (uo * NA + ao) * 2;
        const uint32_t k0 = C.k[s], k1 = C.k[s + 1];
        int n0 = 0, n1 = 0;
        for (int uo2 = 0; uo2 < Ly.nu; ++uo2) {
            int a0, a1;
            w4_arange(D, dc, j, uo2, a0, a1);
            const uint2* kl = reinterpret_cast<const uint2*>(C.k + j * SL + uo2 * NA * 2);
            for (int ao2 = a0; ao2 <= a1; ++ao2) {
                const uint2 q = kl[ao2];
                n0 += (q.x < k0 ? 1 : 0) + (q.y < k0 ? 1 : 0);
                n1 += (q.x < k1 ? 1 : 0) + (q.y < k1 ? 1 : 0);
            }
        }
        C.c[s] = k0 == kW4None ? kW4NoC : (uint8_t)n0;
        C.c[s + 1] = k1 == kW4None ? kW4NoC : (uint8_t)n1;
    }
    if (lane < 16) b.ncnt[lane >> 1][lane & 1] = 0u;
}

// vertex keys of the child's layers 1 .. LEN-1 (D3: layer 1 only), from the edge keys: a layer's
// creation order is the order of its keys, so the least creation rank of a vertex's in- (out-) edges
// is that of their least key.  Runs in the rank phase (it reads only keys).
PCUB_HD void w4_ph_vkey(const W4Dims& D, int dc, const W4View& C, W4Buf& b, int lane) {
    const int LEN = kW4L >> dc, SL = D.sl(dc), NA = D.na(dc), AM = D.amin(dc), lg = w4_lpl_log(dc);
    const int l = lane >> lg;
    if (l == 0 || l >= LEN) return;
    for (int po = lane & ((1 << lg) - 1); po < D.pw; po += 1 << lg) {
        const int p = D.lo(l << dc) + po;
        uint32_t vk = kW4NoV;
        if (p <= D.hi(l << dc)) {
            uint32_t k0 = kW4None;
            const int plo = D.lo((l - 1) << dc), pnu = w4_nu(D, (l - 1) << dc);
            for (int ao = 0; ao < NA; ++ao) {
                const int uo = p - AM - ao - plo;
                if (uo < 0 || uo >= pnu) continue;
                const uint2 q = *reinterpret_cast<const uint2*>(C.k + (l - 1) * SL + (uo * NA + ao) * 2);
                k0 = q.x < k0 ? q.x : k0;
                k0 = q.y < k0 ? q.y : k0;
            }
            if (k0 != kW4None) {
                vk = k0;
            } else {
                uint32_t k1 = kW4None;
                int a0, a1;
                w4_arange(D, dc, l, po, a0, a1);
                for (int ao = a0; ao <= a1; ++ao) {
                    const uint2 q = *reinterpret_cast<const uint2*>(C.k + l * SL + (po * NA + ao) * 2);
                    k1 = q.x < k1 ? q.x : k1;
                    k1 = q.y < k1 ? q.y : k1;
                }
                if (k1 != kW4None) vk = 0x80000000u | k1;
            }
        }
        b.vkey[l - 1][po] = vk;
    }
}

// vertex insertion ranks from the keys (layer 0: the start vertex alone)
PCUB_HD void w4_ph_vrank(const W4Dims& D, int dc, const W4View& C, const W4Buf& b, int lane) {
    const int LEN = kW4L >> dc, lg = w4_lpl_log(dc);
    const int l = lane >> lg;
    if (l >= 1 && l < LEN)
        for (int po = lane & ((1 << lg) - 1); po < D.pw; po += 1 << lg) {
            const uint32_t vk = b.vkey[l - 1][po];
            int r = 0, nv = 0;
            for (int t = 0; t < D.pw; ++t) {
                const uint32_t o = b.vkey[l - 1][t];
                r += o < vk ? 1 : 0;
                nv += o != kW4NoV ? 1 : 0;
            }
            if (vk != kW4NoV) {
                C.vr[l][po] = (uint8_t)r;
                C.vo[l][r] = (uint8_t)po;
            } else {
                C.vr[l][po] = kW4NoC;
            }
            if (po == 0) C.nv[l] = (uint8_t)nv;
        }
    if (lane < kW4PW) C.vr[0][lane] = lane == 0 ? 0 : kW4NoC;
    if (lane == 0) {
        C.vo[0][0] = 0;
        C.nv[0] = 1;
    }
}

// normalisation order: each edge's position among its layer's same-label edges by (from-vertex rank,
// creation rank), its probability scattered there.  Items (from-vertex, label) of the lane's layer: the
// edges of the vertices ranked before it, then its own by creation rank.
PCUB_HD void w4_ph_norder(const W4Dims& D, int dc, const W4View& C, W4Buf& b, int lane) {
    const int SL = D.sl(dc), NA = D.na(dc), lg = w4_lpl_log(dc);
    const int half = SL / 2;
    const int j = lane >> lg;
    const int nu = w4_nu(D, j << dc);
    for (int r = lane & ((1 << lg) - 1); r < 2 * nu; r += 1 << lg) {
        const int uo = r >> 1, x = r & 1;
        const int vr = C.vr[j][uo];
        if (vr == kW4NoC) continue;
        const uint8_t* cl = C.c + j * SL + x;  // label-x slot (uo2, ao2) at cl[2 (uo2 NA + ao2)]
        int base = 0;
        for (int uo2 = 0; uo2 < nu; ++uo2) {
            if (C.vr[j][uo2] >= vr) continue;  // absent vertices (kW4NoC) rank after every present one
            int a0, a1;
            w4_arange(D, dc, j, uo2, a0, a1);
            for (int ao2 = a0; ao2 <= a1; ++ao2) base += cl[2 * (uo2 * NA + ao2)] != kW4NoC ? 1 : 0;
        }
        int a0, a1;
        w4_arange(D, dc, j, uo, a0, a1);
        const uint8_t* own = cl + 2 * uo * NA;
        int cnt = 0;
        for (int ao = a0; ao <= a1; ++ao) {
            const int c = own[2 * ao];
            if (c == kW4NoC) continue;
            ++cnt;
            int n = base;
            for (int ao2 = a0; ao2 <= a1; ++ao2) n += own[2 * ao2] < c ? 1 : 0;
            C.tmp[j * SL + x * half + n] = C.p[j * SL + 2 * (uo * NA + ao) + x];
        }
        if (cnt) {
#if defined(__HIP_DEVICE_COMPILE__)
            atomicAdd(&b.ncnt[j][x], (uint32_t)cnt);
#else
            b.ncnt[j][x] += (uint32_t)cnt;
#endif
        }
    }
}

// the per-(layer, label) sums, each by one lane in order, four terms a step (terms past the count
// read as 0.0, which changes no sum here: every sum is of non-negative terms from +0.0)
PCUB_HD void w4_ph_nsum(const W4Dims& D, int dc, const W4View& C, W4Buf& b, int lane) {
    const int LEN = kW4L >> dc, SL = D.sl(dc);
    if (lane < 2 * LEN) {
        const int j = lane >> 1, x = lane & 1;
        const double* t = C.tmp + j * SL + x * (SL / 2);
        const int n = (int)b.ncnt[j][x];
        double s = 0.0;
        for (int i = 0; i < n; i += 4) {
            const double t0 = t[i], t1 = i + 1 < n ? t[i + 1] : 0.0, t2 = i + 2 < n ? t[i + 2] : 0.0,
                         t3 = i + 3 < n ? t[i + 3] : 0.0;
            s += t0;
            s += t1;
            s += t2;
            s += t3;
        }
        b.sums[j][x] = s;
    }
}

// normalize: every edge of layer j divided by max(s0, s1) (1 when both are 0)
PCUB_HD void w4_ph_ndiv(const W4Dims& D, int dc, const W4View& C, const W4Buf& b, int lane) {
    const int SL = D.sl(dc), NA = D.na(dc), lg = w4_lpl_log(dc);
    W4Layer Ly;
    Ly.set(D, dc, lane >> lg);
    const double s0 = b.sums[Ly.j][0], s1 = b.sums[Ly.j][1];
    double dv = s0 >= s1 ? s0 : s1;
    if (dv == 0.0) dv = 1.0;
    for (int r = lane & ((1 << lg) - 1); r < Ly.nu * Ly.K; r += 1 << lg) {
        int uo, ao;
        if (!Ly.item(D, dc, r, uo, ao)) continue;
        const int s = Ly.j * SL + (uo * NA + ao) * 2;
        for (int x = 0; x < 2; ++x)
            if (C.c[s + x] != kW4NoC) C.p[s + x] = C.p[s + x] / dv;
    }
}

// ---- depth 3 (the length-2 trellis) and its collapse, without the generic phases ----
//
// Its layer 0 leaves the start vertex only and its layer 1 enters the end vertex m only, so every edge
// is (0 -> w, x) or (w -> m, x) for the <= 9 middle vertices w: the creation order that matters is the
// label order of each (0, w) and (w, m) pair and the key order of layer 0's edges, the middle vertices'
// insertion order is the rank of their (phase, least key), and each normaliser is a short ordered sum.
// Same values and orders as the generic phases (w4_check compares them with the Trel walk).

// F1: middle-vertex keys (lanes 0..8); layer 0's edges scattered by key order per label (lanes 16..)
PCUB_HD void w4_ph_f1(const W4Dims& D, const W4View& C, W4Buf& b, int lane) {
    const int NA = D.na(3), AM = D.amin(3);
    const int wlo = D.lo(8), nw = w4_nu(D, 8);
    if (lane < nw) {
        const int w = wlo + lane;
        uint32_t vk = kW4NoV;
        const int a1 = w - AM;
        if (a1 >= 0 && a1 < NA) {
            const uint2 q = *reinterpret_cast<const uint2*>(C.k + 2 * a1);
            const uint32_t k0 = q.x < q.y ? q.x : q.y;
            if (k0 != kW4None) vk = k0;
        }
        if (vk == kW4NoV) {
            const int a2 = D.m - w - AM;
            if (a2 >= 0 && a2 < NA) {
                const uint2 q = *reinterpret_cast<const uint2*>(C.k + D.sl(3) + (lane * NA + a2) * 2);
                const uint32_t k1 = q.x < q.y ? q.x : q.y;
                if (k1 != kW4None) vk = 0x80000000u | k1;
            }
        }
        b.vkey[0][lane] = vk;
    }
    int e0, e1;  // layer 0's enumerated advance offsets (the slots outside are never written)
    w4_arange(D, 3, 0, 0, e0, e1);
    if (lane >= 16 && lane < 16 + 2 * NA) {
        const int i = lane - 16, ao = i >> 1, x = i & 1;
        if (ao >= e0 && ao <= e1) {
            const uint32_t k = C.k[2 * ao + x];
            if (k != kW4None) {
                int n = 0;
                for (int a2 = e0; a2 <= e1; ++a2) n += C.k[2 * a2 + x] < k ? 1 : 0;
                C.tmp[x * 16 + n] = C.p[2 * ao + x];
            }
        }
    }
    if (lane >= 48 && lane < 50) {  // layer 0's edge count per label
        const int x = lane - 48;
        int n = 0;
        for (int a2 = e0; a2 <= e1; ++a2) n += C.k[2 * a2 + x] != kW4None ? 1 : 0;
        b.ncnt[0][x] = (uint32_t)n;
    }
}

// F2: middle-vertex insertion order (lanes 0..8); layer 0's normaliser sums (lanes 16, 17)
PCUB_HD void w4_ph_f2(const W4Dims& D, const W4View& C, W4Buf& b, int lane) {
    const int nw = w4_nu(D, 8);
    if (lane < nw) {
        const uint32_t vk = b.vkey[0][lane];
        int r = 0, nv = 0;
        for (int t = 0; t < nw; ++t) {
            const uint32_t o = b.vkey[0][t];
            r += o < vk ? 1 : 0;
            nv += o != kW4NoV ? 1 : 0;
        }
        if (vk != kW4NoV) C.vo[1][r] = (uint8_t)lane;
        if (lane == 0) C.nv[1] = (uint8_t)nv;
    }
    if (lane == 16 || lane == 17) {
        const int x = lane - 16;
        const int n = (int)b.ncnt[0][x];
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += C.tmp[x * 16 + i];
        b.sums[0][x] = s;
    }
}

// F3: layer 1's normaliser (vertices in insertion order, one edge a label each) and the three
// collapsed rows from the normalised edges (lanes 0, 1, 2: minus, plus after 0, plus after 1)
PCUB_HD void w4_ph_f3(const W4Dims& D, const W4View& C, W4Buf& b, int lane) {
    if (lane >= 3) return;
    const int NA = D.na(3), AM = D.amin(3);
    const int wlo = D.lo(8);
    const int nv1 = C.nv[1];
    const int L1 = D.sl(3);  // layer 1's first slot
    double t0 = 0.0, t1 = 0.0;
    for (int r = 0; r < nv1; ++r) {
        const int wo = C.vo[1][r];
        const int a2 = D.m - (wlo + wo) - AM;
        if (a2 < 0 || a2 >= NA) continue;
        const int ib = L1 + (wo * NA + a2) * 2;
        if (C.k[ib] != kW4None) t0 += C.p[ib];
        if (C.k[ib + 1] != kW4None) t1 += C.p[ib + 1];
    }
    double d0 = b.sums[0][0] >= b.sums[0][1] ? b.sums[0][0] : b.sums[0][1];
    if (d0 == 0.0) d0 = 1.0;
    double d1 = t0 >= t1 ? t0 : t1;
    if (d1 == 0.0) d1 = 1.0;
    double m0 = 0.0, m1 = 0.0;
    for (int r = 0; r < nv1; ++r) {
        const int wo = C.vo[1][r];
        const int w = wlo + wo;
        const int a1 = w - AM, a2 = D.m - w - AM;
        if (a1 < 0 || a1 >= NA || a2 < 0 || a2 >= NA) continue;
        const int ia = 2 * a1, ib = L1 + (wo * NA + a2) * 2;
        const uint32_t ka0 = C.k[ia], ka1 = C.k[ia + 1], kb0 = C.k[ib], kb1 = C.k[ib + 1];
        const int fa = ka1 < ka0 ? 1 : 0, fb = kb1 < kb0 ? 1 : 0;
        for (int t = 0; t < 2; ++t) {
            const int la = fa ^ t;
            if ((la ? ka1 : ka0) == kW4None) continue;
            const double pa = C.p[ia + la] / d0;
            for (int q = 0; q < 2; ++q) {
                const int lb = fb ^ q;
                if ((lb ? kb1 : kb0) == kW4None) continue;
                const double prob = pa * (C.p[ib + lb] / d1);
                const int ml = la ^ lb;
                int x = ml;
                if (lane > 0) {
                    if (ml != lane - 1) continue;
                    x = lb;
                }
                if (x) m1 += prob;
                else m0 += prob;
            }
        }
    }
    b.out[lane] = norm_pack(m0, m1);
}

// ---- the per-trellis cache of the depth-1 and depth-2 trellises ----
//
// Node k's depth-1 trellis depends only on k >> 2 (minus for k < 4, the plus child under the first
// four nodes' decisions after), its depth-2 trellis only on k >> 1: the kernel keeps the last of each
// per trellis in global memory (kW4Cache bytes a trellis) and reloads instead of rebuilding -- what the
// next transform reads: probabilities, creation ranks, middle-layer vertex orders.
constexpr int kW4C1 = 4096;  // depth 1: p[432] doubles, c[432], vo[9][9], nv[9]
constexpr int kW4C2 = 3328;  // depth 2: p[360] doubles, c[360], vo[5][9], nv[5]
constexpr int kW4Cache = kW4C1 + kW4C2;
enum { kW4Load1 = 1, kW4Save1 = 2, kW4Load2 = 4, kW4Save2 = 8 };

PCUB_HD void w4_cache_io(const W4Dims& D, int d, const W4View& V, uint8_t* g, bool save, int lane) {
    const int LEN = kW4L >> d, n = LEN * D.sl(d);
    const int cap = d == 1 ? kW4SA : kW4SB;
    double* gp = reinterpret_cast<double*>(g);
    uint8_t* gc = g + cap * 8;
    uint8_t* gv = gc + cap;
    uint8_t* vo = &V.vo[0][0];
    const int nvo = (LEN + 1) * kW4PW;
    if (save) {
        for (int i = lane; i < n; i += 64) {
            gp[i] = V.p[i];
            gc[i] = V.c[i];
        }
        for (int i = lane; i < nvo; i += 64) gv[i] = vo[i];
        if (lane <= LEN) gv[nvo + lane] = V.nv[lane];
    } else {
        for (int i = lane; i < n; i += 64) {
            V.p[i] = gp[i];
            V.c[i] = gc[i];
        }
        for (int i = lane; i < nvo; i += 64) vo[i] = gv[i];
        if (lane <= LEN) V.nv[lane] = gv[nvo + lane];
    }
}

// The re-encoding of a node's returned bits: x[2h] = ym[h] ^ yp[h], x[2h+1] = yp[h] (DelNode)
PCUB_HD uint32_t w4_combine(uint32_t ym, uint32_t yp, int H) {
    uint32_t x = 0;
    for (int h = 0; h < H; ++h) x |= ((((ym ^ yp) >> h) & 1u) << (2 * h)) | (((yp >> h) & 1u) << (2 * h + 1));
    return x;
}
// node i's two bits (depth 3) -> its 2-bit encoding
PCUB_HD uint32_t w4_enc2(uint32_t hist, int i) {
    const uint32_t xm = (hist >> (2 * i)) & 1u, xp = (hist >> (2 * i + 1)) & 1u;
    return (xm ^ xp) | (xp << 1);
}
PCUB_HD uint32_t w4_enc4(uint32_t hist, int i) { return w4_combine(w4_enc2(hist, 2 * i), w4_enc2(hist, 2 * i + 1), 2); }
PCUB_HD uint32_t w4_enc8(uint32_t hist, int i) { return w4_combine(w4_enc4(hist, 2 * i), w4_enc4(hist, 2 * i + 1), 4); }
PCUB_HD uint32_t w4_enc16(uint32_t hist) { return w4_combine(w4_enc8(hist, 0), w4_enc8(hist, 1), 8); }

// One task: depth-3 node k of a segment with decision history hist (bit 2i / 2i+1: the minus / plus
// subtree of node i < k).  `run(f)` runs f(lane) on every lane of the wave, then a wave barrier.
// With a cache (kW4Cache bytes, this trellis's), `mode` loads the depth-1 / depth-2 trellis from it
// instead of building it (kW4Load1 / kW4Load2: the caller knows it holds node k's) or saves the built
// one (kW4Save1 / kW4Save2).  Leaves b.out[0..2] = the minus row, the plus row after decision 0, after 1.
template <class Run>
PCUB_HD void w4_task(const Run& run, W4Buf& b, const W4Dims& D, int k, uint32_t hist, uint8_t* cache = nullptr,
                     int mode = 0) {
    if (D.m > kW4L) {  // no edges (BaseT with m > L): every row is the collapse of an empty trellis
        run([&](int lane) {
            if (lane < 3) b.out[lane] = norm_pack(0.0, 0.0);
        });
        return;
    }
    if (!cache) mode = 0;
    const W4View A = w4_view_a(b), B = w4_view_b(b);
    const bool p1 = (k >> 2) & 1, p2 = (k >> 1) & 1, p3 = k & 1;
    const uint32_t d1 = p1 ? w4_enc8(hist, 0) : 0u;
    const uint32_t d2 = p2 ? w4_enc4(hist, (k >> 1) - 1) : 0u;
    const uint32_t d3 = p3 ? w4_enc2(hist, k - 1) : 0u;
    if (!(mode & kW4Load2)) {
        // depth 1 (region A) from the base, or from the cache
        if (mode & kW4Load1) {
            run([&](int lane) { w4_cache_io(D, 1, A, cache, false, lane); });
        } else {
            run([&](int lane) { w4_ph_edges(D, 0, A, A, d1, p1, lane); });
            run([&](int lane) {
                w4_ph_rank(D, 1, A, b, lane);
                w4_ph_vkey(D, 1, A, b, lane);
            });
            run([&](int lane) { w4_ph_vrank(D, 1, A, b, lane); });
            run([&](int lane) { w4_ph_norder(D, 1, A, b, lane); });
            run([&](int lane) { w4_ph_nsum(D, 1, A, b, lane); });
            run([&](int lane) { w4_ph_ndiv(D, 1, A, b, lane); });
        }
        // depth 2 (region B)
        run([&](int lane) {
            if (mode & kW4Save1) w4_cache_io(D, 1, A, cache, true, lane);
            w4_ph_edges(D, 1, A, B, d2, p2, lane);
        });
        run([&](int lane) {
            w4_ph_rank(D, 2, B, b, lane);
            w4_ph_vkey(D, 2, B, b, lane);
        });
        run([&](int lane) { w4_ph_vrank(D, 2, B, b, lane); });
        run([&](int lane) { w4_ph_norder(D, 2, B, b, lane); });
        run([&](int lane) { w4_ph_nsum(D, 2, B, b, lane); });
        run([&](int lane) { w4_ph_ndiv(D, 2, B, b, lane); });
    } else {
        run([&](int lane) { w4_cache_io(D, 2, B, cache + kW4C1, false, lane); });
    }
    // depth 3 (region A again) and the rows
    run([&](int lane) {
        if (mode & kW4Save2) w4_cache_io(D, 2, B, cache + kW4C1, true, lane);
        w4_ph_edges(D, 2, B, A, d3, p3, lane);
    });
    run([&](int lane) { w4_ph_f1(D, A, b, lane); });
    run([&](int lane) { w4_ph_f2(D, A, b, lane); });
    run([&](int lane) { w4_ph_f3(D, A, b, lane); });
}

}  // namespace pcub
