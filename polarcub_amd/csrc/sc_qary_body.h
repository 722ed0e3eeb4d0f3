// sc_qary_body.h -- one-codeword q-ary SC decode schedule (host + device).
//
// Replaces QaryPolarEncoderDecoder.recursiveEncodeDecode (decode branch,
// QaryPolarEncoderDecoder.py:318-401) over QaryMemorylessVectorDistribution
// (VectorDistributions/QaryMemorylessVectorDistribution.py:26-118), linear domain.
// Arithmetic contract:
//   minus  new[u] = 0.0, then new[(x1+x2)%q] += a[x1]*b[x2] with x1 outer, x2 inner (:36-42)
//   plus   new[u2] = 0.0 + a[(u1+u2)%q] * b[(q-u2)%q]                           (:55-62)
//   normalise t = ((0 + p0) + p1) + ... ; if t != 0: p[x] /= t                      (:92-118)
//   leaf   s = sum as above; m = p/s (or 1/q); u = first argmax(m)                  (:69-90, :342)
//   frozen symbols are 0 (:347-351); the a-priori tree is never consulted.
//   combine x[2h] = (xm+xp)%q, x[2h+1] = (q-xp)%q                                    (:397-399)
//
// Schedule (as the binary kernel, sc_bin_body.h, with one codeword per lane):
// half-split order inside every node; the bottom S positions of every chain live
// in registers (QSub<S>); stage levels 1..D-1 in a per-slot scratch (q doubles
// per position as ceil(q/2) 16-byte pairs, slot-minor, so a wave's access is one
// contiguous 1 KiB); the re-encoded symbols one byte each, four to a 32-bit word
// (combined word-wise, see q_combine_words).  A chain -- one plus transform, then minus transforms
// down to depth D -- is evaluated in passes of up to two fused levels per column,
// so a level written inside a pass is consumed from registers by the next one.
// Nodes whose u range is entirely frozen are never evaluated (their symbols are 0
// and so is their re-encoding), driven by the per-code rate-0 depth table `ef`.
//
// G lanes per codeword (G = 1, 2, 4), as in the binary kernel: lane j owns the
// positions p = j (mod G) of every node of length >= G, so every butterfly of a
// node of length >= 2G is lane-local and each lane runs the G = 1 schedule on a
// virtual tree of N/G positions; a virtual leaf is a real node of G positions,
// one per lane, finished by QXSub<G> with cross-lane exchanges.  More lanes per
// codeword = fewer stage levels in memory (the kernel is bound by their traffic).
#pragma once
#include "sc_bin_body.h"  // first_frozen_depth, launder
#include "sc_common.h"

namespace pcub {

template <int Q>
struct QV {
    double p[Q];
};

template <int Q>
PCUB_HD QV<Q> q_normalize(QV<Q> v) {
    double t = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) t = t + v.p[x];
    if (t != 0.0) {
#pragma unroll
        for (int x = 0; x < Q; ++x) v.p[x] = v.p[x] / t;
    }
    return v;
}

template <int Q>
PCUB_HD QV<Q> q_minus(const QV<Q>& a, const QV<Q>& b) {
    QV<Q> o;
#pragma unroll
    for (int u = 0; u < Q; ++u) o.p[u] = 0.0;
#pragma unroll
    for (int x1 = 0; x1 < Q; ++x1)
#pragma unroll
        for (int x2 = 0; x2 < Q; ++x2) {
            const int u1 = (x1 + x2) % Q;
            o.p[u1] = o.p[u1] + a.p[x1] * b.p[x2];
        }
    return q_normalize<Q>(o);
}

template <int Q>
PCUB_HD QV<Q> q_plus(const QV<Q>& a, const QV<Q>& b, int u1) {
    QV<Q> o;
#pragma unroll
    for (int u2 = 0; u2 < Q; ++u2) {
        // a[(u1+u2)%Q] with a lane-divergent u1: select instead of indexing
        const int x1 = (u1 + u2) % Q;
        double ax = a.p[0];
#pragma unroll
        for (int x = 1; x < Q; ++x) ax = (x1 == x) ? a.p[x] : ax;
        o.p[u2] = 0.0 + ax * b.p[(Q - u2) % Q];
    }
    return q_normalize<Q>(o);
}

template <int Q>
PCUB_HD int q_leaf(const QV<Q>& v) {
    double s = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) s = s + v.p[x];
    int arg = 0;
    double best = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) {
        const double m = (s > 0.0) ? v.p[x] / s : 1.0 / (double)Q;
        if (x == 0 || m > best) {
            best = m;
            arg = x;
        }
    }
    return arg;
}

struct QArgs {
    const double* xy;       // [N][B][Q]
    long long B;
    int n;
    const uint8_t* frozen;  // [N] 0/1
    const uint8_t* ef;      // [2^D] first rate-0 depth on each register subtree's chain
    uint8_t* info;          // [K][B]
    uint8_t* xhat;          // [N][B] or null
    double2* scratch;       // [(N - 2S) positions][ceil(Q/2)][nslots]
    uint32_t* ysym;         // [N/4 words][nslots], symbol of position p in byte p % 4 of word p / 4
    long long nslots;
};

// Re-encoded symbols, four per word.  SWAR on bytes: every byte holds a value
// < 2Q <= 16, so byte sums never carry, and (b | 0x80) - Q >= 0x78 never
// borrows; its bit 7 is set iff b >= Q.
template <int Q>
PCUB_HD uint32_t q_mod_bytes(uint32_t s) {
    const uint32_t ge = (((s | 0x80808080u) - (uint32_t)Q * 0x01010101u) & 0x80808080u) >> 7;
    return s - ge * (uint32_t)Q;
}

// parent = [(ym + yp) % Q | (Q - yp) % Q]  (QaryPolarEncoderDecoder.py:397-399, half-split order)
template <int Q>
PCUB_HD void q_combine_words(uint32_t& m, uint32_t& p) {
    const uint32_t mm = q_mod_bytes<Q>(m + p);
    p = q_mod_bytes<Q>((uint32_t)Q * 0x01010101u - p);
    m = mm;
}

PCUB_HD int q_sym(const uint32_t* Y, long long ns, int pos) {
    return (int)((Y[(long long)(pos >> 2) * ns] >> ((pos & 3) * 8)) & 0xffu);
}

// Decisions of the register subtree: information symbols go out in u order
// (identical in the G lanes of a codeword; lane w % G stores row w).
struct QInfo {
    const QArgs* A;
    long long cw;
    bool store;
    int w;     // next information row
    int j;     // lane of the codeword
    int gm;    // G - 1
    PCUB_HD void put(int u) {
        if (store && (w & gm) == j) A->info[(long long)w * A->B + cw] = (uint8_t)u;
        ++w;
    }
};

// Exchange of a whole q-vector with lane ^ MASK.
template <int Q, int MASK>
PCUB_HD QV<Q> q_shfl(const QV<Q>& v) {
    QV<Q> w;
#pragma unroll
    for (int x = 0; x < Q; ++x) w.p[x] = xor_shfl_c<MASK>(v.p[x]);
    return w;
}

// A real node of M <= G positions, position (lane & (M-1)) in each lane; leaf u
// indices UB .. UB+M-1.  Returns this lane's symbol of the node's re-encoding.
template <int Q, int M>
struct QXSub {
    static PCUB_HD int run(const QV<Q>& v, int ub, QInfo& qi, int lane) {
        const QV<Q> w = q_shfl<Q, M / 2>(v);
        const bool lo = (lane & (M / 2)) == 0;
        QV<Q> a, b;
#pragma unroll
        for (int x = 0; x < Q; ++x) {
            a.p[x] = lo ? v.p[x] : w.p[x];
            b.p[x] = lo ? w.p[x] : v.p[x];
        }
        int ym, yp;
        if constexpr (M == 2) {
            ym = 0;
            if (!qi.A->frozen[ub]) {
                ym = q_leaf<Q>(q_minus<Q>(a, b));
                qi.put(ym);
            }
            yp = 0;
            if (!qi.A->frozen[ub + 1]) {
                yp = q_leaf<Q>(q_plus<Q>(a, b, ym));
                qi.put(yp);
            }
        } else {
            ym = QXSub<Q, M / 2>::run(q_minus<Q>(a, b), ub, qi, lane);
            yp = QXSub<Q, M / 2>::run(q_plus<Q>(a, b, ym), ub + M / 2, qi, lane);
        }
        return lo ? (ym + yp) % Q : (Q - yp) % Q;
    }
};

// Register-resident node of L virtual positions (half-split); virtual leaves
// VB .. VB+L-1, i.e. real u indices VB*G .. (VB+L)*G - 1.
template <int Q, int L, int G>
struct QSub {
    static PCUB_HD void run(const QV<Q>* v, uint8_t* y, int vb, QInfo& qi, int lane) {
        if constexpr (L == 1 && G > 1) {
            y[0] = (uint8_t)QXSub<Q, G>::run(v[0], vb * G, qi, lane);
        } else if constexpr (L == 1) {
            int u = 0;
            if (!qi.A->frozen[vb]) {
                u = q_leaf<Q>(v[0]);
                qi.put(u);
            }
            y[0] = (uint8_t)u;
        } else {
            constexpr int H = L / 2;
            QV<Q> c[H];
            uint8_t ym[H], yp[H];
#pragma unroll
            for (int j = 0; j < H; ++j) c[j] = q_minus<Q>(v[j], v[j + H]);
            QSub<Q, H, G>::run(c, ym, vb, qi, lane);
#pragma unroll
            for (int j = 0; j < H; ++j) c[j] = q_plus<Q>(v[j], v[j + H], ym[j]);
            QSub<Q, H, G>::run(c, yp, vb + H, qi, lane);
#pragma unroll
            for (int j = 0; j < H; ++j) {
                y[j] = (uint8_t)((ym[j] + yp[j]) % Q);
                y[j + H] = (uint8_t)((Q - yp[j]) % Q);
            }
        }
    }
};

template <int Q>
PCUB_HD QV<Q> q_load(const double* base, long long pos, long long stride) {
    QV<Q> v;
#pragma unroll
    for (int x = 0; x < Q; ++x) v.p[x] = base[(pos * Q + x) * stride];
    return v;
}

// stage levels: position pos as QP = ceil(Q/2) pairs (an odd Q pads the last one)
template <int Q>
PCUB_HD QV<Q> q_load2(const double2* base, long long pos, long long stride) {
    constexpr int QP = (Q + 1) / 2;
    QV<Q> v;
#pragma unroll
    for (int h = 0; h < QP; ++h) {
        const double2 d = ld2(base + (pos * QP + h) * stride);
        v.p[2 * h] = d.x;
        if (2 * h + 1 < Q) v.p[2 * h + 1] = d.y;
    }
    return v;
}

template <int Q>
PCUB_HD void q_store2(double2* base, long long pos, long long stride, const QV<Q>& v) {
    constexpr int QP = (Q + 1) / 2;
#pragma unroll
    for (int h = 0; h < QP; ++h)
        st2(base + (pos * QP + h) * stride, double2{v.p[2 * h], (2 * h + 1 < Q) ? v.p[2 * h + 1] : 0.0});
}

// Value at position p of the depth-a node on the current chain: the raw root for
// a == 0 (half-split position p = natural row bitrev_n(p)), else stage level a.
struct QLev {
    const double* in;   // root: row i, symbol x at in[(i * B) * Q + x]
    long long B;
    int n;
    const double2* scr;
    long long ns;
    int N;
    template <int Q>
    PCUB_HD QV<Q> get(int a, int p) const {
        if (a == 0) return q_load<Q>(in, (long long)bitrev((uint32_t)p, n) * B, 1);
        return q_load2<Q>(scr, (long long)N - 2 * (N >> a) + p, ns);
    }
};

// S = register positions per lane (a power of two), G lanes per codeword
// (lane j of them, `lane` = wave lane id); requires N >= 2*S*G.  Below, n and N
// are the virtual (per-lane) tree: n = log2(N_real / G).
template <int Q, int S, int G = 1>
PCUB_HD void decode_qary_cw(const QArgs& A, long long cw, long long slot, bool store, int j = 0, int lane = 0) {
    constexpr int s = (S == 1) ? 0 : (S == 2) ? 1 : (S == 4) ? 2 : (S == 8) ? 3 : 4;
    constexpr int g = (G == 1) ? 0 : (G == 2) ? 1 : 2;
    static_assert(G == 1 || G == 2 || G == 4, "lanes per codeword");
    const int n = A.n - g;
    const int N = 1 << n;
    const long long ns = A.nslots;
    const int D = n - s;  // depth of the register nodes
    double2* scr = A.scratch + slot;
    uint32_t* Y = A.ysym + slot;
    // root rows of lane j: real position j + G*t is row bitrev_n(j) + bitrev_{n-g}(t)
    QLev lv{A.xy + (cw + (long long)bitrev((uint32_t)j, A.n) * A.B) * Q, A.B, n, scr, ns, N};
    QInfo qi{&A, cw, store, 0, j, G - 1};
    for (int k = 0; k < (1 << D); ++k) {
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        const int e0 = A.ef[k];  // first all-frozen depth on this chain (D + 1: none)
        const int stop = e0 <= D ? e0 - 1 : D;  // deepest level to evaluate
        int a = d0 - 1;
        bool gop = (k != 0);
        // stored levels a+1 .. min(stop, D-1), two per pass
        while (a < (stop < D ? stop : D - 1)) {
            const int last = stop < D ? stop : D - 1;
            const int F = (last - a) >= 2 ? 2 : 1;
            const int La = N >> a;
            const int ystart = (k >> (D - a)) << (n - a);  // minus child's first Y position
            if (F == 2) {
                const int C = La >> 2;
                for (int p = 0; p < C; ++p) {
                    QV<Q> l1[2];
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        const QV<Q> x0 = lv.template get<Q>(a, p + m * C), x1 = lv.template get<Q>(a, p + (m + 2) * C);
                        l1[m] = gop ? q_plus<Q>(x0, x1, q_sym(Y, ns, ystart + p + m * C)) : q_minus<Q>(x0, x1);
                        q_store2<Q>(scr, (long long)N - 2 * (N >> (a + 1)) + p + m * C, ns, l1[m]);
                    }
                    q_store2<Q>(scr, (long long)N - 2 * (N >> (a + 2)) + p, ns, q_minus<Q>(l1[0], l1[1]));
                }
            } else {
                const int C = La >> 1;
                for (int p = 0; p < C; ++p) {
                    const QV<Q> x0 = lv.template get<Q>(a, p), x1 = lv.template get<Q>(a, p + C);
                    const QV<Q> o = gop ? q_plus<Q>(x0, x1, q_sym(Y, ns, ystart + p)) : q_minus<Q>(x0, x1);
                    q_store2<Q>(scr, (long long)N - 2 * (N >> (a + 1)) + p, ns, o);
                }
            }
            a += F;
            gop = false;
        }
        uint8_t y[S];
        if (stop == D) {
            // level D into registers, then the register subtree
            const int ystart = (k >> (D - a)) << (n - a);
            QV<Q> v[S];
#pragma unroll
            for (int p = 0; p < S; ++p) {
                const QV<Q> x0 = lv.template get<Q>(a, p), x1 = lv.template get<Q>(a, p + S);
                v[p] = gop ? q_plus<Q>(x0, x1, q_sym(Y, ns, ystart + p)) : q_minus<Q>(x0, x1);
            }
            QSub<Q, S, G>::run(v, y, k * S, qi, lane);
        } else {
#pragma unroll
            for (int j = 0; j < S; ++j) y[j] = 0;  // rate-0: symbols 0, re-encoding 0
        }
        // the subtree's symbols into its words (S < 4: a part of one word)
        if constexpr (S >= 4) {
#pragma unroll
            for (int w = 0; w < S / 4; ++w)
                Y[(long long)(k * S / 4 + w) * ns] = (uint32_t)y[4 * w] | ((uint32_t)y[4 * w + 1] << 8) |
                                                     ((uint32_t)y[4 * w + 2] << 16) | ((uint32_t)y[4 * w + 3] << 24);
        } else {
            uint32_t* yw = Y + (long long)((k * S) >> 2) * ns;
            const int sh = ((k * S) & 3) * 8;
            uint32_t ws = 0;
#pragma unroll
            for (int j = 0; j < S; ++j) ws |= (uint32_t)y[j] << (8 * j);
            *yw = (sh == 0 ? 0u : (*yw & ((1u << sh) - 1u))) | (ws << sh);
        }
        // combine completed plus children: [(ym+yp)%q | (q-yp)%q]
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = N >> d;
            const long long st = (long long)(k >> (D - d + 1)) * 2 * Lc;
            if (Lc >= 4) {
                for (int w = 0; w < Lc / 4; ++w) {
                    uint32_t* pm = Y + (st / 4 + w) * ns;
                    uint32_t* pp = Y + (st / 4 + Lc / 4 + w) * ns;
                    uint32_t m = *pm, p = *pp;
                    q_combine_words<Q>(m, p);
                    *pm = m;
                    *pp = p;
                }
            } else {  // Lc = 1, 2: the parent is 2 or 4 bytes of one word
                uint32_t* pw = Y + (st >> 2) * ns;
                const int sh = (int)(st & 3) * 8;
                const uint32_t lm = (Lc == 1) ? 0xffu : 0xffffu;
                uint32_t m = (*pw >> sh) & lm, p = (*pw >> (sh + 8 * Lc)) & lm;
                q_combine_words<Q>(m, p);
                *pw = (*pw & ~(((lm << (8 * Lc)) | lm) << sh)) | (((p << (8 * Lc)) | m) << sh);
            }
        }
    }
    // x_hat[i] is the root's half-split position bitrev(i): lane j holds the rows
    // bitrev_n(j) + bitrev_{n-g}(t), t = its local position
    if (A.xhat && store) {
        uint8_t* xo = A.xhat + cw + (long long)bitrev((uint32_t)j, A.n) * A.B;
        for (int t = 0; t < N; ++t) xo[(long long)bitrev((uint32_t)t, n) * A.B] = (uint8_t)q_sym(Y, ns, t);
    }
}

}  // namespace pcub
