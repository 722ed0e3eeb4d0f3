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
// per position, slot-minor).  A chain -- one plus transform, then minus transforms
// down to depth D -- is evaluated in passes of up to two fused levels per column,
// so a level written inside a pass is consumed from registers by the next one.
// Nodes whose u range is entirely frozen are never evaluated (their symbols are 0
// and so is their re-encoding), driven by the per-code rate-0 depth table `ef`.
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
    double* scratch;        // [(N - 2S) positions][Q][nslots]
    uint8_t* ysym;          // [N][nslots]
    long long nslots;
};

// Decisions of the register subtree: information symbols go out in u order.
struct QInfo {
    const QArgs* A;
    long long cw;
    bool store;
    int w;  // next information row
    PCUB_HD void put(int u) {
        if (store) A->info[(long long)w * A->B + cw] = (uint8_t)u;
        ++w;
    }
};

// Register-resident node of L positions (half-split); leaf u indices UB .. UB+L-1.
template <int Q, int L>
struct QSub {
    static PCUB_HD void run(const QV<Q>* v, uint8_t* y, int ub, QInfo& qi) {
        if constexpr (L == 1) {
            int u = 0;
            if (!qi.A->frozen[ub]) {
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
            QSub<Q, H>::run(c, ym, ub, qi);
#pragma unroll
            for (int j = 0; j < H; ++j) c[j] = q_plus<Q>(v[j], v[j + H], ym[j]);
            QSub<Q, H>::run(c, yp, ub + H, qi);
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

template <int Q>
PCUB_HD void q_store(double* base, long long pos, long long stride, const QV<Q>& v) {
#pragma unroll
    for (int x = 0; x < Q; ++x) base[(pos * Q + x) * stride] = v.p[x];
}

// Value at position p of the depth-a node on the current chain: the raw root for
// a == 0 (half-split position p = natural row bitrev_n(p)), else stage level a.
struct QLev {
    const double* in;   // root: row i, symbol x at in[(i * B) * Q + x]
    long long B;
    int n;
    const double* scr;
    long long ns;
    int N;
    template <int Q>
    PCUB_HD QV<Q> get(int a, int p) const {
        if (a == 0) return q_load<Q>(in, (long long)bitrev((uint32_t)p, n) * B, 1);
        return q_load<Q>(scr, (long long)N - 2 * (N >> a) + p, ns);
    }
};

// S = register positions (a power of two, N >= 2S).
template <int Q, int S>
PCUB_HD void decode_qary_cw(const QArgs& A, long long cw, long long slot, bool store) {
    constexpr int s = (S == 1) ? 0 : (S == 2) ? 1 : (S == 4) ? 2 : (S == 8) ? 3 : 4;
    const int n = A.n;
    const int N = 1 << n;
    const long long ns = A.nslots;
    const int D = n - s;  // depth of the register nodes
    double* scr = A.scratch + slot;
    uint8_t* Y = A.ysym + slot;
    QLev lv{A.xy + cw * Q, A.B, n, scr, ns, N};
    QInfo qi{&A, cw, store, 0};
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
                        l1[m] = gop ? q_plus<Q>(x0, x1, Y[(long long)(ystart + p + m * C) * ns]) : q_minus<Q>(x0, x1);
                        q_store<Q>(scr, (long long)N - 2 * (N >> (a + 1)) + p + m * C, ns, l1[m]);
                    }
                    q_store<Q>(scr, (long long)N - 2 * (N >> (a + 2)) + p, ns, q_minus<Q>(l1[0], l1[1]));
                }
            } else {
                const int C = La >> 1;
                for (int p = 0; p < C; ++p) {
                    const QV<Q> x0 = lv.template get<Q>(a, p), x1 = lv.template get<Q>(a, p + C);
                    const QV<Q> o = gop ? q_plus<Q>(x0, x1, Y[(long long)(ystart + p) * ns]) : q_minus<Q>(x0, x1);
                    q_store<Q>(scr, (long long)N - 2 * (N >> (a + 1)) + p, ns, o);
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
                v[p] = gop ? q_plus<Q>(x0, x1, Y[(long long)(ystart + p) * ns]) : q_minus<Q>(x0, x1);
            }
            QSub<Q, S>::run(v, y, k * S, qi);
        } else {
#pragma unroll
            for (int j = 0; j < S; ++j) y[j] = 0;  // rate-0: symbols 0, re-encoding 0
        }
#pragma unroll
        for (int j = 0; j < S; ++j) Y[(long long)(k * S + j) * ns] = y[j];
        // combine completed plus children: [(ym+yp)%q | (q-yp)%q]
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = N >> d;
            const long long st = (long long)(k >> (D - d + 1)) * 2 * Lc;
            for (int p = 0; p < Lc; ++p) {
                const int ym = Y[(st + p) * ns], yp = Y[(st + Lc + p) * ns];
                Y[(st + p) * ns] = (uint8_t)((ym + yp) % Q);
                Y[(st + Lc + p) * ns] = (uint8_t)((Q - yp) % Q);
            }
        }
    }
    if (A.xhat && store)
        for (int i = 0; i < N; ++i) A.xhat[(long long)i * A.B + cw] = Y[(long long)bitrev((uint32_t)i, n) * ns];
}

}  // namespace pcub
