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
// Every quotient p/t is the correctly rounded one (q_div: one IEEE division for
// RN(1/t) per vector, then Markstein's correction per component, inside a guarded
// range; plain division outside it).
//
// Schedule (as the binary kernel, sc_bin_body.h): half-split order inside every
// node; G lanes per codeword, lane j owning positions p = j (mod G) of every node
// of length >= G, so every butterfly of a node of length >= 2G is lane-local and
// each lane runs the one-lane schedule on a virtual tree of N/G positions; a
// virtual leaf is a real node of G positions, one per lane, finished by QXSub<G>
// with cross-lane exchanges.  The bottom S virtual positions of every chain live
// in registers (QSub<S>); stage levels 1..D-1 in a per-slot scratch (q doubles per
// position as ceil(q/2) 16-byte pairs, slot-minor, so a wave's access is one
// contiguous run); re-encoded symbols in 32-bit words (QPack: 2-bit fields at q = 4, else bytes).
//
// Traffic.  Register subtree k is reached by a chain: one plus transform from
// depth d0-1 (minus for k = 0), then minus transforms down to depth D.  A chain
// is evaluated in passes of up to three fused levels, each column depth-first
// (QCol), every level of the pass stored once for the plus transforms to come and
// consumed from registers by the next level; the last pass lands in registers.
// So a stored node is written once and read once (by its plus child's chain),
// except the source of a pass after the first (an extra read, 1/8 of the first
// pass's source).  Nodes whose u range is entirely frozen are never evaluated
// (their symbols are 0 and so is their re-encoding), driven by the per-code
// rate-0 depth table `ef`.
#pragma once
#include "sc_bin_body.h"  // first_frozen_depth, launder, xor_shfl_c, ld2/st2
#include "sc_common.h"

namespace pcub {

template <int Q>
struct QV {
    double p[Q];
};

PCUB_HD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }

// v[x] / t for every component, each the correctly rounded quotient the
// reference's `p[x] /= t` produces.  Fast path: y = RN(1/t) by one IEEE division,
// then per component q0 = RN(p*y) (within an ulp of p/t), r = p - q0*t (exact by
// fma) and RN(q0 + r*y) = RN(p/t) (Markstein).  The guard keeps t, y and every
// quotient far from underflow/overflow (t in [2^-200, 2^200], p = 0 or
// p >= t * 2^-800), where those steps are exact; outside it, plain division.
// tests/emu checks the fast path against division over random and edge inputs.
template <int Q>
PCUB_HD void q_div(QV<Q>& v, double t) {
    // (bitwise & and |, not && and ||: the short-circuit form compiled to one exec-masked branch per
    // component, ~20 scalar instructions a call)
    const double lo = t * 0x1p-800;
    bool fast = (t >= 0x1p-200) & (t <= 0x1p+200);
#pragma unroll
    for (int x = 0; x < Q; ++x) fast = fast & ((v.p[x] == 0.0) | (v.p[x] >= lo));
    // A wave-uniform branch on the vote: when every lane is inside the guard (the common case) the
    // fast path runs with no exec-mask bookkeeping; otherwise the per-lane choice.
    auto fast_div = [&]() {
        const double y = 1.0 / t;
#pragma unroll
        for (int x = 0; x < Q; ++x) {
            const double q0 = v.p[x] * y;
            const double r = fma_d(-q0, t, v.p[x]);
            v.p[x] = fma_d(r, y, q0);
        }
    };
#ifdef __HIP_DEVICE_COMPILE__
    if (__all(fast)) {
        fast_div();
        return;
    }
#endif
    if (fast) {
        fast_div();
    } else if (t != 0.0) {
#pragma unroll
        for (int x = 0; x < Q; ++x) v.p[x] = v.p[x] / t;
    }
}

// t = ((0 + p0) + p1) + ...; p[x] /= t unless t == 0 (then q_div leaves the vector, as the
// reference's `if t != 0` does: the check sits in q_div's per-lane fallback, off the uniform path)
template <int Q>
PCUB_HD QV<Q> q_normalize(QV<Q> v) {
    double t = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) t = t + v.p[x];
    q_div<Q>(v, t);
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
    // r[u2] = a[(u1+u2)%Q] with a lane-divergent u1: rotate by each set bit of u1
    // (ceil(log2 Q) rounds of Q selects) instead of selecting every element
    QV<Q> r = a;
#pragma unroll
    for (int sh = 1; sh < Q; sh <<= 1) {
        const bool on = (u1 & sh) != 0;
        QV<Q> t;
#pragma unroll
        for (int i = 0; i < Q; ++i) t.p[i] = on ? r.p[(i + sh) % Q] : r.p[i];
        r = t;
    }
    QV<Q> o;
#pragma unroll
    for (int u2 = 0; u2 < Q; ++u2) o.p[u2] = 0.0 + r.p[u2] * b.p[(Q - u2) % Q];
    return q_normalize<Q>(o);
}

template <int Q>
PCUB_HD int q_leaf(QV<Q> v) {
    double s = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) s = s + v.p[x];
    if (!(s > 0.0)) return 0;  // every marginal 1/q: the first index
    q_div<Q>(v, s);
    int arg = 0;
    double best = v.p[0];
#pragma unroll
    for (int x = 1; x < Q; ++x) {
        if (v.p[x] > best) {
            best = v.p[x];
            arg = x;
        }
    }
    return arg;
}

struct QArgs {
    const double* xy;        // [N][B][Q]
    long long B;
    int n;
    const uint32_t* fwords;  // [ceil(N/32)] frozen mask, bit i = position i
    const uint8_t* ef;       // [2^D] first rate-0 depth on each register subtree's chain
    uint8_t* info;           // [K][B]
    uint8_t* xhat;           // [N][B] or null
    double2* scratch;        // [(N/G - 2S) positions][ceil(Q/2)][nslots]
    uint32_t* ysym;          // [ceil(N/G/PER) words][nslots], symbol of position p in field p % PER of word p / PER
                             // (QPack: PER = 16 2-bit fields at q = 4, else 4 bytes)
    long long nslots;
    int ylds_words;          // symbol words per thread in LDS (YL kernels; the HL column follows them)
    int tile;                // root layout: 0 = [N][B][Q]; T > 0 = [ceil(B/T)][N][T][Q] (T codewords a tile)
    unsigned long long* wtiles = nullptr;  // wave tiles from this counter (zeroed per launch), or the static stride
};

// Re-encoded symbols packed into 32-bit words: q = 4 in 2-bit fields (16 a word: the C4 kernel's
// column is 4 words a thread at N = 256, which lets four split-level workgroups share a CU's LDS),
// every other q one byte each (four a word).
template <int Q>
struct QPack {
    static constexpr int BITS = (Q == 4) ? 2 : 8;
    static constexpr int PER = 32 / BITS;  // symbols per word
    static constexpr uint32_t M = (1u << BITS) - 1u;
};

// SWAR on bytes: every byte holds a value < 2Q <= 16, so byte sums never carry, and
// (b | 0x80) - Q >= 0x78 never borrows; its bit 7 is set iff b >= Q.
template <int Q>
PCUB_HD uint32_t q_mod_bytes(uint32_t s) {
    const uint32_t ge = (((s | 0x80808080u) - (uint32_t)Q * 0x01010101u) & 0x80808080u) >> 7;
    return s - ge * (uint32_t)Q;
}

// 2-bit fields: a + b mod 4 in every field (the low bits' sum carries into the high bit, the high
// bits XOR; nothing crosses a field)
PCUB_HD uint32_t add_mod4_fields(uint32_t a, uint32_t b) {
    constexpr uint32_t H = 0xAAAAAAAAu;
    return ((a & ~H) + (b & ~H)) ^ ((a ^ b) & H);
}

// parent = [(ym + yp) % Q | (Q - yp) % Q]  (QaryPolarEncoderDecoder.py:397-399, half-split order)
template <int Q>
PCUB_HD void q_combine_words(uint32_t& m, uint32_t& p) {
    if constexpr (QPack<Q>::BITS == 2) {
        const uint32_t mm = add_mod4_fields(m, p);
        p = add_mod4_fields(~p, 0x55555555u);  // -p = ~p + 1 (mod 4) in every field
        m = mm;
    } else {
        const uint32_t mm = q_mod_bytes<Q>(m + p);
        p = q_mod_bytes<Q>((uint32_t)Q * 0x01010101u - p);
        m = mm;
    }
}

// YL: the symbols live in LDS (this thread's column, ldy/sty of sc_bin_body.h)
template <int Q, bool YL = false>
PCUB_HD int q_sym(const uint32_t* Y, long long ns, int pos) {
    using P = QPack<Q>;
    return (int)((ldy<YL>(Y + (long long)(pos / P::PER) * ns) >> ((pos % P::PER) * P::BITS)) & P::M);
}

// Decisions of the register subtree: information symbols go out in u order
// (identical in the G lanes of a codeword; lane w % G stores row w).  Plain
// fields, no pointer to the kernel argument (that would put it in scratch).
struct QInfo {
    uint8_t* info;
    long long B;
    long long cw;
    bool store;
    int w;     // next information row
    int j;     // lane of the codeword
    int gm;    // G - 1
    uint64_t fm;  // frozen bits of the current register subtree's real u range
    PCUB_HD void put(int u) {
        if (store && (w & gm) == j) info[(long long)w * B + cw] = (uint8_t)u;
        ++w;
    }
    PCUB_HD bool frozen(int ub) const { return (fm >> ub) & 1ull; }
};

// Exchange of a whole q-vector with lane ^ MASK.
template <int Q, int MASK>
PCUB_HD QV<Q> q_shfl(const QV<Q>& v) {
    QV<Q> w;
#pragma unroll
    for (int x = 0; x < Q; ++x) w.p[x] = xor_shfl_c<MASK>(v.p[x]);
    return w;
}

// The pair (a, b) = (the value of the pair's first lane, of its second) in both lanes of every
// pair (lane, lane ^ H), H = 1 or 2 (inside a quad): two DPP broadcasts per 32 bits, quad_perm
// [0,0,2,2] / [1,1,3,3] (H = 1) or [0,1,0,1] / [2,3,2,3] (H = 2), instead of an exchange with the
// partner and a select of the q doubles by lane parity (round 5).  Wider pairs: the exchange.
template <int Q, int H>
PCUB_HD void q_pair(const QV<Q>& v, int lane, QV<Q>& a, QV<Q>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (H == 1 || H == 2) {
        constexpr int LO = H == 1 ? 0xA0 : 0x44, HI = H == 1 ? 0xF5 : 0xEE;
#pragma unroll
        for (int x = 0; x < Q; ++x) {
            const unsigned long long bits = (unsigned long long)as_bits(v.p[x]);
            const unsigned l0 = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)bits, LO, 0xF, 0xF, false);
            const unsigned l1 = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(bits >> 32), LO, 0xF, 0xF, false);
            const unsigned h0 = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)bits, HI, 0xF, 0xF, false);
            const unsigned h1 = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(bits >> 32), HI, 0xF, 0xF, false);
            a.p[x] = from_bits((long long)(((unsigned long long)l1 << 32) | l0));
            b.p[x] = from_bits((long long)(((unsigned long long)h1 << 32) | h0));
        }
        return;
    }
#endif
    const QV<Q> w = q_shfl<Q, H>(v);
    const bool lo = (lane & H) == 0;
#pragma unroll
    for (int x = 0; x < Q; ++x) {
        a.p[x] = lo ? v.p[x] : w.p[x];
        b.p[x] = lo ? w.p[x] : v.p[x];
    }
}

// A real node of M <= G positions, position (lane & (M-1)) in each lane; leaf u
// indices UB .. UB+M-1 of the register subtree.  Returns this lane's symbol of
// the node's re-encoding.
template <int Q, int M>
struct QXSub {
    static PCUB_HD int run(const QV<Q>& v, int ub, QInfo& qi, int lane) {
        const bool lo = (lane & (M / 2)) == 0;
        QV<Q> a, b;
        q_pair<Q, M / 2>(v, lane, a, b);
        int ym, yp;
        if constexpr (M == 2) {
            ym = 0;
            if (!qi.frozen(ub)) {
                ym = q_leaf<Q>(q_minus<Q>(a, b));
                qi.put(ym);
            }
            yp = 0;
            if (!qi.frozen(ub + 1)) {
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
// VB .. VB+L-1 of the subtree, i.e. its real u indices VB*G .. (VB+L)*G - 1.
template <int Q, int L, int G>
struct QSub {
    static PCUB_HD void run(const QV<Q>* v, uint8_t* y, int vb, QInfo& qi, int lane) {
        if constexpr (L == 1 && G > 1) {
            y[0] = (uint8_t)QXSub<Q, G>::run(v[0], vb * G, qi, lane);
        } else if constexpr (L == 1) {
            int u = 0;
            if (!qi.frozen(vb)) {
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
PCUB_HD QV<Q> q_load(const double* base, long long off) {
    QV<Q> v;
#pragma unroll
    for (int x = 0; x < Q; ++x) v.p[x] = base[off + x];
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

// One pass of a chain: source depth a (the raw root when a == 0), levels
// a+1 .. a+F evaluated column by column.  Column c (C = La >> F columns) holds
// level a+e at positions c + m*C, m < 2^(F-e).
struct QPass {
    const double* in;     // root: half-split position p of lane j is row rowbase + bitrev_{nv}(p)
    uint32_t lin;         // TR: this lane's byte offset from in (a wave-uniform tile base); else 0
    long long B;
    int nv;               // log2 of the virtual (per-lane) length
    const double2* src;   // stored source level (a > 0)
    double2* lev[4];      // destinations: levels a+1 .. a+F (stored ones)
    long long ns;
    const uint32_t* Y;    // re-encoded symbols (plus transform decisions), word w at Y[w * ys]
    long long ys;
    int ystart;           // first Y position of the minus child at depth a+1
};

template <int Q, bool ROOT>
PCUB_HD QV<Q> q_src(const QPass& P, int pos) {
    if constexpr (ROOT)
        return q_load<Q>((const double*)((const char*)(P.in + (long long)bitrev((uint32_t)pos, P.nv) * P.B * Q) + P.lin), 0);
    else return q_load2<Q>(P.src, pos, P.ns);
}

// Value of level a+E at index M of column c (position c + M*C), depth-first; every
// level below a+F, and a+F itself unless FINAL, is stored on the way.
template <int Q, int F, int E, int M, bool GOP, bool ROOT, bool FINAL, bool YL>
struct QCol {
    static PCUB_HD QV<Q> run(const QPass& P, int c, int C) {
        QV<Q> v;
        if constexpr (E == 1) {
            const QV<Q> x0 = q_src<Q, ROOT>(P, c + M * C);
            const QV<Q> x1 = q_src<Q, ROOT>(P, c + (M + (1 << (F - 1))) * C);
            if constexpr (GOP) v = q_plus<Q>(x0, x1, q_sym<Q, YL>(P.Y, P.ys, P.ystart + c + M * C));
            else v = q_minus<Q>(x0, x1);
        } else {
            const QV<Q> l = QCol<Q, F, E - 1, M, GOP, ROOT, FINAL, YL>::run(P, c, C);
            const QV<Q> r = QCol<Q, F, E - 1, M + (1 << (F - E)), GOP, ROOT, FINAL, YL>::run(P, c, C);
            v = q_minus<Q>(l, r);
        }
        if constexpr (E < F || !FINAL) q_store2<Q>(P.lev[E - 1], c + M * C, P.ns, v);
        return v;
    }
};

// Non-final pass over all La >> F columns (U columns per iteration: loads of the
// next column in flight while the current one computes).
template <int Q, int F, bool GOP, bool ROOT, int U = 1, bool YL = false>
PCUB_HD void q_pass(const QPass& P, int La) {
    const int C = La >> F;
    if constexpr (U == 1) {
#pragma unroll 1
        for (int c = 0; c < C; ++c) QCol<Q, F, F, 0, GOP, ROOT, false, YL>::run(P, c, C);
    } else {
        int c = 0;
#pragma unroll 1
        for (; c + U <= C; c += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) QCol<Q, F, F, 0, GOP, ROOT, false, YL>::run(P, c + u, C);
        }
#pragma unroll 1
        for (; c < C; ++c) QCol<Q, F, F, 0, GOP, ROOT, false, YL>::run(P, c, C);
    }
}

// Final pass: level D (S values) into registers.
template <int Q, int S, int F, bool GOP, bool ROOT, bool YL>
PCUB_HD void q_final(const QPass& P, QV<Q>* v) {
#pragma unroll
    for (int c = 0; c < S; ++c) v[c] = QCol<Q, F, F, 0, GOP, ROOT, true, YL>::run(P, c, S);
}

// Final pass of a split-level (HL) chain: the 2S positions of level D, the first S into this
// thread's LDS column hl (component x of position c at hl[(c * Q + x) * kQHlStride]), the
// last S into registers.
constexpr int kQHlStride = 256;  // threads per workgroup (kQaryBlock)

template <int Q, int S, int F, bool GOP, bool ROOT, bool YL>
PCUB_HD void q_final_hl(const QPass& P, QV<Q>* v, double* hl) {
#pragma unroll
    for (int c = 0; c < 2 * S; ++c) {
        const QV<Q> x = QCol<Q, F, F, 0, GOP, ROOT, true, YL>::run(P, c, 2 * S);
        if (c < S) {
#pragma unroll
            for (int t = 0; t < Q; ++t) hl[(c * Q + t) * kQHlStride] = x.p[t];
        } else {
            v[c - S] = x;
        }
    }
}

template <int Q>
PCUB_HD QV<Q> q_hl_load(const double* hl, int c) {
    QV<Q> v;
#pragma unroll
    for (int t = 0; t < Q; ++t) v.p[t] = hl[(c * Q + t) * kQHlStride];
    return v;
}

// The split level's node: 2S positions per lane, the first S in the LDS column, the last S in
// registers (QSub<Q, 2S, G>'s top node with its parent split); a child whose u range is all
// frozen is not evaluated (symbols 0, as the rate-0 chains).
template <int Q, int S, int G>
PCUB_HD void q_hl_run(const double* hl, const QV<Q>* vr, uint8_t* y, QInfo& qi, int lane) {
    constexpr int SH = S * G;  // u positions per child
    constexpr uint64_t HM = (SH == 64) ? ~0ull : ((1ull << SH) - 1ull);
    QV<Q> c[S];
    uint8_t ym[S], yp[S];
    if ((qi.fm & HM) == HM) {
#pragma unroll
        for (int t = 0; t < S; ++t) ym[t] = 0;
    } else {
#pragma unroll
        for (int t = 0; t < S; ++t) c[t] = q_minus<Q>(q_hl_load<Q>(hl, t), vr[t]);
        QSub<Q, S, G>::run(c, ym, 0, qi, lane);
    }
    if (((qi.fm >> SH) & HM) == HM) {
#pragma unroll
        for (int t = 0; t < S; ++t) yp[t] = 0;
    } else {
#pragma unroll
        for (int t = 0; t < S; ++t) c[t] = q_plus<Q>(q_hl_load<Q>(hl, t), vr[t], ym[t]);
        QSub<Q, S, G>::run(c, yp, S, qi, lane);
    }
#pragma unroll
    for (int t = 0; t < S; ++t) {
        y[t] = (uint8_t)((ym[t] + yp[t]) % Q);
        y[t + S] = (uint8_t)((Q - yp[t]) % Q);
    }
}

template <int Q, int F, int U, bool YL>
PCUB_HD void q_pass_dispatch(const QPass& P, int La, bool gop, bool root) {
    if (root) {
        if (gop) q_pass<Q, F, true, true, U, YL>(P, La);
        else q_pass<Q, F, false, true, U, YL>(P, La);
    } else {
        if (gop) q_pass<Q, F, true, false, U, YL>(P, La);
        else q_pass<Q, F, false, false, U, YL>(P, La);
    }
}

template <int Q, int S, int F, bool YL, bool HL = false>
PCUB_HD void q_final_dispatch(const QPass& P, QV<Q>* v, bool gop, bool root, double* hl = nullptr) {
    if constexpr (HL) {
        if (root) {
            if (gop) q_final_hl<Q, S, F, true, true, YL>(P, v, hl);
            else q_final_hl<Q, S, F, false, true, YL>(P, v, hl);
        } else {
            if (gop) q_final_hl<Q, S, F, true, false, YL>(P, v, hl);
            else q_final_hl<Q, S, F, false, false, YL>(P, v, hl);
        }
    } else {
        if (root) {
            if (gop) q_final<Q, S, F, true, true, YL>(P, v);
            else q_final<Q, S, F, false, true, YL>(P, v);
        } else {
            if (gop) q_final<Q, S, F, true, false, YL>(P, v);
            else q_final<Q, S, F, false, false, YL>(P, v);
        }
    }
}

// S = register positions per lane (a power of two), G lanes per codeword
// (lane j of them, `lane` = wave lane id); requires N >= 2*S*G and S*G <= 64.
// G = 8, 16 hold one or two more tree levels per codeword on chip than G = 4 (one
// stored stage level fewer each) at the price of duplicated work in the cross-lane
// leaf levels (both lanes of an exchanging pair evaluate the same transform).
// YL: the symbols in LDS (ylds = this thread's column, word w at ylds[w * ystride])
// HL: the chain ends at a split level of 2S positions per lane (the first S in the LDS column
//     hl, the rest in registers; q_hl_run): one stored stage depth fewer (8qN bytes written and
//     8qN read less per codeword)
// NC >= 0: the code length 2^NC is a compile-time constant (the kernel runs only at it), so the per-
// position row offsets and level bases fold (binary decode_codeword's NC); TR kernels also know
// their tile width, 64 / G.
template <int Q, int S, int G = 1, int U = 1, bool YL = false, bool HL = false, bool TR = false, int NC = -1>
PCUB_HD void decode_qary_cw(const QArgs& A, long long cw, long long slot, bool store, int j = 0, int lane = 0,
                            uint32_t* ylds = nullptr, long long ystride = 0, double* hl = nullptr) {
    constexpr int SR = HL ? 2 * S : S;  // positions per lane at the chain's last level
    constexpr int s = (SR == 1) ? 0 : (SR == 2) ? 1 : (SR == 4) ? 2 : (SR == 8) ? 3 : (SR == 16) ? 4 : 5;
    constexpr int g = (G == 1) ? 0 : (G == 2) ? 1 : (G == 4) ? 2 : (G == 8) ? 3 : 4;
    constexpr int SU = SR * G;  // real u positions per chain-end subtree
    constexpr int QP = (Q + 1) / 2;
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "lanes per codeword");
    static_assert(SU <= 64, "a register subtree's frozen bits fit one 64-bit word");
    const int n = NC >= 0 ? NC : A.n;
    const int nv = n - g;
    const int Nv = 1 << nv;
    const long long ns = A.nslots;
    const int D = nv - s;  // depth of the register nodes
    double2* scr = A.scratch + slot;
    uint32_t* Y = YL ? ylds : A.ysym + slot;
    const long long ys = YL ? ystride : ns;  // symbol word stride
    // root rows of lane j: real position j + G*t is row bitrev_n(j) + bitrev_{nv}(t)
    // tiled layout: codeword cw's row 0 at ((cw / T) N) T + cw % T, rows T apart
    const long long rs = TR ? 64 / G : A.tile > 0 ? (long long)A.tile : A.B;
    const long long rb = A.tile > 0 ? (cw / rs) * (rs << n) + cw % rs : cw;
    // TR (tile = the wave's 64 / G codewords): the tile's base wave-uniform (SGPRs), this lane's rows
    // a 32-bit byte offset (binary decode_codeword's TR)
    const double* in;
    uint32_t lin = 0;
    if constexpr (TR) {
        in = A.xy + uniform64((cw / rs) * (rs << n)) * Q;
        lin = (uint32_t)((cw % rs + (long long)bitrev((uint32_t)j, n) * rs) * Q * 8);
    } else {
        in = A.xy + (rb + (long long)bitrev((uint32_t)j, n) * rs) * Q;
    }
    QInfo qi{A.info, A.B, cw, store, 0, j, G - 1, 0u};
    for (int k = 0; k < (1 << D); ++k) {
        if constexpr (TR) in = launder_s(in);
        else in = launder(in);
        scr = launder(scr);
        if constexpr (!YL) Y = launder(Y);
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        const int e0 = A.ef[k];  // first all-frozen depth on this chain (D + 1: none)
        const int stop = e0 <= D ? e0 - 1 : D;  // deepest level to evaluate
        int a = d0 - 1;
        bool gop = (k != 0);
        QPass P;
        P.in = in;
        P.lin = lin;
        P.B = rs;
        P.nv = nv;
        P.ns = ns;
        P.Y = Y;
        P.ys = ys;
        // passes of up to three levels, greedily from the top; the last one (when the
        // chain reaches depth D) lands in registers
        while (true) {
            const int last = stop;  // deepest level of this chain
            const int T = last - a;
            if (T <= 0) break;
            const bool fin = (last == D) && T <= 3;
            const int F = T >= 3 ? 3 : T;
            P.src = a > 0 ? scr + (long long)(Nv - 2 * (Nv >> a)) * QP * ns : nullptr;
            P.ystart = (k >> (D - a)) << (nv - a);
#pragma unroll
            for (int e = 1; e <= 3; ++e)
                P.lev[e - 1] = (a + e < D) ? scr + (long long)(Nv - 2 * (Nv >> (a + e))) * QP * ns : nullptr;
            if (fin) break;
            const int La = Nv >> a;
            if (F == 3) q_pass_dispatch<Q, 3, U, YL>(P, La, gop, a == 0);
            else if (F == 2) q_pass_dispatch<Q, 2, U, YL>(P, La, gop, a == 0);
            else q_pass_dispatch<Q, 1, U, YL>(P, La, gop, a == 0);
            a += F;
            gop = false;
        }
        uint8_t y[SR];
        if (stop == D) {
            QV<Q> v[S];
            const int F = D - a;
            if (F == 3) q_final_dispatch<Q, S, 3, YL, HL>(P, v, gop, a == 0, hl);
            else if (F == 2) q_final_dispatch<Q, S, 2, YL, HL>(P, v, gop, a == 0, hl);
            else q_final_dispatch<Q, S, 1, YL, HL>(P, v, gop, a == 0, hl);
            const int us = k * SU;
            if constexpr (SU == 64) qi.fm = (uint64_t)A.fwords[us >> 5] | ((uint64_t)A.fwords[(us >> 5) + 1] << 32);
            else if constexpr (SU == 32) qi.fm = (uint64_t)A.fwords[us >> 5];
            else qi.fm = (uint64_t)(A.fwords[us >> 5] >> (us & 31));
            if constexpr (HL) q_hl_run<Q, S, G>(hl, v, y, qi, lane);
            else QSub<Q, S, G>::run(v, y, 0, qi, lane);
        } else {
#pragma unroll
            for (int t = 0; t < SR; ++t) y[t] = 0;  // rate-0: symbols 0, re-encoding 0
        }
        // the subtree's symbols into its words (SR < PER: a part of one word)
        constexpr int PER = QPack<Q>::PER, BITS = QPack<Q>::BITS;
        if constexpr (SR >= PER) {
#pragma unroll
            for (int w = 0; w < SR / PER; ++w) {
                uint32_t ws = 0;
#pragma unroll
                for (int t = 0; t < PER; ++t) ws |= (uint32_t)y[PER * w + t] << (BITS * t);
                sty<YL>(Y + (long long)(k * SR / PER + w) * ys, ws);
            }
        } else {
            uint32_t* yw = Y + (long long)((k * SR) / PER) * ys;
            const int sh = ((k * SR) % PER) * BITS;
            uint32_t ws = 0;
#pragma unroll
            for (int t = 0; t < SR; ++t) ws |= (uint32_t)y[t] << (BITS * t);
            sty<YL>(yw, (sh == 0 ? 0u : (ldy<YL>(yw) & ((1u << sh) - 1u))) | (ws << sh));
        }
        // combine completed plus children: [(ym+yp)%q | (q-yp)%q]
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = Nv >> d;
            const long long st = (long long)(k >> (D - d + 1)) * 2 * Lc;
            if (Lc >= PER) {
                for (int w = 0; w < Lc / PER; ++w) {
                    uint32_t* pm = Y + (st / PER + w) * ys;
                    uint32_t* pp = Y + (st / PER + Lc / PER + w) * ys;
                    uint32_t m = ldy<YL>(pm), p = ldy<YL>(pp);
                    q_combine_words<Q>(m, p);
                    sty<YL>(pm, m);
                    sty<YL>(pp, p);
                }
            } else {  // 2 Lc <= PER: the parent is 2 Lc fields of one word
                uint32_t* pw = Y + (st / PER) * ys;
                const int sh = (int)(st % PER) * BITS;
                const uint32_t lm = (1u << (BITS * Lc)) - 1u;
                const uint32_t w0 = ldy<YL>(pw);
                uint32_t m = (w0 >> sh) & lm, p = (w0 >> (sh + BITS * Lc)) & lm;
                q_combine_words<Q>(m, p);
                sty<YL>(pw, (w0 & ~(((lm << (BITS * Lc)) | lm) << sh)) | ((((p & lm) << (BITS * Lc)) | (m & lm)) << sh));
            }
        }
    }
    // x_hat[i] is the root's half-split position bitrev(i): lane j holds the rows
    // bitrev_n(j) + bitrev_{nv}(t), t = its local position
    if (A.xhat && store) {
        uint8_t* xo = A.xhat + cw + (long long)bitrev((uint32_t)j, n) * A.B;
        for (int t = 0; t < Nv; ++t) xo[(long long)bitrev((uint32_t)t, nv) * A.B] = (uint8_t)q_sym<Q, YL>(Y, ys, t);
    }
}

}  // namespace pcub
