// sc_bin_body.h -- one-codeword SC decode schedule (binary, uniform prior).
//
// Replaces BinaryPolarEncoderDecoder.recursiveEncodeDecode (decode branch,
// BinaryPolarEncoderDecoder.py:223-325).  G lanes decode one codeword (G = 1, 2,
// 4, 8); all lanes of a wave run the identical (data-independent) tree schedule.
//
// Storage ("half-split" = bit-reversed order inside every node).  A node of
// length L keeps its values at positions p = 0..L-1 such that its minus/plus
// children are  out[p] = op(in[p], in[p + L/2]).  The reference pairs rows
// (2h, 2h+1); position p holds row bitrev_L(p), which makes both statements
// the same computation.  The node's re-encoded vector in the same order is
//     y = [ y_minus ^ y_plus | y_plus ]
// (BinaryPolarEncoderDecoder.py:319-323 permuted), so partial sums are combined
// IN PLACE by a word-wise XOR of the left half with the right half.
//
// Lanes of a codeword.  Lane j of the G lanes owns the positions p = j (mod G)
// of every node with L >= G (local index t = p / G).  Because p and p + L/2
// have the same residue, every butterfly with L >= 2G is lane-local, and each
// lane runs exactly the G = 1 schedule on a "virtual" tree of length N/G.  A
// virtual leaf is a real node of length G holding one value per lane; it is
// finished by XSub<G> with cross-lane exchanges (lane ^ G/2, ^ G/4, .., ^ 1).
// The re-encoded bits also stay lane-local, and x_hat's natural-order segment
// k (N/G bits) is exactly lane bitrev_g(k)'s local bits, bit-reversed.
//
// Levels (per lane, virtual): depth d holds N_v >> d values.  Depth 0 is the
// input (never normalised, never copied).  Depths 1 .. D-1 live in a per-slot
// scratch buffer (compact f64, two values per 16-byte access, slot-minor so a
// wave's access is one contiguous 1 KiB).  Depth D = log2(N_v / S) goes straight
// to registers and the S-value subtree below it is fully unrolled (SubV).
#pragma once
#include "sc_common.h"

namespace pcub {

struct BinArgs {
    const double2* xy;         // [N][B] raw pairs
    long long B;
    int n;                     // log2 N
    const uint32_t* fmask;     // ceil(N/32)
    const uint32_t* fval;      // ceil(N/32)
    uint32_t* info;            // [ceil(K/32)][B]
    uint32_t* xhat;            // [ceil(N/32)][B] or null
    uint32_t* uout;            // [ceil(N/32)][B] or null
    double2* scratch;          // [(N_v/2 - S) pairs][nslots]
    uint32_t* ybits;           // [N_v/32][nslots]
    long long nslots;
};

#if defined(__HIP_DEVICE_COMPILE__)
PCUB_HD double xor_shfl(double v, int mask) { return __shfl_xor(v, mask); }
#else
PCUB_HD double xor_shfl(double v, int) { return v; }  // host emulation runs G = 1 only
#endif

// A real node of length M (M <= G) with position (lane & (M-1)) held by each lane.
// Returns this lane's bit of the node's (half-split) encoding; ORs the M
// decisions u_UBASE .. u_UBASE+M-1 (identical in all lanes) into ub.
template <int M, int UBASE>
struct XSub {
    static PCUB_HD uint32_t run(double v, uint64_t& ub, uint64_t fm, uint64_t fv, int lane) {
        const double w = xor_shfl(v, M / 2);
        const bool lo = (lane & (M / 2)) == 0;
        const double a = lo ? v : w, b = lo ? w : v;
        if constexpr (M == 2) {
            const uint32_t u0 = ((fm >> UBASE) & 1u) ? (uint32_t)((fv >> UBASE) & 1u) : leaf_f(a, b);
            const uint32_t u1 = ((fm >> (UBASE + 1)) & 1u) ? (uint32_t)((fv >> (UBASE + 1)) & 1u) : leaf_g(a, b, u0);
            ub |= ((uint64_t)u0 << UBASE) | ((uint64_t)u1 << (UBASE + 1));
            return lo ? (u0 ^ u1) : u1;
        } else {
            const uint32_t ym = XSub<M / 2, UBASE>::run(op_f(a, b), ub, fm, fv, lane);
            const uint32_t yp = XSub<M / 2, UBASE + M / 2>::run(op_g(a, b, ym), ub, fm, fv, lane);
            return lo ? (ym ^ yp) : yp;
        }
    }
};

// Register-resident virtual subtree of L values per lane; virtual leaf BASE_V
// covers real u positions [BASE_V*G, BASE_V*G + G).  Returns L local encoding bits.
template <int L, int BASE_V, int G>
struct SubV {
    static PCUB_HD uint32_t run(const double* v, uint64_t& ub, uint64_t fm, uint64_t fv, int lane) {
        if constexpr (L == 1) {
            static_assert(G >= 2, "G == 1 stops at L == 2");
            return XSub<G, BASE_V * G>::run(v[0], ub, fm, fv, lane);
        } else if constexpr (L == 2 && G == 1) {
            const uint32_t u0 = ((fm >> BASE_V) & 1u) ? (uint32_t)((fv >> BASE_V) & 1u) : leaf_f(v[0], v[1]);
            const uint32_t u1 =
                ((fm >> (BASE_V + 1)) & 1u) ? (uint32_t)((fv >> (BASE_V + 1)) & 1u) : leaf_g(v[0], v[1], u0);
            ub |= ((uint64_t)u0 << BASE_V) | ((uint64_t)u1 << (BASE_V + 1));
            return (u0 ^ u1) | (u1 << 1);
        } else {
            double c[L / 2];
#pragma unroll
            for (int t = 0; t < L / 2; ++t) c[t] = op_f(v[t], v[t + L / 2]);
            const uint32_t ym = SubV<L / 2, BASE_V, G>::run(c, ub, fm, fv, lane);
#pragma unroll
            for (int t = 0; t < L / 2; ++t) c[t] = op_g(v[t], v[t + L / 2], (ym >> t) & 1u);
            const uint32_t yp = SubV<L / 2, BASE_V + L / 2, G>::run(c, ub, fm, fv, lane);
            return (ym ^ yp) | (yp << (L / 2));
        }
    }
};

// op from a level held in scratch (compact values), two outputs per pair.
// Outputs pairs [0, Po) of depth d from the node at depth d-1 (2*Po pairs).
template <bool G_OP>
PCUB_HD void level_from_scratch(const double2* src, double2* dst, long long ns, int Po, const uint32_t* ybase) {
#pragma unroll 2
    for (int jp = 0; jp < Po; ++jp) {
        const double2 a = src[(long long)jp * ns];
        const double2 b = src[(long long)(jp + Po) * ns];
        double2 o;
        if (G_OP) {
            const uint32_t w = ybase[(long long)(jp >> 4) * ns];
            const uint32_t sh = (uint32_t)(2 * jp) & 31u;
            o.x = op_g(a.x, b.x, (w >> sh) & 1u);
            o.y = op_g(a.y, b.y, (w >> (sh + 1)) & 1u);
        } else {
            o.x = op_f(a.x, b.x);
            o.y = op_f(a.y, b.y);
        }
        dst[(long long)jp * ns] = o;
    }
}

// Natural row pair of the root at local position t of lane j: real position
// p = j + G*t < N/2 pairs rows (2q, 2q+1) with q = bitrev_{n-1}(p).
template <int G>
PCUB_HD long long root_pair(int j, int t, int n) {
    return (long long)bitrev((uint32_t)(j + G * t), n - 1);
}

// op from the raw root (depth 0).  For even t, p + G sets bit g of p, so
// q(t+1) = q(t) + N/(4G).
template <bool G_OP, int G>
PCUB_HD void level_from_root(const double2* in, long long B, int n, int j, double2* dst, long long ns,
                             const uint32_t* ybase) {
    const int Po = (1 << (n - 2)) / G;  // N/(4G) output pairs
    const long long step = (1LL << (n - 2)) / G;
#pragma unroll 2
    for (int jp = 0; jp < Po; ++jp) {
        const int t = 2 * jp;
        const long long p0 = root_pair<G>(j, t, n);
        const long long p1 = p0 + step;
        const double2 a0 = in[(2 * p0) * B], b0 = in[(2 * p0 + 1) * B];
        const double2 a1 = in[(2 * p1) * B], b1 = in[(2 * p1 + 1) * B];
        double2 o;
        if (G_OP) {
            const uint32_t w = ybase[(long long)(t >> 5) * ns];
            const uint32_t sh = (uint32_t)t & 31u;
            o.x = op_g_raw(a0, b0, (w >> sh) & 1u);
            o.y = op_g_raw(a1, b1, (w >> (sh + 1)) & 1u);
        } else {
            o.x = op_f_raw(a0, b0);
            o.y = op_f_raw(a1, b1);
        }
        dst[(long long)jp * ns] = o;
    }
}

// Final op into registers: v[t] = op(in[t], in[t+S]) for the depth D-1 node of 2S local values.
template <int S, bool G_OP>
PCUB_HD void final_from_scratch(const double2* src, long long ns, double* v, uint32_t ybits) {
#pragma unroll
    for (int jp = 0; jp < S / 2; ++jp) {
        const double2 a = src[(long long)jp * ns];
        const double2 b = src[(long long)(jp + S / 2) * ns];
        if (G_OP) {
            v[2 * jp] = op_g(a.x, b.x, (ybits >> (2 * jp)) & 1u);
            v[2 * jp + 1] = op_g(a.y, b.y, (ybits >> (2 * jp + 1)) & 1u);
        } else {
            v[2 * jp] = op_f(a.x, b.x);
            v[2 * jp + 1] = op_f(a.y, b.y);
        }
    }
}

template <int S, bool G_OP, int G>
PCUB_HD void final_from_root(const double2* in, long long B, int n, int j, double* v, uint32_t ybits) {
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const long long p = root_pair<G>(j, t, n);
        const double2 a = in[(2 * p) * B], b = in[(2 * p + 1) * B];
        v[t] = G_OP ? op_g_raw(a, b, (ybits >> t) & 1u) : op_f_raw(a, b);
    }
}

// Decode codeword `cw` (clamped to a valid index for loads) with lane j of its
// G lanes (`lane` = wave lane id, for the exchanges) in scratch slot `slot`.
// S = virtual register subtree (values per lane) in {8, 16, 32}; requires
// N >= 2*S*G and N >= 32*G.  `store` is false for padding codewords.
template <int S, int G>
PCUB_HD void decode_codeword(const BinArgs& A, long long cw, int j, int lane, long long slot, bool store) {
    static_assert(S == 8 || S == 16 || S == 32, "register subtree must fit one Y word");
    static_assert(G == 1 || G == 2 || G == 4 || G == 8, "lanes per codeword");
    constexpr int s = (S == 8) ? 3 : (S == 16) ? 4 : 5;
    constexpr int g = (G == 1) ? 0 : (G == 2) ? 1 : (G == 4) ? 2 : 3;
    constexpr uint32_t SMASK = (S == 32) ? 0xffffffffu : ((1u << S) - 1u);
    constexpr int SU = S * G;  // real u positions per register subtree (<= 64)
    static_assert(SU <= 64, "u decisions of one subtree must fit 64 bits");
    constexpr uint64_t SUMASK = (SU == 64) ? ~0ull : ((1ull << SU) - 1ull);
    const int n = A.n;
    const int nv = n - g;
    const int Nv = 1 << nv;
    const int D = nv - s;
    const long long ns = A.nslots;
    const long long B = A.B;
    const double2* in = A.xy + cw;
    double2* scr = A.scratch + slot;
    uint32_t* Y = A.ybits + slot;

    uint64_t acc = 0;
    int nacc = 0;
    int infow = 0;

    for (int k = 0; k < (1 << D); ++k) {
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        // depths d0 .. D-1 into scratch
        for (int d = d0; d < D; ++d) {
            const bool gop = (d == d0) && (k != 0);
            const int Po = Nv >> (d + 1);  // output pairs at depth d
            double2* dst = scr + (long long)(Nv / 2 - (Nv >> d)) * ns;
            // minus child of the depth d-1 node: local u range starts at (k >> (D-d+1)) * (Nv >> (d-1))
            const uint32_t* yb = Y + (long long)(((k >> (D - d + 1)) << (nv - d + 1)) >> 5) * ns;
            if (d == 1) {
                if (gop) level_from_root<true, G>(in, B, n, j, dst, ns, yb);
                else level_from_root<false, G>(in, B, n, j, dst, ns, yb);
            } else {
                const double2* src = scr + (long long)(Nv / 2 - (Nv >> (d - 1))) * ns;
                if (gop) level_from_scratch<true>(src, dst, ns, Po, yb);
                else level_from_scratch<false>(src, dst, ns, Po, yb);
            }
        }
        // depth D into registers.  The minus child of the depth D-1 node starts
        // at local bit (k>>1)*2S.
        double v[S];
        const bool gD = (d0 == D) && (k != 0);
        const int mstart = (k >> 1) * 2 * S;
        const uint32_t ybD = gD ? (Y[(long long)(mstart >> 5) * ns] >> (mstart & 31)) : 0u;
        if (D == 1) {
            if (gD) final_from_root<S, true, G>(in, B, n, j, v, ybD);
            else final_from_root<S, false, G>(in, B, n, j, v, ybD);
        } else {
            const double2* src = scr + (long long)(Nv / 2 - (Nv >> (D - 1))) * ns;
            if (gD) final_from_scratch<S, true>(src, ns, v, ybD);
            else final_from_scratch<S, false>(src, ns, v, ybD);
        }
        // frozen bits of real u range [k*SU, (k+1)*SU)
        const int ustart = k * SU;
        const int uw = ustart >> 5, ush = ustart & 31;
        uint64_t fm, fv;
        if constexpr (SU == 64) {
            fm = (uint64_t)A.fmask[uw] | ((uint64_t)A.fmask[uw + 1] << 32);
            fv = (uint64_t)A.fval[uw] | ((uint64_t)A.fval[uw + 1] << 32);
        } else {
            fm = (uint64_t)((A.fmask[uw] >> ush) & (uint32_t)SUMASK);
            fv = (uint64_t)((A.fval[uw] >> ush) & (uint32_t)SUMASK);
        }
        uint64_t ub = 0;
        const uint32_t y = SubV<S, 0, G>::run(v, ub, fm, fv, lane) & SMASK;
        // local encoding bits of virtual subtree k
        const int lstart = k * S;
        uint32_t* yw = Y + (long long)(lstart >> 5) * ns;
        if (S == 32) *yw = y;
        else *yw = ((lstart & 31) == 0 ? 0u : (*yw & ((1u << (lstart & 31)) - 1u))) | (y << (lstart & 31));
        if (A.uout && store && j == 0) {
            uint32_t* uo = A.uout + (long long)uw * B + cw;
            if constexpr (SU == 64) {
                uo[0] = (uint32_t)ub;
                uo[B] = (uint32_t)(ub >> 32);
            } else if constexpr (SU == 32) {
                *uo = (uint32_t)ub;
            } else {
                *uo = (ush == 0 ? 0u : (*uo & ((1u << ush) - 1u))) | ((uint32_t)ub << ush);
            }
        }
        // information bits of this subtree, in u order (identical in all G lanes)
        for (uint64_t im = ~fm & SUMASK; im != 0ull; im &= im - 1ull) {
            const int q = __builtin_ctzll(im);
            acc |= ((ub >> q) & 1ull) << nacc;
            if (++nacc == 32) {
                if (store && (infow & (G - 1)) == j) A.info[(long long)infow * B + cw] = (uint32_t)acc;
                acc = 0;
                nacc = 0;
                ++infow;
            }
        }
        // combine completed plus children upward: parent = [left ^ right | right]
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = Nv >> d;
            if (Lc < 32) {  // parent fits in one word (S < 32, deepest levels)
                const int pstart = (k >> (D - d + 1)) * 2 * Lc;
                uint32_t* pw = Y + (long long)(pstart >> 5) * ns;
                const uint32_t w = *pw >> (pstart & 31);
                const uint32_t lm = (1u << Lc) - 1u;
                *pw ^= ((w >> Lc) & lm) << (pstart & 31);
                continue;
            }
            const int Wc = Lc >> 5;
            uint32_t* base = Y + (long long)((k >> (D - d + 1)) * (2 * Wc)) * ns;
            for (int w = 0; w < Wc; ++w) base[(long long)w * ns] ^= base[(long long)(w + Wc) * ns];
        }
    }
    if (nacc && store && (infow & (G - 1)) == j) A.info[(long long)infow * B + cw] = (uint32_t)acc;
    // x_hat natural segment k = bitrev_g(j) is this lane's local Y, bit-reversed over nv bits
    if (A.xhat && store) {
        const int seg = (int)bitrev((uint32_t)j, g);
        const int W = Nv >> 5;
        for (int w = 0; w < W; ++w) {
            uint32_t o = 0;
            for (int t = 0; t < 32; ++t) {
                const uint32_t p = bitrev((uint32_t)(32 * w + t), nv);
                o |= ((Y[(long long)(p >> 5) * ns] >> (p & 31u)) & 1u) << t;
            }
            A.xhat[(long long)(seg * W + w) * B + cw] = o;
        }
    }
}

// Small codes (N <= 32): everything in registers, one lane per codeword.
template <int NN>
PCUB_HD void decode_small(const BinArgs& A, long long cw, bool store) {
    constexpr int n = (NN <= 1) ? 0 : (NN <= 2) ? 1 : (NN <= 4) ? 2 : (NN <= 8) ? 3 : (NN <= 16) ? 4 : 5;
    const long long B = A.B;
    const double2* in = A.xy + cw;
    const uint64_t fm = A.fmask[0], fv = A.fval[0];
    uint64_t ub = 0;
    uint32_t y;
    if constexpr (NN == 1) {
        // leaf on the raw root: calcMarginalizedProbabilities (:52-69) on an
        // un-normalised pair, decided exactly as the reference does.
        const double2 a = in[0];
        double s = 0.0;
        s += a.x;
        s += a.y;
        uint32_t d = 0;
        if (s > 0.0) d = (a.x / s >= a.y / s) ? 0u : 1u;
        ub = (fm & 1u) ? (fv & 1u) : d;
        y = (uint32_t)ub;
    } else {
        double c[NN / 2];
#pragma unroll
        for (int t = 0; t < NN / 2; ++t) {
            const int p = (int)bitrev((uint32_t)t, n - 1);
            c[t] = op_f_raw(in[(long long)(2 * p) * B], in[(long long)(2 * p + 1) * B]);
        }
        uint32_t ym, yp;
        if constexpr (NN == 2) {
            ym = ((fm & 1u) ? (uint32_t)(fv & 1u) : leaf_v(c[0]));
            ub |= ym;
        } else {
            ym = SubV<NN / 2, 0, 1>::run(c, ub, fm, fv, 0);
        }
#pragma unroll
        for (int t = 0; t < NN / 2; ++t) {
            const int p = (int)bitrev((uint32_t)t, n - 1);
            c[t] = op_g_raw(in[(long long)(2 * p) * B], in[(long long)(2 * p + 1) * B], (ym >> t) & 1u);
        }
        if constexpr (NN == 2) {
            yp = ((fm & 2u) ? (uint32_t)((fv >> 1) & 1u) : leaf_v(c[0]));
            ub |= (uint64_t)yp << 1;
        } else {
            yp = SubV<NN / 2, NN / 2, 1>::run(c, ub, fm, fv, 0);
        }
        y = (ym ^ yp) | (yp << (NN / 2));
    }
    if (!store) return;
    uint32_t acc = 0;
    int nacc = 0;
    const uint32_t valid = (NN == 32) ? 0xffffffffu : ((1u << NN) - 1u);
    for (uint32_t im = ~(uint32_t)fm & valid; im != 0u; im &= im - 1u) {
        acc |= (uint32_t)((ub >> __builtin_ctz(im)) & 1u) << nacc;
        ++nacc;
    }
    if (nacc) A.info[cw] = acc;
    if (A.uout) A.uout[cw] = (uint32_t)ub;
    if (A.xhat) {
        uint32_t x = 0;  // x_hat[i] = y[bitrev_n(i)]
#pragma unroll
        for (int i = 0; i < NN; ++i) x |= ((y >> bitrev((uint32_t)i, n)) & 1u) << i;
        A.xhat[cw] = x;
    }
}

}  // namespace pcub
