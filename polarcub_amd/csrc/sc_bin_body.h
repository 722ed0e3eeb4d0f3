// sc_bin_body.h -- one-codeword SC decode schedule (binary, uniform prior).
//
// Replaces BinaryPolarEncoderDecoder.recursiveEncodeDecode (decode branch,
// BinaryPolarEncoderDecoder.py:223-325).  One lane decodes one codeword; all
// lanes of a wave run the identical (data-independent) tree schedule, so there
// is no divergence except inside the plus transform's two cases.
//
// Storage ("half-split" = bit-reversed order inside every node).  A node of
// length L keeps its values at positions j = 0..L-1 such that its minus/plus
// children are  out[j] = op(in[j], in[j + L/2]).  The reference pairs rows
// (2h, 2h+1); position j holds row bitrev_L(j), which makes both statements
// the same computation.  The node's re-encoded vector in the same order is
//     y = [ y_minus ^ y_plus | y_plus ]
// (BinaryPolarEncoderDecoder.py:319-323 permuted), so partial sums are combined
// IN PLACE by a word-wise XOR of the left half with the right half, in an
// N-bit array Y indexed by u position.  At the end Y = bitrev_N(x_hat).
//
// Levels: depth d holds N >> d values.  Depth 0 is the input (never
// normalised, never copied).  Depths 1 .. D-1 live in a per-slot scratch
// buffer in HBM (compact f64, two values per 16-byte access, slot-minor so a
// wave's access is one contiguous 1 KiB).  Depth D = log2(N/S) goes straight to
// registers and the S-leaf subtree below it is fully unrolled (Sub<S>).
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
    double2* scratch;          // [(N/2 - S) pairs][nslots]
    uint32_t* ybits;           // [N/32][nslots]
    long long nslots;
};

// op from a level held in scratch (compact values), two outputs per pair.
// Outputs pairs [0, Po) of depth d from the node at depth d-1 (2*Po pairs).
template <bool G>
PCUB_HD void level_from_scratch(const double2* src, double2* dst, long long ns, int Po, const uint32_t* ybase) {
#pragma unroll 2
    for (int jp = 0; jp < Po; ++jp) {
        const double2 a = src[(long long)jp * ns];
        const double2 b = src[(long long)(jp + Po) * ns];
        double2 o;
        if (G) {
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

// op from the raw root (depth 0): half-split position j of the root is natural
// row bitrev_n(j), and (j, j + N/2) are the natural rows (2p, 2p+1), p = bitrev_{n-1}(j).
template <bool G>
PCUB_HD void level_from_root(const double2* in, long long B, int n, double2* dst, long long ns, const uint32_t* ybase) {
    const int Po = 1 << (n - 2);  // N/4 output pairs
#pragma unroll 2
    for (int jp = 0; jp < Po; ++jp) {
        const int j = 2 * jp;
        const long long p0 = bitrev((uint32_t)j, n - 1);
        const long long p1 = p0 + (1LL << (n - 2));  // bitrev(j+1) for even j
        const double2 a0 = in[(2 * p0) * B], b0 = in[(2 * p0 + 1) * B];
        const double2 a1 = in[(2 * p1) * B], b1 = in[(2 * p1 + 1) * B];
        double2 o;
        if (G) {
            const uint32_t w = ybase[(long long)(j >> 5) * ns];
            const uint32_t sh = (uint32_t)j & 31u;
            o.x = op_g_raw(a0, b0, (w >> sh) & 1u);
            o.y = op_g_raw(a1, b1, (w >> (sh + 1)) & 1u);
        } else {
            o.x = op_f_raw(a0, b0);
            o.y = op_f_raw(a1, b1);
        }
        dst[(long long)jp * ns] = o;
    }
}

// Final op into registers: v[j] = op(in[j], in[j+S]) for the depth D-1 node of length 2S.
template <int S, bool G>
PCUB_HD void final_from_scratch(const double2* src, long long ns, double* v, uint32_t ybits) {
#pragma unroll
    for (int jp = 0; jp < S / 2; ++jp) {
        const double2 a = src[(long long)jp * ns];
        const double2 b = src[(long long)(jp + S / 2) * ns];
        if (G) {
            v[2 * jp] = op_g(a.x, b.x, (ybits >> (2 * jp)) & 1u);
            v[2 * jp + 1] = op_g(a.y, b.y, (ybits >> (2 * jp + 1)) & 1u);
        } else {
            v[2 * jp] = op_f(a.x, b.x);
            v[2 * jp + 1] = op_f(a.y, b.y);
        }
    }
}

template <int S, bool G>
PCUB_HD void final_from_root(const double2* in, long long B, int n, double* v, uint32_t ybits) {
#pragma unroll
    for (int j = 0; j < S; ++j) {
        const long long p = bitrev((uint32_t)j, n - 1);
        const double2 a = in[(2 * p) * B], b = in[(2 * p + 1) * B];
        v[j] = G ? op_g_raw(a, b, (ybits >> j) & 1u) : op_f_raw(a, b);
    }
}

// Decode codeword `cw` (clamped to a valid index for loads) in scratch slot `slot`.
// S in {8, 16, 32} (requires N >= 2S).  `store` is false for padding lanes.
template <int S>
PCUB_HD void decode_codeword(const BinArgs& A, long long cw, long long slot, bool store) {
    static_assert(S == 8 || S == 16 || S == 32, "register subtree must fit one Y word");
    constexpr int s = (S == 8) ? 3 : (S == 16) ? 4 : 5;
    constexpr uint32_t SMASK = (S == 32) ? 0xffffffffu : ((1u << S) - 1u);
    const int n = A.n;
    const int N = 1 << n;
    const int D = n - s;
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
            const bool g = (d == d0) && (k != 0);
            const int Po = N >> (d + 1);                      // output pairs at depth d
            double2* dst = scr + (long long)(N / 2 - (N >> d)) * ns;
            // minus child of the depth d-1 node: u range starts at (k >> (D-d+1)) * (N >> (d-1))
            const uint32_t* yb = Y + (long long)(((k >> (D - d + 1)) << (n - d + 1)) >> 5) * ns;
            if (d == 1) {
                if (g) level_from_root<true>(in, B, n, dst, ns, yb);
                else level_from_root<false>(in, B, n, dst, ns, yb);
            } else {
                const double2* src = scr + (long long)(N / 2 - (N >> (d - 1))) * ns;
                if (g) level_from_scratch<true>(src, dst, ns, Po, yb);
                else level_from_scratch<false>(src, dst, ns, Po, yb);
            }
        }
        // depth D into registers.  The minus child of the depth D-1 node
        // starts at u = (k>>1)*2S: word (k>>1)*2S/32, bit offset ((k>>1)*2S)%32.
        double v[S];
        const bool gD = (d0 == D) && (k != 0);
        const int mstart = (k >> 1) * 2 * S;
        const uint32_t ybD = gD ? (Y[(long long)(mstart >> 5) * ns] >> (mstart & 31)) : 0u;
        if (D == 1) {
            if (gD) final_from_root<S, true>(in, B, n, v, ybD);
            else final_from_root<S, false>(in, B, n, v, ybD);
        } else {
            const double2* src = scr + (long long)(N / 2 - (N >> (D - 1))) * ns;
            if (gD) final_from_scratch<S, true>(src, ns, v, ybD);
            else final_from_scratch<S, false>(src, ns, v, ybD);
        }
        const int ustart = k * S;
        const int uw = ustart >> 5, ush = ustart & 31;
        const uint32_t fm = (A.fmask[uw] >> ush) & SMASK, fv = (A.fval[uw] >> ush) & SMASK;
        uint32_t ub = 0;
        const uint32_t y = Sub<S, 0>::run(v, ub, fm, fv);
        uint32_t* yw = Y + (long long)uw * ns;
        if (S == 32) *yw = y;
        else *yw = (ush == 0 ? 0u : (*yw & ((1u << ush) - 1u))) | (y << ush);
        if (A.uout && store) {
            uint32_t* uo = A.uout + (long long)uw * B + cw;
            if (S == 32) *uo = ub;
            else *uo = (ush == 0 ? 0u : (*uo & ((1u << ush) - 1u))) | (ub << ush);
        }
        // information bits of this subtree, in u order
        for (uint32_t im = ~fm & SMASK; im != 0u; im &= im - 1u) {
            const int j = __builtin_ctz(im);
            acc |= (uint64_t)((ub >> j) & 1u) << nacc;
            if (++nacc == 32) {
                if (store) A.info[(long long)infow * B + cw] = (uint32_t)acc;
                acc = 0;
                nacc = 0;
                ++infow;
            }
        }
        // combine completed plus children upward: parent = [left ^ right | right]
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = N >> d;
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
            for (int w = 0; w < Wc; ++w)
                base[(long long)w * ns] ^= base[(long long)(w + Wc) * ns];
        }
    }
    if (nacc && store) A.info[(long long)infow * B + cw] = (uint32_t)acc;
    // x_hat = bitrev_N(Y)
    if (A.xhat && store) {
        for (int w = 0; w < (N >> 5); ++w) {
            uint32_t o = 0;
            for (int t = 0; t < 32; ++t) {
                const uint32_t p = bitrev((uint32_t)(32 * w + t), n);
                o |= ((Y[(long long)(p >> 5) * ns] >> (p & 31u)) & 1u) << t;
            }
            A.xhat[(long long)w * B + cw] = o;
        }
    }
}

// Small codes (N <= 32): everything in registers.
template <int NN>
PCUB_HD void decode_small(const BinArgs& A, long long cw, bool store) {
    constexpr int n = (NN <= 1) ? 0 : (NN <= 2) ? 1 : (NN <= 4) ? 2 : (NN <= 8) ? 3 : (NN <= 16) ? 4 : 5;
    const long long B = A.B;
    const double2* in = A.xy + cw;
    const uint32_t fm = A.fmask[0], fv = A.fval[0];
    uint32_t ub = 0, y;
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
        y = ub;
    } else {
        double c[NN / 2];
#pragma unroll
        for (int j = 0; j < NN / 2; ++j) {
            const int p = (int)bitrev((uint32_t)j, n - 1);
            c[j] = op_f_raw(in[(long long)(2 * p) * B], in[(long long)(2 * p + 1) * B]);
        }
        const uint32_t ym = Sub<NN / 2, 0>::run(c, ub, fm, fv);
#pragma unroll
        for (int j = 0; j < NN / 2; ++j) {
            const int p = (int)bitrev((uint32_t)j, n - 1);
            c[j] = op_g_raw(in[(long long)(2 * p) * B], in[(long long)(2 * p + 1) * B], (ym >> j) & 1u);
        }
        const uint32_t yp = Sub<NN / 2, NN / 2>::run(c, ub, fm, fv);
        y = (ym ^ yp) | (yp << (NN / 2));
    }
    if (!store) return;
    // info bits
    uint32_t acc = 0;
    int nacc = 0;
    const uint32_t valid = (NN == 32) ? 0xffffffffu : ((1u << NN) - 1u);
    for (uint32_t im = ~fm & valid; im != 0u; im &= im - 1u) {
        acc |= ((ub >> __builtin_ctz(im)) & 1u) << nacc;
        ++nacc;
    }
    if (nacc) A.info[cw] = acc;
    if (A.uout) A.uout[cw] = ub;
    if (A.xhat) {
        uint32_t x = 0;  // x_hat[i] = y[bitrev_n(i)]
#pragma unroll
        for (int i = 0; i < NN; ++i) x |= ((y >> bitrev((uint32_t)i, n)) & 1u) << i;
        A.xhat[cw] = x;
    }
}

}  // namespace pcub
