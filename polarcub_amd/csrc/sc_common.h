// sc_common.h -- device-side arithmetic shared by the SC kernels (gfx950).
//
// Value representation ("compact normalised pair").  After every minus/plus
// transform the reference max-normalises each pair
// (VectorDistributions/BinaryMemorylessVectorDistribution.py:71-87):
//     t = max(p0, p1); if t == 0: t = 1; p0 /= t; p1 /= t
// so a normalised pair is exactly (1, r), (r, 1) with r = min/max in [0,1], or
// (0, 0).  We store it in ONE binary64:
//     +r   <=> (1, r)
//     -r   <=> (r, 1)        (-0.0 encodes (0, 1); the tie (1,1) may carry either sign)
//     NaN  <=> (0, 0)        (either sign)
// x/x == 1 exactly for finite non-zero x, so the stored form loses nothing.
// (0, 0) is absorbing in both transforms (every product in the output has a
// factor from it), and NaN is absorbing in IEEE arithmetic, so the sentinel
// needs no flag: a (0, 0) that arises inside a transform (0/0 in the
// normalisation) is produced by the division itself, and every decision
// below is a strict comparison, false on NaN, i.e. the reference's decision
// 0 for an all-zero leaf.  No select below may become a min/max instruction
// (those drop NaNs); they are written as compare + select and the library is
// built without fast-math.
//
// Canonical arithmetic.  Swapping the two components of an input flips the
// output of the minus transform (its two sums are the same rounded terms,
// commuted), and flips the plus transform's output when both inputs flip.
// Hence each transform is evaluated on the canonical forms (1, ra), (1, rb)
// and the orientation is tracked with an XOR; every formula below is an exact
// restatement of the reference's rounded operations for the actual pair (see
// DESIGN.md, "Arithmetic contract").  Division is the compiler's IEEE
// correctly-rounded f64 sequence; the library is built with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PCUB_HD __host__ __device__ __forceinline__

namespace pcub {


PCUB_HD long long as_bits(double v) { return __builtin_bit_cast(long long, v); }
PCUB_HD double from_bits(long long b) { return __builtin_bit_cast(double, b); }

struct CV {
    double r;    // ratio in [0,1], NaN for (0, 0)
    uint32_t s;  // orientation: 1 <=> (r, 1)
};

PCUB_HD CV cv_load(double v) {
    CV c;
    c.s = (uint32_t)((unsigned long long)as_bits(v) >> 63);
    c.r = __builtin_fabs(v);
    return c;
}

PCUB_HD double cv_pack(double q, uint32_t s) {
    // q >= +0 (or NaN), so OR-ing the sign bit in is exact negation.
    return from_bits(as_bits(q) | (long long)((unsigned long long)s << 63));
}

// RN(num / den) for the minus transform's normalisation: den = max(1 + ra*rb, ra + rb) in [1, 2]
// (or NaN), num = the min in [0, 2].  The compiler's IEEE sequence without v_div_scale /
// v_div_fixup: those only act near the ends of the exponent range (div_scale: a denominator or
// quotient near overflow/underflow, a numerator below 2^-969; fixup: zero, inf, NaN operands).
// Here den is in [1, 2]; a numerator below 2^-969 needs ra + rb < 2^-969, so ra*rb underflows and
// den = 1 + 0 = 1 exactly, where y = rcp(1) = 1, q = num, r = 0: the exact quotient, which is what
// the scaled sequence returns; num = 0 gives +0; NaN stays NaN.  Elsewhere the two sequences are
// the same operations on the same values (rcp, two Newton steps, q = num*y, r = fma(-den, q, num),
// fma(r, y, q)), bit for bit.
PCUB_HD double div_den12(double num, double den) {
#if defined(__HIP_DEVICE_COMPILE__)
    double y = __builtin_amdgcn_rcp(den);
    double e = __builtin_fma(-den, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-den, y, 1.0);
    y = __builtin_fma(y, e, y);
    const double q = num * y;
    const double r = __builtin_fma(-den, q, num);
    return __builtin_fma(r, y, q);
#else
    return num / den;
#endif
}

// max-normalise an un-normalised pair (p0, p1 >= 0) into compact form;
// (0, 0) gives 0/0 = NaN, the sentinel.
PCUB_HD double norm_pack(double p0, double p1) {
    const bool sw = p1 > p0;
    const double num = sw ? p0 : p1;
    const double den = sw ? p1 : p0;
    return cv_pack(num / den, sw ? 1u : 0u);
}

// high word of a double, and q with its high word replaced: the orientation bookkeeping below works on
// the sign bits in place (v_xor3 / v_and_or on the high words; round 5, 89.6 -> 90.4 M cw/s at C2)
PCUB_HD uint32_t hi32(double v) { return (uint32_t)((unsigned long long)as_bits(v) >> 32); }
PCUB_HD double with_hi(double q, uint32_t hi) {
    return from_bits((long long)(((unsigned long long)hi << 32) | ((unsigned long long)as_bits(q) & 0xffffffffull)));
}

// minus transform (BinaryMemorylessVectorDistribution.py:15-29) + normalise,
// on compact inputs a = row 2h, b = row 2h+1.
//   canonical:  p0 = 1*1 + ra*rb,  p1 = 1*rb + ra*1
// Symmetric in (a, b): every term commutes and the orientation is a.s ^ b.s ^ sw, so the cross-lane
// leaves call it on (own, partner) without selecting which is row 2h.
PCUB_HD double op_f(double va, double vb) {
    const double ar = __builtin_fabs(va), br = __builtin_fabs(vb);
    const double m = ar * br;
    const double p0 = 1.0 + m;
    const double p1 = ar + br;
    const bool sw = p1 > p0;
    const double num = __builtin_fmin(p0, p1);
    const double den = __builtin_fmax(p0, p1);
    const double q = div_den12(num, den);
    const uint32_t hs = (hi32(va) ^ hi32(vb) ^ (sw ? 0x80000000u : 0u)) & 0x80000000u;
    return with_hi(q, hi32(q) | hs);
}

// plus transform (BinaryMemorylessVectorDistribution.py:31-47) + normalise.
// u == 1 swaps a's components.  Same orientation: (1*1, ra*rb) -> (1, ra*rb),
// no division.  Opposite orientation: the pair is (ra, rb) or (rb, ra), whose
// normalised ratio is min/max.  (The if/else stays a branch: when every lane of the wave has the
// same orientation the division is skipped, which a select-based form measured 8 % slower for.)
PCUB_HD double op_g(double va, double vb, uint32_t u) {
    const double ar = __builtin_fabs(va), br = __builtin_fabs(vb);
    const uint32_t sb = hi32(vb) & 0x80000000u;
    double q = ar * br;
    uint32_t s = sb;
    if ((int32_t)(hi32(va) ^ hi32(vb) ^ (u << 31)) < 0) {
        const bool agt = ar > br;
        const double mx = agt ? ar : br;
        const double mn = agt ? br : ar;
        s = sb ^ (agt ? 0u : 0x80000000u);
        q = mn / mx;
    }
    return with_hi(q, hi32(q) | s);
}

// The cross-lane forms: this lane holds v, its partner w, and lo says whether v is the pair's first
// row (a = lo ? v : w, b = lo ? w : v).  The products, sums, min / max and orientation tests are
// symmetric in (a, b), so only single bits are selected by lo, not the doubles (XSub; with the
// symmetric op_f and DPP moves without an old operand, 90.4 -> 92.2 M cw/s at C2).  Same values as
// op_g(a, b, u) / leaf_pair(a, b) bit for bit (a NaN operand may surface as another NaN: either is
// the (0, 0) sentinel).
PCUB_HD double op_g_x(double v, double w, bool lo, uint32_t u) {
    const double vr = __builtin_fabs(v), wr = __builtin_fabs(w);
    const uint32_t sv = hi32(v) & 0x80000000u, sw_ = hi32(w) & 0x80000000u;
    const uint32_t sb = lo ? sw_ : sv;
    double q = vr * wr;
    uint32_t s = sb;
    if ((int32_t)(hi32(v) ^ hi32(w) ^ (u << 31)) < 0) {
        const bool gvw = vr > wr, gwv = wr > vr;
        const bool agt = lo ? gvw : gwv;
        const double mx = gvw ? vr : wr;
        const double mn = gvw ? wr : vr;
        s = sb ^ (agt ? 0u : 0x80000000u);
        q = mn / mx;
    }
    return with_hi(q, hi32(q) | s);
}

PCUB_HD void leaf_pair_x(double v, double w, bool lo, uint32_t& d0, uint32_t& d1u0, uint32_t& d1u1) {
    const double vr = __builtin_fabs(v), wr = __builtin_fabs(w);
    const bool vs = (int32_t)hi32(v) < 0, ws = (int32_t)hi32(w) < 0;
    const double m = vr * wr;
    const double p0 = 1.0 + m;
    const double p1 = vr + wr;
    const bool diff = vs != ws;
    d0 = (diff ? (p0 > p1) : (p1 > p0)) ? 1u : 0u;
    const bool bs = lo ? ws : vs;
    const bool agt = lo ? (vr > wr) : (wr > vr);
    const bool bgt = lo ? (wr > vr) : (vr > wr);
    const uint32_t ds = (bs && (m < 1.0)) ? 1u : 0u;
    const uint32_t dd = (bs ? agt : bgt) ? 1u : 0u;
    d1u0 = diff ? dd : ds;
    d1u1 = diff ? ds : dd;
}

// Leaf pair (a, b) = rows (2h, 2h+1) of a length-2 node: u0's decision (leaf_f) and u1's
// decision (leaf_g) for both values of u0, from one product.
PCUB_HD void leaf_pair(double va, double vb, uint32_t& d0, uint32_t& d1u0, uint32_t& d1u1) {
    const CV a = cv_load(va), b = cv_load(vb);
    const double m = a.r * b.r;
    const double p0 = 1.0 + m;
    const double p1 = a.r + b.r;
    d0 = ((a.s ^ b.s) ? (p0 > p1) : (p1 > p0)) ? 1u : 0u;
    const uint32_t ds = (b.s && (m < 1.0)) ? 1u : 0u;                // same orientation
    const uint32_t dd = (b.s ? (a.r > b.r) : (b.r > a.r)) ? 1u : 0u;  // opposite orientation
    const bool same0 = a.s == b.s;
    d1u0 = same0 ? ds : dd;
    d1u1 = same0 ? dd : ds;
}

// raw (un-normalised) root rows: the root is never normalised by the reference.
PCUB_HD double op_f_raw(double2 a, double2 b) {
    const double p0 = a.x * b.x + a.y * b.y;
    const double p1 = a.x * b.y + a.y * b.x;
    return norm_pack(p0, p1);
}

PCUB_HD double op_g_raw(double2 a, double2 b, uint32_t u) {
    const double p0 = u ? a.y * b.x : a.x * b.x;
    const double p1 = u ? a.x * b.y : a.y * b.y;
    return norm_pack(p0, p1);
}

// Leaf decisions.  The reference normalises the leaf, takes m = p / (p0 + p1)
// and decides 0 iff m0 >= m1 (BinaryPolarEncoderDecoder.py:250-252).  For a
// normalised (1, r) that is always 0; for (r, 1) with r < 1 it is always 1
// (r/s < 1/2 <= 1/s with s = fl(1 + r)); (0,0) gives 0.  So the
// decision is "p1 > p0" of the un-normalised transform output.
PCUB_HD uint32_t leaf_f(double va, double vb) {
    const CV a = cv_load(va), b = cv_load(vb);
    const double m = a.r * b.r;
    const double p0 = 1.0 + m;
    const double p1 = a.r + b.r;
    const bool d = (a.s ^ b.s) ? (p0 > p1) : (p1 > p0);
    return d ? 1u : 0u;
}

PCUB_HD uint32_t leaf_g(double va, double vb, uint32_t u) {
    const CV a = cv_load(va), b = cv_load(vb);
    bool d;
    if ((a.s ^ u) == b.s) {
        d = b.s && (a.r * b.r < 1.0);
    } else {
        // actual pair (x0, x1) = b.s ? (rb, ra) : (ra, rb)
        d = b.s ? (a.r > b.r) : (b.r > a.r);
    }
    return d ? 1u : 0u;
}

// single leaf from a compact value: 1 <=> (r, 1) with r < 1.  (A tie (1,1) may
// be stored as +1.0 or -1.0; both decide 0.)
PCUB_HD uint32_t leaf_v(double v) {
    const CV a = cv_load(v);
    return (a.s && a.r < 1.0) ? 1u : 0u;
}

// Re-encoding of known bits (frozen subtrees).  The half-split encoding of a
// node, y = [y_minus ^ y_plus | y_plus], is the polar transform in natural
// order: y_i = XOR of u_j over all j whose bits include i's.  Up to 64 bits.
PCUB_HD uint64_t polar_bits(uint64_t x) {
    x ^= (x >> 1) & 0x5555555555555555ull;
    x ^= (x >> 2) & 0x3333333333333333ull;
    x ^= (x >> 4) & 0x0F0F0F0F0F0F0F0Full;
    x ^= (x >> 8) & 0x00FF00FF00FF00FFull;
    x ^= (x >> 16) & 0x0000FFFF0000FFFFull;
    x ^= (x >> 32) & 0x00000000FFFFFFFFull;
    return x;
}

// Bits 0, G, 2G, .. of x, packed (the positions one lane of G owns).
template <int G>
PCUB_HD uint64_t gather_stride(uint64_t x) {
    if constexpr (G == 1) {
        return x;
    } else if constexpr (G == 2) {
        x &= 0x5555555555555555ull;
        x = (x | (x >> 1)) & 0x3333333333333333ull;
        x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
        x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
        x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
        return (x | (x >> 16)) & 0x00000000FFFFFFFFull;
    } else if constexpr (G == 4) {
        x &= 0x1111111111111111ull;
        x = (x | (x >> 3)) & 0x0303030303030303ull;
        x = (x | (x >> 6)) & 0x000F000F000F000Full;
        x = (x | (x >> 12)) & 0x000000FF000000FFull;
        return (x | (x >> 24)) & 0x000000000000FFFFull;
    } else if constexpr (G == 8) {
        x &= 0x0101010101010101ull;
        x = (x | (x >> 7)) & 0x0003000300030003ull;
        x = (x | (x >> 14)) & 0x0000000F0000000Full;
        return (x | (x >> 28)) & 0x00000000000000FFull;
    } else if constexpr (G == 16) {
        x &= 0x0001000100010001ull;
        x = (x | (x >> 15)) & 0x0000000300000003ull;
        return (x | (x >> 30)) & 0x000000000000000Full;
    } else if constexpr (G == 32) {
        x &= 0x0000000100000001ull;
        return (x | (x >> 31)) & 0x3ull;
    } else {
        static_assert(G == 64, "lanes per codeword");
        return x & 1ull;
    }
}

// Local encoding bits of a frozen node of LV values per lane spread over G
// lanes (real length LV*G <= 64, known bits fv at bit 0), for lane position j.
template <int LV, int G>
PCUB_HD uint32_t frozen_local(uint64_t fv, int j) {
    constexpr int R = LV * G;
    const uint64_t m = (R == 64) ? ~0ull : ((1ull << R) - 1ull);
    if constexpr (LV == 1) {
        return (uint32_t)((polar_bits(fv & m) >> j) & 1ull);  // one value per lane, any G <= 64
    } else {
        return (uint32_t)gather_stride<G>(polar_bits(fv & m) >> j);
    }
}

template <int R>
PCUB_HD bool all_frozen(uint64_t fm, int base) {
    constexpr uint64_t m = (R == 64) ? ~0ull : ((1ull << R) - 1ull);
    return ((fm >> base) & m) == m;
}

PCUB_HD uint32_t bitrev(uint32_t x, int nbits) {
    return nbits == 0 ? 0u : (__builtin_bitreverse32(x) >> (32 - nbits));
}

// Register-resident subtree of length L (compile-time), half-split storage:
// children are f/g of (v[j], v[j + L/2]); the encoding of the node is
// [ym ^ yp | yp] (bit j of the result = encoded bit at half-split position j).
// u decisions for leaf BASE+i are OR-ed into ub bit BASE+i.
template <int L, int BASE>
struct Sub {
    static PCUB_HD uint32_t run(const double* v, uint32_t& ub, uint32_t fm, uint32_t fv) {
        double c[L / 2];
#pragma unroll
        for (int j = 0; j < L / 2; ++j) c[j] = op_f(v[j], v[j + L / 2]);
        const uint32_t ym = Sub<L / 2, BASE>::run(c, ub, fm, fv);
#pragma unroll
        for (int j = 0; j < L / 2; ++j) c[j] = op_g(v[j], v[j + L / 2], (ym >> j) & 1u);
        const uint32_t yp = Sub<L / 2, BASE + L / 2>::run(c, ub, fm, fv);
        return (ym ^ yp) | (yp << (L / 2));
    }
};

template <int BASE>
struct Sub<2, BASE> {
    static PCUB_HD uint32_t run(const double* v, uint32_t& ub, uint32_t fm, uint32_t fv) {
        const uint32_t fz0 = (fm >> BASE) & 1u, fz1 = (fm >> (BASE + 1)) & 1u;
        const uint32_t u0 = fz0 ? ((fv >> BASE) & 1u) : leaf_f(v[0], v[1]);
        const uint32_t u1 = fz1 ? ((fv >> (BASE + 1)) & 1u) : leaf_g(v[0], v[1], u0);
        ub |= (u0 << BASE) | (u1 << (BASE + 1));
        return (u0 ^ u1) | (u1 << 1);
    }
};

template <int BASE>
struct Sub<1, BASE> {
    static PCUB_HD uint32_t run(const double* v, uint32_t& ub, uint32_t fm, uint32_t fv) {
        const uint32_t u0 = ((fm >> BASE) & 1u) ? ((fv >> BASE) & 1u) : leaf_v(v[0]);
        ub |= u0 << BASE;
        return u0;
    }
};

}  // namespace pcub
