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
    const uint8_t* ef;         // [2^D] first rate-0 depth of each subtree's chain (first_frozen_depth)
};

// Rate-0 table.  Register subtree k (real u range [k*SU, (k+1)*SU)) is reached
// by a chain that starts at depth d0(k) = 1 (k = 0) or D - ctz(k).  Returns the
// smallest depth e in [d0, D] whose node on that chain has every u frozen, or
// D + 1.  Such a node is never evaluated: nothing outside it reads it, and the
// reference's decisions inside it are the frozen values.
PCUB_HD bool range_frozen(const uint32_t* fmask, long long a, long long len) {
    if (len < 32) {
        const uint32_t m = ((1u << len) - 1u) << (a & 31);
        return (fmask[a >> 5] & m) == m;
    }
    for (long long w = a >> 5; w < (a + len) >> 5; ++w)
        if (fmask[w] != 0xffffffffu) return false;
    return true;
}

PCUB_HD int first_frozen_depth(const uint32_t* fmask, int k, int D, int SU) {
    const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
    for (int e = d0; e <= D; ++e) {
        const long long sub = 1LL << (D - e);  // register subtrees under a depth-e node
        const long long first = ((long long)k >> (D - e)) << (D - e);
        if (range_frozen(fmask, first * SU, sub * SU)) return e;
    }
    return D + 1;
}

#if defined(__HIP_DEVICE_COMPILE__)
// Exchange with lane ^ MASK.  Inside a row of 16 lanes this is DPP (VALU moves, no
// LDS round trip: the cross-lane leaf chains are serial, so the ds_bpermute latency
// is on the critical path): MASK 1, 2 a quad_perm; MASK 8 the row rotation by 8;
// MASK 4 the rotation by 12 (row_ror:k gives lane i the value of lane i - k mod 16),
// then banks 1 and 3 of the row (lanes 4-7, 12-15) overwritten by the rotation by 4
// (checked on the GPU by tests/emu/dpp_check.hip).  Wider masks use __shfl_xor.  Every caller
// exchanges inside an aligned group of >= 2*MASK lanes that share their control
// flow, so the source lane is always active.
template <int CTRL, int BANKS = 0xF>
PCUB_HD unsigned dpp32(unsigned old, unsigned src) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, 0xF, BANKS, false);
}

template <int MASK>
PCUB_HD unsigned xor_lane32(unsigned x) {
    if constexpr (MASK == 1) return dpp32<0xB1>(0u, x);         // quad_perm [1,0,3,2]
    else if constexpr (MASK == 2) return dpp32<0x4E>(0u, x);    // quad_perm [2,3,0,1]
    else if constexpr (MASK == 8) return dpp32<0x128>(0u, x);   // row_ror:8
    else return dpp32<0x124, 0xA>(dpp32<0x12C>(0u, x), x);      // row_ror:12, banks 1,3: row_ror:4
}

template <int MASK>
PCUB_HD double xor_shfl_c(double v) {
    if constexpr (MASK == 1 || MASK == 2 || MASK == 4 || MASK == 8) {
        const unsigned long long b = (unsigned long long)as_bits(v);
        const unsigned lo = xor_lane32<MASK>((unsigned)b);
        const unsigned hi = xor_lane32<MASK>((unsigned)(b >> 32));
        return from_bits((long long)(((unsigned long long)hi << 32) | lo));
    } else {
        return __shfl_xor(v, MASK);
    }
}
#else
template <int MASK>
PCUB_HD double xor_shfl_c(double v) { return v; }  // host emulation runs G = 1 only
#endif

// A real node of length M (M <= G) with position (lane & (M-1)) held by each lane.
// Returns this lane's bit of the node's (half-split) encoding; ORs the M
// decisions u_UBASE .. u_UBASE+M-1 (identical in all lanes) into ub.
template <int M, int UBASE>
struct XSub {
    static PCUB_HD uint32_t run(double v, uint64_t& ub, uint64_t fm, uint64_t fv, int lane) {
        const double w = xor_shfl_c<M / 2>(v);
        const bool lo = (lane & (M / 2)) == 0;
        const double a = lo ? v : w, b = lo ? w : v;
        if constexpr (M == 2) {
            const uint32_t u0 = ((fm >> UBASE) & 1u) ? (uint32_t)((fv >> UBASE) & 1u) : leaf_f(a, b);
            const uint32_t u1 = ((fm >> (UBASE + 1)) & 1u) ? (uint32_t)((fv >> (UBASE + 1)) & 1u) : leaf_g(a, b, u0);
            ub |= ((uint64_t)u0 << UBASE) | ((uint64_t)u1 << (UBASE + 1));
            return lo ? (u0 ^ u1) : u1;
        } else {
            // a frozen child (wave-uniform test) is not evaluated: its decisions are
            // the frozen values and its encoding their polar transform
            constexpr int H = M / 2;
            constexpr uint64_t HM = (1ull << H) - 1ull;
            const int pos = lane & (H - 1);
            uint32_t ym, yp;
            if (all_frozen<H>(fm, UBASE)) {
                ym = frozen_local<1, H>(fv >> UBASE, pos) & 1u;
                ub |= fv & (HM << UBASE);
            } else {
                ym = XSub<H, UBASE>::run(op_f(a, b), ub, fm, fv, lane);
            }
            if (all_frozen<H>(fm, UBASE + H)) {
                yp = frozen_local<1, H>(fv >> (UBASE + H), pos) & 1u;
                ub |= fv & (HM << (UBASE + H));
            } else {
                yp = XSub<H, UBASE + H>::run(op_g(a, b, ym), ub, fm, fv, lane);
            }
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
            // Rate-0 children (all u frozen; the test is wave-uniform) are skipped:
            // the reference's decisions there are the frozen values whatever the
            // probabilities, so only their re-encoding is needed.
            constexpr int H = L / 2;
            constexpr int HR = H * G;  // real leaves per child
            constexpr uint64_t HM = (HR == 64) ? ~0ull : ((1ull << HR) - 1ull);
            constexpr uint32_t LMASK = (H == 32) ? 0xffffffffu : ((1u << H) - 1u);
            const int j = lane & (G - 1);
            double c[H];
            uint32_t ym, yp;
            if (all_frozen<HR>(fm, BASE_V * G)) {
                ym = frozen_local<H, G>(fv >> (BASE_V * G), j) & LMASK;
                ub |= fv & (HM << (BASE_V * G));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_f(v[t], v[t + H]);
                ym = SubV<H, BASE_V, G>::run(c, ub, fm, fv, lane);
            }
            if (all_frozen<HR>(fm, (BASE_V + H) * G)) {
                yp = frozen_local<H, G>(fv >> ((BASE_V + H) * G), j) & LMASK;
                ub |= fv & (HM << ((BASE_V + H) * G));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_g(v[t], v[t + H], (ym >> t) & 1u);
                yp = SubV<H, BASE_V + H, G>::run(c, ub, fm, fv, lane);
            }
            return (ym ^ yp) | (yp << H);
        }
    }
};

// One stored level of compact values: pair q (positions 2q, 2q+1) at p[q * s].
struct Lvl {
    double2* p;
    long long s;
};

// Source of a fused chain pass: the raw root (depth 0) or a stored level, plus
// the partial sums of the first op's minus child when that op is a plus transform.
struct Chain {
    const double2* in;  // root: this lane's row 2*bitrev_{nv-1}(t) at in[2*bitrev(t)*B] (lane part folded in)
    long long B;
    int nv;             // log2 of the virtual (per-lane) length
    Lvl src;            // compact source level (depth a > 0)
    const uint32_t* Y;  // local re-encoded bits, word w at Y[w * ns]
    long long ns;
    int ystart;         // first local u position of the minus child at depth a+1
};

// Global-memory access helpers.  The per-k pointer laundering (see launder())
// hides the pointers' provenance, so without an explicit address-space cast the
// compiler emits flat instructions (which also tie up the LDS counter).  GL =
// false keeps a generic access (for a level that may live in LDS).  NT = non-
// temporal: the input rows are streamed exactly twice, far apart in time.
#if defined(__HIP_DEVICE_COMPILE__)
typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) d2v gd2v;
typedef __attribute__((address_space(1))) uint32_t gu32;
#endif

template <bool NT = false, bool GL = true>
PCUB_HD double2 ld2(const double2* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (GL) {
        const gd2v* g = (const gd2v*)p;
        const d2v v = NT ? __builtin_nontemporal_load(g) : *g;
        return double2{v.x, v.y};
    }
#endif
    return *p;
}

template <bool NT = false, bool GL = true>
PCUB_HD void st2(double2* p, double2 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (GL) {
        gd2v* g = (gd2v*)p;
        d2v t;
        t.x = v.x;
        t.y = v.y;
        if constexpr (NT) __builtin_nontemporal_store(t, g);
        else *g = t;
        return;
    }
#endif
    *p = v;
}

PCUB_HD uint32_t ldu(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const gu32*)p;
#else
    return *p;
#endif
}

PCUB_HD void stu(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    *(gu32*)p = v;
#else
    *p = v;
#endif
}

// Re-encoded bits (Y): a per-slot global buffer, or (YL) this thread's column of an LDS
// array (word w at Y[w * kBinBlock]): the plus passes read them and every combine rewrites
// them, so in LDS they never travel to L2/HBM.
template <bool YL>
PCUB_HD uint32_t ldy(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (YL) return *(const __attribute__((address_space(3))) uint32_t*)p;
#endif
    return ldu(p);
}

template <bool YL>
PCUB_HD void sty(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (YL) {
        *(__attribute__((address_space(3))) uint32_t*)p = v;
        return;
    }
#endif
    stu(p, v);
}

// Root rows.  Local position t of lane j is real position p = j + G*t < N/2,
// which pairs natural rows (2q, 2q+1) with q = bitrev_{n-1}(p).  The bits of j
// and of G*t are disjoint, so q = bitrev_{n-1}(j) + bitrev_{nv-1}(t): the lane
// part is folded into the lane's root pointer (Chain::in) once, and the row
// offset of a position is wave-uniform.
PCUB_HD long long root_row(int t, int nv) { return (long long)bitrev((uint32_t)t, nv - 1); }

// Makes a per-lane pointer opaque to the optimiser at this point, so addresses
// derived from it are recomputed in the loop (one or two VALU ops) instead of
// being hoisted out of it and held live in registers across the whole schedule.
template <class T>
PCUB_HD T* launder(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(p));
#endif
    return p;
}

// Keeps the scheduler from hoisting the next column's loads above this point
// (bounds the live registers of the unrolled final pass).
PCUB_HD void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}

// Fused column pair.  From the depth-a node (La local values) evaluate F levels
// for the two columns p, p+1 (p even) of stride C = La >> F: level a+e holds
// positions p + m*C, m < 2^(F-e), and needs level a+e-1 at m and m + 2^(F-e).
// The first op is a plus transform when FG (bits of the minus child), else a
// minus transform; every later op is a minus transform (an SC chain descends
// through minus children).  y receives levels a+1 .. a+F back to back
// (2^(F-1), 2^(F-2), .., 1 entries; .x = column p, .y = column p+1).
template <int F, bool FG, int R, int G, bool NS = false, bool GL = true, bool YL = false>
PCUB_HD void colpair(const Chain& c, int p, int C, double2* y) {
    constexpr bool ROOT = R != 0;
    constexpr int H = 1 << (F - 1);
#pragma unroll
    for (int m = 0; m < H; ++m) {
        const int P = p + m * C;
        uint32_t u0 = 0, u1 = 0;
        if (FG) {
            const int bp = c.ystart + P;  // even: bits bp, bp+1 share a word
            const uint32_t w = ldy<YL>(c.Y + (long long)(bp >> 5) * c.ns) >> (bp & 31);
            u0 = w & 1u;
            u1 = (w >> 1) & 1u;
        }
        double2 o;
        if (ROOT) {
            // positions P, P + Nv/2 are rows (2q, 2q+1); P+1 adds Nv/4 to q
            const long long q0 = root_row(P, c.nv);
            const long long q1 = q0 + (1LL << (c.nv - 2));
            const double2 a0 = ld2<R == 2>(c.in + (2 * q0) * c.B);
            const double2 b0 = ld2<R == 2>(c.in + (2 * q0 + 1) * c.B);
            const double2 a1 = ld2<R == 2>(c.in + (2 * q1) * c.B);
            const double2 b1 = ld2<R == 2>(c.in + (2 * q1 + 1) * c.B);
            o.x = FG ? op_g_raw(a0, b0, u0) : op_f_raw(a0, b0);
            o.y = FG ? op_g_raw(a1, b1, u1) : op_f_raw(a1, b1);
        } else {
            const double2 a = ld2<NS, GL>(c.src.p + (long long)(P >> 1) * c.src.s);
            const double2 b = ld2<NS, GL>(c.src.p + (long long)((P + H * C) >> 1) * c.src.s);
            o.x = FG ? op_g(a.x, b.x, u0) : op_f(a.x, b.x);
            o.y = FG ? op_g(a.y, b.y, u1) : op_f(a.y, b.y);
        }
        y[m] = o;
    }
    int in_off = 0, out_off = H;
#pragma unroll
    for (int e = 2; e <= F; ++e) {
        const int He = 1 << (F - e);
#pragma unroll
        for (int m = 0; m < He; ++m) {
            y[out_off + m].x = op_f(y[in_off + m].x, y[in_off + m + He].x);
            y[out_off + m].y = op_f(y[in_off + m].y, y[in_off + m + He].y);
        }
        in_off = out_off;
        out_off += He;
    }
}

// Where stored level d (1 <= d <= D-1) lives: the per-slot scratch, or `last` for d == D-1.
struct LevelMap {
    double2* scr;
    long long ns;
    int Nv;
    int D;
    Lvl last;
    PCUB_HD Lvl get(int d) const {
        if (last.p && d == D - 1) return last;
        return Lvl{scr + (long long)(Nv / 2 - (Nv >> d)) * ns, ns};
    }
};

// Non-final pass: levels a+1 .. a+F are all stored.
template <int F, bool FG, int R, int G, bool NS, bool YL>
PCUB_HD void chain_pass(const Chain& c, int La, const LevelMap& lm, int a) {
    Lvl lv[F];
#pragma unroll
    for (int e = 1; e <= F; ++e) lv[e - 1] = lm.get(a + e);
    const int C = La >> F;
#pragma unroll 1
    for (int p = 0; p < C; p += 2) {
        double2 y[(1 << F) - 1];
        colpair<F, FG, R, G, NS, true, YL>(c, p, C, y);
        int off = 0;
#pragma unroll
        for (int e = 1; e <= F; ++e) {
            const int He = 1 << (F - e);
#pragma unroll
            for (int m = 0; m < He; ++m) st2<NS>(lv[e - 1].p + (long long)((p + m * C) >> 1) * lv[e - 1].s, y[off + m]);
            off += He;
        }
    }
}

// Final pass into registers (F = 1 or 2): with F = 2, level D-1 is stored to
// lv[0]; level D (S values) goes into v.  Level D-1 is touched only by final
// passes (stored here, or read as c.src when F = 1), which lets it live in LDS
// with static addressing.  (A three-level final pass from the root needs more
// than the 168 VGPRs of three waves/SIMD with S = 32 and spills.)
template <int S, int F, bool FG, int R, int G, bool NS, bool LL, bool YL>
PCUB_HD void chain_final(const Chain& c, const Lvl* lv, double* v) {
    static_assert(F == 1 || F == 2, "final pass fuses at most two levels");
#pragma unroll
    for (int p = 0; p < S; p += 2) {
        double2 y[(1 << F) - 1];
        colpair<F, FG, R, G, NS && F == 2, F == 2 || !LL, YL>(c, p, S, y);
        if constexpr (F == 2) {
#pragma unroll
            for (int m = 0; m < 2; ++m) st2<false, !LL>(lv[0].p + (long long)((p + m * S) >> 1) * lv[0].s, y[m]);
        }
        v[p] = y[(1 << F) - 2].x;
        v[p + 1] = y[(1 << F) - 2].y;
        sched_fence();
    }
}

// root: 0 = compact source level, RR = root (1 plain, 2 non-temporal loads)
// NS: non-temporal access to the upper stage levels (all but level D-1)
template <int F, int G, int RR, bool NS, bool YL>
PCUB_HD void dispatch_pass(const Chain& c, int La, const LevelMap& lm, int a, bool fg, bool root) {
    if (root) {
        if (fg) chain_pass<F, true, RR, G, NS, YL>(c, La, lm, a);
        else chain_pass<F, false, RR, G, NS, YL>(c, La, lm, a);
    } else {
        if (fg) chain_pass<F, true, 0, G, NS, YL>(c, La, lm, a);
        else chain_pass<F, false, 0, G, NS, YL>(c, La, lm, a);
    }
}

template <int S, int F, int G, int RR, bool NS, bool LL, bool YL>
PCUB_HD void dispatch_final(const Chain& c, const Lvl* lv, double* v, bool fg, bool root) {
    if (root) {
        if (fg) chain_final<S, F, true, RR, G, NS, LL, YL>(c, lv, v);
        else chain_final<S, F, false, RR, G, NS, LL, YL>(c, lv, v);
    } else {
        if (fg) chain_final<S, F, true, 0, G, NS, LL, YL>(c, lv, v);
        else chain_final<S, F, false, 0, G, NS, LL, YL>(c, lv, v);
    }
}

// Split of a T-level chain into passes.  Each pass reads only its source level,
// and levels halve at every depth, so passes are fused greedily from the top
// (three levels each) and the final pass into registers (one or two levels)
// takes the remainder: T = 3 -> 2 + 1, 4 -> 3 + 1, 5 -> 3 + 2, 6 -> 3 + 2 + 1.
// With the deepest stage level in LDS (stored only by a final pass) the final
// pass is two levels whenever T >= 2.
template <bool LDS>
PCUB_HD int final_levels(int T) {
    if constexpr (LDS) return T >= 2 ? 2 : 1;
    return (T % 3 == 2) ? 2 : 1;
}

// Decode codeword `cw` (clamped to a valid index for loads) with lane j of its
// G lanes (`lane` = wave lane id, for the exchanges) in scratch slot `slot`.
// S = virtual register subtree (values per lane) in {8, 16, 32}; requires
// N >= 2*S*G and N >= 32*G.  `store` is false for padding codewords.
//
// A register subtree's u decisions and frozen bits live in NW 64-bit windows
// (NW = S*G/64 when the subtree has more than 64 real positions): WinTree splits
// the subtree at its top nodes until each part is one window.
template <int L, int G, int NWIN>
struct WinTree {
    static PCUB_HD uint32_t run(const double* v, uint64_t* ub, const uint64_t* fm, const uint64_t* fv, int lane) {
        if constexpr (NWIN == 1) {
            return SubV<L, 0, G>::run(v, ub[0], fm[0], fv[0], lane);
        } else {
            constexpr int H = L / 2;
            constexpr int HW = NWIN / 2;
            double c[H];
            uint32_t ym, yp;
            if (frozen_windows(fm)) {
                ym = WinTree<H, G, HW>::frozen(ub, fv, lane & (G - 1));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_f(v[t], v[t + H]);
                ym = WinTree<H, G, HW>::run(c, ub, fm, fv, lane);
            }
            if (frozen_windows(fm + HW)) {
                yp = WinTree<H, G, HW>::frozen(ub + HW, fv + HW, lane & (G - 1));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_g(v[t], v[t + H], (ym >> t) & 1u);
                yp = WinTree<H, G, HW>::run(c, ub + HW, fm + HW, fv + HW, lane);
            }
            return (ym ^ yp) | (yp << H);
        }
    }

    // NWIN/2 full windows all frozen (the half is rate-0)
    static PCUB_HD bool frozen_windows(const uint64_t* fm) {
        bool all = true;
#pragma unroll
        for (int w = 0; w < NWIN / 2; ++w) all = all && (fm[w] == ~0ull);
        return all;
    }

    // a rate-0 subtree: decisions = frozen values, encoding = their polar transform
    static PCUB_HD uint32_t frozen(uint64_t* ub, const uint64_t* fv, int j) {
        if constexpr (NWIN == 1) {
            constexpr uint64_t WM = (L * G == 64) ? ~0ull : ((1ull << (L * G)) - 1ull);
            ub[0] = fv[0] & WM;
            return frozen_local<L, G>(fv[0], j);
        } else {
            constexpr int H = L / 2;
            const uint32_t ym = WinTree<H, G, NWIN / 2>::frozen(ub, fv, j);
            const uint32_t yp = WinTree<H, G, NWIN / 2>::frozen(ub + NWIN / 2, fv + NWIN / 2, j);
            return (ym ^ yp) | (yp << H);
        }
    }
};

template <int S, int G>
struct SubWin {
    static constexpr int SU = S * G;
    static constexpr int NW = SU > 64 ? SU / 64 : 1;
    static constexpr int SUW = SU > 64 ? 64 : SU;  // bits per window
    static constexpr uint64_t WMASK = (SUW == 64) ? ~0ull : ((1ull << SUW) - 1ull);
    static_assert(SU <= 512, "at most eight windows");

    // decisions of the subtree from its S level-D values
    static PCUB_HD uint32_t run(const double* v, uint64_t* ub, const uint64_t* fm, const uint64_t* fv, int lane) {
        return WinTree<S, G, NW>::run(v, ub, fm, fv, lane);
    }

    static PCUB_HD uint32_t frozen(uint64_t* ub, const uint64_t* fv, int j) { return WinTree<S, G, NW>::frozen(ub, fv, j); }
};

// NT: 0 = cached loads/stores, 1 = non-temporal input rows, 2 = also the upper stage levels
// YL: the re-encoded bits in LDS (ylds = this thread's column, word w at ylds[w * ystride])
template <int S, int G, bool LDS = false, int NT = 0, bool YL = false>
PCUB_HD void decode_codeword(const BinArgs& A, long long cw, int j, int lane, long long slot, bool store,
                             Lvl last = Lvl{nullptr, 0}, uint32_t* ylds = nullptr, long long ystride = 0) {
    static_assert(S == 8 || S == 16 || S == 32, "register subtree must fit one Y word");
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "lanes per codeword");
    constexpr int s = (S == 8) ? 3 : (S == 16) ? 4 : 5;
    constexpr int g = (G == 1) ? 0 : (G == 2) ? 1 : (G == 4) ? 2 : (G == 8) ? 3 : 4;
    constexpr uint32_t SMASK = (S == 32) ? 0xffffffffu : ((1u << S) - 1u);
    constexpr int SU = S * G;  // real u positions per register subtree (<= 128)
    using W = SubWin<S, G>;
    constexpr int NW = W::NW;
    constexpr int RR = NT >= 1 ? 2 : 1;
    constexpr bool NS = NT >= 2;
    const int n = A.n;
    const int nv = n - g;
    const int Nv = 1 << nv;
    const int D = nv - s;
    const long long ns = A.nslots;
    const long long B = A.B;
    const double2* in = A.xy + cw + 2 * (long long)bitrev((uint32_t)j, n - 1) * B;
    double2* scr = A.scratch + slot;
    uint32_t* Y = YL ? ylds : A.ybits + slot;
    const long long ys = YL ? ystride : ns;  // Y word stride

    // stored levels 1 .. D-2 in the slot scratch; level D-1 there too, or in LDS (`last`)
    LevelMap lm;
    lm.scr = scr;
    lm.ns = ns;
    lm.Nv = Nv;
    lm.D = D;
    lm.last = Lvl{nullptr, 0};
    Lvl lastlv;
    if constexpr (LDS) lastlv = last;
    else lastlv = lm.get(D - 1);

    uint64_t acc = 0;
    int nacc = 0;
    int infow = 0;

    for (int k = 0; k < (1 << D); ++k) {
        in = launder(in);
        scr = launder(scr);
        if constexpr (!YL) Y = launder(Y);
        lm.scr = scr;
        if constexpr (!LDS) lastlv = lm.get(D - 1);
        // The chain for subtree k: a plus transform at depth d0-1 (minus for k == 0)
        // then minus transforms down to depth D.  Passes of up to 3 fused levels;
        // the last pass (1 or 2 levels) ends in registers.  Only a pass's source
        // level is read from memory: every level written inside a chain is
        // consumed from registers by the next transform.
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        const int e0 = A.ef[k];  // first rate-0 depth on this chain (D + 1: none)
        int a = d0 - 1;
        bool fg = (k != 0);
        Chain c;
        c.in = in;
        c.B = B;
        c.nv = nv;
        c.Y = Y;
        c.ns = ys;
        // frozen bits of real u range [k*SU, (k+1)*SU), in NW windows
        uint64_t fm[NW], fv[NW], ub[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const int us = k * SU + 64 * w;
            const int uw = us >> 5, ush = us & 31;
            if constexpr (W::SUW == 64) {
                fm[w] = (uint64_t)A.fmask[uw] | ((uint64_t)A.fmask[uw + 1] << 32);
                fv[w] = (uint64_t)A.fval[uw] | ((uint64_t)A.fval[uw + 1] << 32);
            } else {
                fm[w] = (uint64_t)((A.fmask[uw] >> ush) & (uint32_t)W::WMASK);
                fv[w] = (uint64_t)((A.fval[uw] >> ush) & (uint32_t)W::WMASK);
            }
            ub[w] = 0;
        }
        uint32_t y;
        if (e0 <= D - 1) {
            // the chain enters a rate-0 node above the register level: evaluate
            // (and store, for the plus children to come) only depths d0 .. e0-1
            int T = e0 - 1 - a;
            while (T > 0) {
                const int F = T >= 3 ? 3 : T;
                c.src = a > 0 ? lm.get(a) : Lvl{nullptr, 0};
                c.ystart = (k >> (D - a)) << (nv - a);
                const int La = Nv >> a;
                if (F == 3) dispatch_pass<3, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                else if (F == 2) dispatch_pass<2, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                else dispatch_pass<1, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
                a += F;
                T -= F;
                fg = false;
            }
            y = W::frozen(ub, fv, j) & SMASK;
        } else {
        int T = D - a;
        const int Ffin = final_levels<LDS>(T);
        while (T > Ffin) {
            const int F = (T - Ffin) >= 3 ? 3 : (T - Ffin);
            c.src = a > 0 ? lm.get(a) : Lvl{nullptr, 0};
            c.ystart = (k >> (D - a)) << (nv - a);
            const int La = Nv >> a;
            if (F == 3) dispatch_pass<3, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
            else if (F == 2) dispatch_pass<2, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
            else dispatch_pass<1, G, RR, NS, YL>(c, La, lm, a, fg, a == 0);
            a += F;
            T -= F;
            fg = false;
        }
        double v[S];
        c.ystart = (k >> (D - a)) << (nv - a);
        if (Ffin == 2) {
            c.src = a > 0 ? lm.get(a) : Lvl{nullptr, 0};
            dispatch_final<S, 2, G, RR, NS, LDS, YL>(c, &lastlv, v, fg, a == 0);
        } else if (a > 0) {
            c.src = lastlv;
            dispatch_final<S, 1, G, RR, NS, LDS, YL>(c, &lastlv, v, fg, false);
        } else {
            dispatch_final<S, 1, G, RR, NS, LDS, YL>(c, &lastlv, v, fg, true);
        }
        if (e0 == D) {  // the register subtree itself is rate-0 (its level-D values go unused)
            y = W::frozen(ub, fv, j) & SMASK;
        } else {
            y = W::run(v, ub, fm, fv, lane) & SMASK;
        }
        }
        // local encoding bits of virtual subtree k
        const int lstart = k * S;
        uint32_t* yw = Y + (long long)(lstart >> 5) * ys;
        if (S == 32) sty<YL>(yw, y);
        else sty<YL>(yw, ((lstart & 31) == 0 ? 0u : (ldy<YL>(yw) & ((1u << (lstart & 31)) - 1u))) | (y << (lstart & 31)));
        if (A.uout && store && j == 0) {
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const int us = k * SU + 64 * w;
                const int ush = us & 31;
                uint32_t* uo = A.uout + (long long)(us >> 5) * B + cw;
                if constexpr (W::SUW == 64) {
                    uo[0] = (uint32_t)ub[w];
                    uo[B] = (uint32_t)(ub[w] >> 32);
                } else if constexpr (W::SUW == 32) {
                    *uo = (uint32_t)ub[w];
                } else {
                    *uo = (ush == 0 ? 0u : (*uo & ((1u << ush) - 1u))) | ((uint32_t)ub[w] << ush);
                }
            }
        }
        // information bits of this subtree, in u order (identical in all G lanes)
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            for (uint64_t im = ~fm[w] & W::WMASK; im != 0ull; im &= im - 1ull) {
                const int q = __builtin_ctzll(im);
                acc |= ((ub[w] >> q) & 1ull) << nacc;
                if (++nacc == 32) {
                    if (store && (infow & (G - 1)) == j) A.info[(long long)infow * B + cw] = (uint32_t)acc;
                    acc = 0;
                    nacc = 0;
                    ++infow;
                }
            }
        }
        // combine completed plus children upward: parent = [left ^ right | right]
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = Nv >> d;
            if (Lc < 32) {  // parent fits in one word (S < 32, deepest levels)
                const int pstart = (k >> (D - d + 1)) * 2 * Lc;
                uint32_t* pw = Y + (long long)(pstart >> 5) * ys;
                const uint32_t w0 = ldy<YL>(pw);
                const uint32_t w = w0 >> (pstart & 31);
                const uint32_t lm = (1u << Lc) - 1u;
                sty<YL>(pw, w0 ^ (((w >> Lc) & lm) << (pstart & 31)));
                continue;
            }
            const int Wc = Lc >> 5;
            uint32_t* base = Y + (long long)((k >> (D - d + 1)) * (2 * Wc)) * ys;
            for (int w = 0; w < Wc; ++w)
                sty<YL>(base + (long long)w * ys, ldy<YL>(base + (long long)w * ys) ^ ldy<YL>(base + (long long)(w + Wc) * ys));
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
                o |= ((ldy<YL>(Y + (long long)(p >> 5) * ys) >> (p & 31u)) & 1u) << t;
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
