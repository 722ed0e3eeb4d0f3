// sc_bin_sched.h -- the binary SC decode schedule (chain passes, register subtrees,
// decode_codeword); included only by the binary decode kernels (sc_bin_kern.h) and the
// host emulator, so the q-ary / deletion kernels do not rebuild when it changes.
//
// Replaces BinaryPolarEncoderDecoder.recursiveEncodeDecode (decode branch,
// BinaryPolarEncoderDecoder.py:223-325); storage and lane layout: sc_bin_body.h.
#pragma once
#include "sc_bin_body.h"

namespace pcub {

// Fused column pair.  From the depth-a node (La local values) evaluate F levels
// for the two columns p, p+1 (p even) of stride C = La >> F: level a+e holds
// positions p + m*C, m < 2^(F-e), and needs level a+e-1 at m and m + 2^(F-e).
// The first op is a plus transform when FG (bits of the minus child), else a
// minus transform; every later op is a minus transform (an SC chain descends
// through minus children).  y receives levels a+1 .. a+F back to back
// (2^(F-1), 2^(F-2), .., 1 entries; .x = column p, .y = column p+1).
//
// Split into a load stage (ColLoad: the source rows / values and the minus child's
// bits) and a compute stage, so a pass can issue the loads of later columns before it
// computes the current one (software pipelining: the HBM latency of a column is covered by
// the arithmetic of the columns before it instead of by other waves alone).
// R: 0 = a stored compact level, 1 / 2 = the raw root (plain / non-temporal loads), 3 = a
// compact root (normalised rows, one double each: the root transforms are then the compact
// ones, which is the reference's arithmetic on rows (1, r) / (r, 1) exactly).
template <int F, bool FG, int R>
struct ColLoad {
    static constexpr int H = 1 << (F - 1);
    static constexpr int NX = (R == 1 || R == 2) ? 4 * H : 2 * H;  // 16-byte values loaded
    double2 x[NX];
    uint32_t w[FG ? H : 1];  // minus-child bits of column P at bit 0, P+1 at bit 1
};

template <int F, bool FG, int R, bool NS = false, bool GL = true, bool YL = false>
PCUB_HD void col_load(const Chain& c, int p, int C, ColLoad<F, FG, R>& L) {
    constexpr int H = 1 << (F - 1);
#pragma unroll
    for (int m = 0; m < H; ++m) {
        const int P = p + m * C;
        if constexpr (FG) {
            const int bp = c.ystart + P;  // even: bits bp, bp+1 share a word
            L.w[m] = ldy<YL>(c.Y + (long long)(bp >> 5) * c.ns) >> (bp & 31);
        }
        if constexpr (R == 3) {
            // (a, b) of column P at x[2m], of column P+1 at x[2m+1]
            const long long q0 = root_row(P, c.nv);
            const long long q1 = q0 + (1LL << (c.nv - 2));
            L.x[2 * m + 0] = double2{ld1nto(c.inc + (2 * q0) * c.B, c.lin), ld1nto(c.inc + (2 * q0 + 1) * c.B, c.lin)};
            L.x[2 * m + 1] = double2{ld1nto(c.inc + (2 * q1) * c.B, c.lin), ld1nto(c.inc + (2 * q1 + 1) * c.B, c.lin)};
        } else if constexpr (R != 0) {
            // positions P, P + Nv/2 are rows (2q, 2q+1); P+1 adds Nv/4 to q
            const long long q0 = root_row(P, c.nv);
            const long long q1 = q0 + (1LL << (c.nv - 2));
            L.x[4 * m + 0] = ld2o<R == 2>(c.in + (2 * q0) * c.B, c.lin);
            L.x[4 * m + 1] = ld2o<R == 2>(c.in + (2 * q0 + 1) * c.B, c.lin);
            L.x[4 * m + 2] = ld2o<R == 2>(c.in + (2 * q1) * c.B, c.lin);
            L.x[4 * m + 3] = ld2o<R == 2>(c.in + (2 * q1 + 1) * c.B, c.lin);
        } else {
            L.x[2 * m + 0] = ld2<NS, GL>(c.src.p + (long long)(P >> 1) * c.src.s);
            L.x[2 * m + 1] = ld2<NS, GL>(c.src.p + (long long)((P + H * C) >> 1) * c.src.s);
        }
    }
}

template <int F, bool FG, int R>
PCUB_HD void col_compute(const ColLoad<F, FG, R>& L, double2* y) {
    constexpr int H = 1 << (F - 1);
#pragma unroll
    for (int m = 0; m < H; ++m) {
        uint32_t u0 = 0, u1 = 0;
        if constexpr (FG) {
            u0 = L.w[m] & 1u;
            u1 = (L.w[m] >> 1) & 1u;
        }
        double2 o;
        if constexpr (R == 3) {
            const double2 c0 = L.x[2 * m], c1 = L.x[2 * m + 1];
            o.x = FG ? op_g(c0.x, c0.y, u0) : op_f(c0.x, c0.y);
            o.y = FG ? op_g(c1.x, c1.y, u1) : op_f(c1.x, c1.y);
        } else if constexpr (R != 0) {
            const double2 a0 = L.x[4 * m], b0 = L.x[4 * m + 1], a1 = L.x[4 * m + 2], b1 = L.x[4 * m + 3];
            o.x = FG ? op_g_raw(a0, b0, u0) : op_f_raw(a0, b0);
            o.y = FG ? op_g_raw(a1, b1, u1) : op_f_raw(a1, b1);
        } else {
            const double2 a = L.x[2 * m], b = L.x[2 * m + 1];
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

template <int F, bool FG, int R, int G, bool NS = false, bool GL = true, bool YL = false>
PCUB_HD void colpair(const Chain& c, int p, int C, double2* y) {
    ColLoad<F, FG, R> L;
    col_load<F, FG, R, NS, GL, YL>(c, p, C, L);
    col_compute<F, FG, R>(L, y);
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
// PD = prefetch distance in column pairs (the loads of pair p + PD are issued before pair p is
// computed; the loop is fully unrolled, so the PD + 1 load buffers are plain registers).
// PF1 >= 0: the prefetch distance of one-level passes (two 16-byte loads a column pair instead of
// eight for a two-level pass from the root: the same registers keep four times the pairs in flight).
template <int S, int F, bool FG, int R, int G, bool NS, bool LL, bool YL, int HS = 0, int PF = 0, int PF1 = -1>
PCUB_HD void chain_final(const Chain& c, const Lvl* lv, double* v, double* hl) {
    static_assert(F == 1 || F == 2, "final pass fuses at most two levels");
    constexpr int NP = S / 2;  // column pairs
    constexpr int PFF = (F == 1 && PF1 >= 0) ? PF1 : PF;
    constexpr int PD = PFF < NP ? PFF : NP - 1;
    constexpr bool NSF = NS && F == 2;
    constexpr bool GLF = F == 2 || !LL;
    ColLoad<F, FG, R> L[PD + 1];
#pragma unroll
    for (int i = 0; i < PD; ++i) col_load<F, FG, R, NSF, GLF, YL>(c, 2 * i, S, L[i]);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int p = 2 * i;
        if (i + PD < NP) col_load<F, FG, R, NSF, GLF, YL>(c, 2 * (i + PD), S, L[(i + PD) % (PD + 1)]);
        double2 y[(1 << F) - 1];
        col_compute<F, FG, R>(L[i % (PD + 1)], y);
        if constexpr (F == 2) {
#pragma unroll
            for (int m = 0; m < 2; ++m) st2<false, !LL>(lv[0].p + (long long)((p + m * S) >> 1) * lv[0].s, y[m]);
        }
        if (p < HS) {  // compile-time after unrolling: the leading HS values go to this thread's LDS column
            stl(hl + (long long)p * kHlStride, y[(1 << F) - 2].x);
            stl(hl + (long long)(p + 1) * kHlStride, y[(1 << F) - 2].y);
        } else {
            v[p - HS] = y[(1 << F) - 2].x;
            v[p + 1 - HS] = y[(1 << F) - 2].y;
        }
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

template <int S, int F, int G, int RR, bool NS, bool LL, bool YL, int HS = 0, int PF = 0, int PF1 = -1>
PCUB_HD void dispatch_final(const Chain& c, const Lvl* lv, double* v, bool fg, bool root, double* hl = nullptr) {
    if (root) {
        if (fg) chain_final<S, F, true, RR, G, NS, LL, YL, HS, PF, PF1>(c, lv, v, hl);
        else chain_final<S, F, false, RR, G, NS, LL, YL, HS, PF, PF1>(c, lv, v, hl);
    } else {
        if (fg) chain_final<S, F, true, 0, G, NS, LL, YL, HS, PF, PF1>(c, lv, v, hl);
        else chain_final<S, F, false, 0, G, NS, LL, YL, HS, PF, PF1>(c, lv, v, hl);
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

// HL subtree: a virtual node of 2S values per lane, values 0..S-1 in the LDS column hl and
// S..2S-1 in vr; its two S-value children are register subtrees (SubWin<S, G>, NW windows
// each).  Returns the node's 2S local encoding bits.  The top minus/plus transforms read the
// LDS half twice; everything below runs in registers as in the plain variants.
template <int S, int G>
PCUB_HD uint64_t hl_run(const double* hl, const double* vr, uint64_t* ub, const uint64_t* fm, const uint64_t* fv,
                        int lane) {
    using W = SubWin<S, G>;
    constexpr int NW = W::NW;
    static_assert(S * G >= 64, "HL halves are whole 64-bit windows");
    const int j = lane & (G - 1);
    double c[S];
    uint32_t ym, yp;
    bool fz = true;
#pragma unroll
    for (int w = 0; w < NW; ++w) fz = fz && (fm[w] == ~0ull);
    if (fz) {
        ym = W::frozen(ub, fv, j);
    } else {
#pragma unroll
        for (int t = 0; t < S; ++t) c[t] = op_f(ldl(hl + (long long)t * kHlStride), vr[t]);
        ym = W::run(c, ub, fm, fv, lane);
    }
    fz = true;
#pragma unroll
    for (int w = 0; w < NW; ++w) fz = fz && (fm[NW + w] == ~0ull);
    if (fz) {
        yp = W::frozen(ub + NW, fv + NW, j);
    } else {
#pragma unroll
        for (int t = 0; t < S; ++t) c[t] = op_g(ldl(hl + (long long)t * kHlStride), vr[t], (ym >> t) & 1u);
        yp = W::run(c, ub + NW, fm + NW, fv + NW, lane);
    }
    constexpr uint64_t SM = (S == 32) ? 0xffffffffull : ((1ull << S) - 1ull);
    return ((uint64_t)((ym ^ yp) & SM)) | ((uint64_t)(yp & SM) << S);
}

template <int S, int G>
PCUB_HD uint64_t hl_frozen(uint64_t* ub, const uint64_t* fv, int j) {
    using W = SubWin<S, G>;
    constexpr uint64_t SM = (S == 32) ? 0xffffffffull : ((1ull << S) - 1ull);
    const uint32_t ym = W::frozen(ub, fv, j), yp = W::frozen(ub + W::NW, fv + W::NW, j);
    return ((uint64_t)((ym ^ yp) & SM)) | ((uint64_t)(yp & SM) << S);
}

// byte permute (v_perm_b32): result byte i = byte sel_i of the 8-byte value {hi, lo} (0..3: lo)
PCUB_HD uint32_t perm_bytes(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7))) & 0xffu) << (8 * i);
    return r;
#endif
}

// 4x4 byte transpose: out[b] byte k = in[k] byte b (v_perm_b32, eight of them)
PCUB_HD void bytes_t4(const uint32_t* in, uint32_t* out) {
    const uint32_t a0 = perm_bytes(in[1], in[0], 0x05010400u);  // in0.0 in1.0 in0.1 in1.1
    const uint32_t a1 = perm_bytes(in[1], in[0], 0x07030602u);  // in0.2 in1.2 in0.3 in1.3
    const uint32_t a2 = perm_bytes(in[3], in[2], 0x05010400u);
    const uint32_t a3 = perm_bytes(in[3], in[2], 0x07030602u);
    out[0] = perm_bytes(a2, a0, 0x05040100u);
    out[1] = perm_bytes(a2, a0, 0x07060302u);
    out[2] = perm_bytes(a3, a1, 0x05040100u);
    out[3] = perm_bytes(a3, a1, 0x07060302u);
}

// x_hat from a lane's local re-encoded bits: x_hat local word w, bit t is Y bit bitrev_nv(32w + t)
// = Y bit (bitrev5(t) 2^R + bitrev_R(w)), R = nv - 5.  With Z'[t][c] = Y bit (bitrev5(t) 2^R + c)
// (Z = Y as 32 rows of 2^R bits, rows taken in bit-reversed order), word w is column bitrev_R(w)
// of Z' (bit t = Z'[t][c]): a bit-matrix transpose instead of 32 single-bit gathers per word.
// R = 3 (nv = 8): Z's rows are the 32 bytes of Y.  Z' rows 8k .. 8k+7 are byte bitrev2(k) of the Y
// words bitrev3(0..7) = 0,4,2,6,1,5,3,7 (byte transposes of those word groups), an 8x8 bit transpose
// per block makes byte c of block k column c's bits 8k .. 8k+7, and byte transposes gather them.
PCUB_HD void xhat_r3(const uint32_t* y, uint32_t* out) {
    const uint32_t ga[4] = {y[0], y[4], y[2], y[6]}, gb[4] = {y[1], y[5], y[3], y[7]};
    uint32_t la[4], lb[4];
    bytes_t4(ga, la);
    bytes_t4(gb, lb);
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int b = (int)bitrev((uint32_t)k, 2);
        uint64_t x = (uint64_t)la[b] | ((uint64_t)lb[b] << 32);  // byte i = row 8k + i of Z'
        uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
        x ^= t ^ (t << 7);
        t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
        x ^= t ^ (t << 14);
        t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
        x ^= t ^ (t << 28);  // byte c = column c over rows 8k .. 8k+7
        lo[k] = (uint32_t)x;
        hi[k] = (uint32_t)(x >> 32);
    }
    uint32_t col[8];
    bytes_t4(lo, col);
    bytes_t4(hi, col + 4);
#pragma unroll
    for (int w = 0; w < 8; ++w) out[w] = col[(int)bitrev((uint32_t)w, 3)];
}

// R = 5 (nv = 10): Z' rows are the Y words in bit-reversed order (a[r] = Y word bitrev5(r)); a
// 32x32 bit transpose in place.
PCUB_HD void xhat_r5(uint32_t* a, uint32_t* out) {
    constexpr uint32_t M[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int jj = 16 >> s;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if (k & jj) continue;
            const uint32_t t = ((a[k] >> jj) ^ a[k + jj]) & M[s];
            a[k + jj] ^= t;
            a[k] ^= t << jj;
        }
    }
#pragma unroll
    for (int w = 0; w < 32; ++w) out[w] = a[(int)bitrev((uint32_t)w, 5)];
}

// Decode codeword `cw` (clamped to a valid index for loads) with lane j of its
// G lanes (`lane` = wave lane id, for the exchanges) in scratch slot `slot`.
// S = virtual register subtree (values per lane) in {8, 16, 32}; requires
// N >= 2*S*G and N >= 32*G (HL: N >= 4*S*G).  `store` is false for padding codewords.
//
// NT: 0 = cached loads/stores, 1 = non-temporal input rows, 2 = also the upper stage levels
// YL: the re-encoded bits in LDS (ylds = this thread's column, word w at ylds[w * ystride])
// HL: the chain ends at a split level of SR = 2S values per lane (first half in the LDS column
//     hl, second half in registers; hl_run), one stored stage depth fewer than the plain S
// PF: prefetch distance of the final passes (column pairs whose loads are in flight ahead)
template <int S, int G, bool LDS = false, int NT = 0, bool YL = false, bool HL = false, int PF = 0, bool CR = false,
          int PF1 = -1, bool TR = false>
PCUB_HD void decode_codeword(const BinArgs& A, long long cw, int j, int lane, long long slot, bool store,
                             Lvl last = Lvl{nullptr, 0}, uint32_t* ylds = nullptr, long long ystride = 0,
                             double* hl = nullptr) {
    static_assert(S == 8 || S == 16 || S == 32, "register subtree must fit one Y word");
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "lanes per codeword");
    static_assert(!(HL && LDS), "the split level replaces the LDS stage level");
    constexpr int SR = HL ? 2 * S : S;  // values per lane at the chain's last level
    constexpr int s = (SR == 8) ? 3 : (SR == 16) ? 4 : (SR == 32) ? 5 : 6;
    constexpr int g = (G == 1) ? 0 : (G == 2) ? 1 : (G == 4) ? 2 : (G == 8) ? 3 : 4;
    constexpr uint64_t SMASK = (SR == 64) ? ~0ull : ((1ull << SR) - 1ull);
    constexpr int SU = SR * G;  // real u positions per chain-end subtree (<= 256)
    using W = SubWin<SR, G>;   // window geometry (HL: the S-value halves run SubWin<S, G>)
    constexpr int NW = W::NW;
    constexpr int RR = CR ? 3 : NT >= 1 ? 2 : 1;  // root loads (CR: the compact root A.xc)
    constexpr bool NS = NT >= 2;
    const int n = A.n;
    const int nv = n - g;
    const int Nv = 1 << nv;
    const int D = nv - s;
    const long long ns = A.nslots;
    const long long B = A.B;
    const long long rs = root_stride(A);  // root row stride: B ([N][B] rows) or the tile width
    // TR (tiled root, tile = the wave's 64 / G codewords): the wave's tile is one contiguous block,
    // its base wave-uniform (SGPRs) and this lane's rows a 32-bit byte offset into it, so a root load
    // is a global load with an SGPR base and a VGPR offset -- no 64-bit address add in the VALU.
    // Otherwise a per-lane pointer (64-bit adds per load).
    long long tbase, lrow;
    if constexpr (TR) {
        tbase = uniform64((cw / A.tile) * ((long long)A.tile << n));
        lrow = cw % A.tile + 2 * (long long)bitrev((uint32_t)j, n - 1) * rs;
    } else {
        tbase = root_base(A, cw) + 2 * (long long)bitrev((uint32_t)j, n - 1) * rs;
        lrow = 0;
    }
    const double2* in = CR ? nullptr : A.xy + tbase;
    const double* inc = CR ? A.xc + tbase : nullptr;
    const uint32_t lin = (uint32_t)(lrow * (CR ? 8 : 16));
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
    uint32_t acc32 = 0;  // the packed path's accumulator (SUW >= 32)

    for (int k = 0; k < (1 << D); ++k) {
        if constexpr (TR) {
            if constexpr (CR) inc = launder_s(inc);
            else in = launder_s(in);
        } else {
            if constexpr (CR) inc = launder(inc);
            else in = launder(in);
        }
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
        c.inc = inc;
        c.lin = lin;
        c.B = rs;
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
        uint64_t y;
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
            if constexpr (HL) y = hl_frozen<S, G>(ub, fv, j);
            else y = W::frozen(ub, fv, j) & SMASK;
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
        constexpr int HS = HL ? S : 0;  // leading values of the last level that go to LDS
        double v[SR - HS];
        c.ystart = (k >> (D - a)) << (nv - a);
        if (Ffin == 2) {
            c.src = a > 0 ? lm.get(a) : Lvl{nullptr, 0};
            dispatch_final<SR, 2, G, RR, NS, LDS, YL, HS, PF, PF1>(c, &lastlv, v, fg, a == 0, hl);
        } else if (a > 0) {
            c.src = lastlv;
            dispatch_final<SR, 1, G, RR, NS, LDS, YL, HS, PF, PF1>(c, &lastlv, v, fg, false, hl);
        } else {
            dispatch_final<SR, 1, G, RR, NS, LDS, YL, HS, PF, PF1>(c, &lastlv, v, fg, true, hl);
        }
        if constexpr (HL) {
            if (e0 == D) y = hl_frozen<S, G>(ub, fv, j);
            else y = hl_run<S, G>(hl, v, ub, fm, fv, lane);
        } else {
            if (e0 == D) {  // the register subtree itself is rate-0 (its level-D values go unused)
                y = W::frozen(ub, fv, j) & SMASK;
            } else {
                y = W::run(v, ub, fm, fv, lane) & SMASK;
            }
        }
        }
        // local encoding bits of virtual subtree k
        const int lstart = k * SR;
        uint32_t* yw = Y + (long long)(lstart >> 5) * ys;
        if constexpr (SR == 64) {
            sty<YL>(yw, (uint32_t)y);
            sty<YL>(yw + ys, (uint32_t)(y >> 32));
        } else if constexpr (SR == 32) {
            sty<YL>(yw, (uint32_t)y);
        } else {
            sty<YL>(yw, ((lstart & 31) == 0 ? 0u : (ldy<YL>(yw) & ((1u << (lstart & 31)) - 1u))) |
                            ((uint32_t)y << (lstart & 31)));
        }
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
        if constexpr (W::SUW >= 32) {
            // per 32-bit word of the window: the information bits packed by the precomputed compress
            // masks (all-frozen words skipped, all-information words taken whole), then appended
#pragma unroll
            for (int w = 0; w < NW; ++w) {
#pragma unroll
                for (int h = 0; h < W::SUW / 32; ++h) {
                    const uint32_t* cm = A.cmask + (long long)((k * SU + 64 * w) / 32 + h) * 8;
                    const int cnt = (int)cm[5];
                    if (cnt == 0) continue;
                    uint32_t x = (uint32_t)(ub[w] >> (32 * h));
                    if (cnt != 32) x = compress_info(x, cm);
                    acc32 |= x << nacc;
                    if (nacc + cnt >= 32) {
                        if (store && (infow & (G - 1)) == j) A.info[(long long)infow * B + cw] = acc32;
                        acc32 = nacc ? (x >> (32 - nacc)) : 0u;
                        ++infow;
                    }
                    nacc = (nacc + cnt) & 31;
                }
            }
        } else {
            // windows narrower than a word (short codes): bit by bit
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
    if constexpr (W::SUW >= 32) acc = acc32;
    if (nacc && store && (infow & (G - 1)) == j) A.info[(long long)infow * B + cw] = (uint32_t)acc;
    // x_hat natural segment k = bitrev_g(j) is this lane's local Y, bit-reversed over nv bits
    if (A.xhat && store && (nv == 8 || nv == 10)) {
        const int seg = (int)bitrev((uint32_t)j, g);
        // the store pointer advances by B per word and is laundered each time, so the per-word
        // addresses are not hoisted out of the tile loop (they were: 32 spilled 64-bit offsets)
        uint32_t* xo = A.xhat + (long long)seg * (Nv >> 5) * B + cw;
        if (nv == 8) {
            uint32_t yw[8], o[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) yw[w] = ldy<YL>(Y + (long long)w * ys);
            xhat_r3(yw, o);
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                stu(xo, o[w]);
                xo = launder(xo + B);
            }
        } else {
            uint32_t yw[32], o[32];
#pragma unroll
            for (int r = 0; r < 32; ++r) yw[r] = ldy<YL>(Y + (long long)bitrev((uint32_t)r, 5) * ys);
            xhat_r5(yw, o);
#pragma unroll
            for (int w = 0; w < 32; ++w) {
                stu(xo, o[w]);
                xo = launder(xo + B);
            }
        }
    } else if (A.xhat && store) {
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

}  // namespace pcub
