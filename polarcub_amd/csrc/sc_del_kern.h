// sc_del_kern.h -- SC decoding over the deletion channel (collection of binary
// trellises): the kernel template (gfx950).  Instantiated per trellis length in
// sc_del_n*.hip; sc_del.hip owns the C-ABI launcher.
//
// Replaces BinaryPolarEncoderDecoder.decode (BinaryPolarEncoderDecoder.py:71-99,
// recursion :223-325) when the xy vector distribution is the
// CollectionOfBinaryTrellises built by
// buildCollectionOfBinaryTrellises_uniformInput_deletion
// (VectorDistributions/CollectionOfBinaryTrellises.py:106-129) from a received
// word, for a batch of received words.
//
// Geometry.  T = 2^(n-n0) trellises per codeword -> T lanes per codeword (one
// trellis per lane; T <= 256, i.e. at most one workgroup), 256/T codewords per
// 256-thread workgroup.  Lane position p (lane & (T-1)) owns trellis bitrev(p).
// Everything above depth n0 -- the trellis levels -- is lane-local: the plus
// transform of trellis t needs only t's slice of the minus child's re-encoded
// vector (CollectionOfBinaryTrellises.py:58-66), and the re-encoding combine
// (BinaryPolarEncoderDecoder.py:319-323) maps trellis t's slices onto itself.  At
// depth n0 the length-1 trellises collapse to the rows of a memoryless node of
// length T (one compact value per lane, half-split order because lane position p
// owns trellis bitrev(p)), decoded by the binary kernel's machinery:
//   * T <= 32: across the codeword's lanes (XSub<T>, sc_bin_body.h);
//   * T >= 64: the workgroup's 256 collapsed values go through LDS to wave 0, which
//     decodes every codeword of the group at once with 16 lanes per codeword and T/16
//     values per lane (WinTree<T/16, 16, T/64>: the binary kernel's register subtree,
//     lane-local top levels + XSub<16>), and hands back the encoding bits and
//     decisions through LDS.
//
// n0 = 2 without guard-band ones (main_deletion.py's default shape at n = 8) runs on
// the register-resident representation of trellis_n02.h (no per-lane memory at
// all); other shapes keep one trellis per depth (the current SC path) in private
// memory (trellis_body.h), with capacities for up to OC guard-band ones.  The
// schedule is identical in every lane, only trip counts of the small edge loops
// differ.
#pragma once
#include <hip/hip_runtime.h>

#include "polarcub_sc.h"
#include "sc_bin_body.h"
#include "trellis_body.h"
#include "trellis_n02.h"

namespace pcub {

constexpr int kDelBlock = 256;

// Workgroup size of the general kernel for T trellises: 256 threads (256 / T codewords), or one
// codeword of T = 512 / 1024 trellises per workgroup of T threads (main_deletion's n0 = n // 3 at
// n = 13, 14: 2^4-input trellises, T = 2^(n - 4)).
template <int T>
constexpr int del_block() { return T > kDelBlock ? T : kDelBlock; }

struct DelArgs {
    const uint8_t* rx;      // [B][stride] received symbols (0/1)
    const int32_t* rx_len;  // [B]
    long long B;
    int stride;
    int n;
    double pd;
    OnesProbs op;           // guard-band ones and their vertex probabilities
    const uint32_t* fmask;
    const uint32_t* fval;
    uint32_t* info;         // [ceil(K/32)][B] or null
    uint32_t* xhat;         // [ceil(N/32)][B] or null
    const uint32_t* fval_cw;  // [ceil(N/32)][B] per-codeword frozen values (export mode), or null
    double* leaf;           // [N][B] compact normalised leaves (export mode)
    int rw;                 // > 0: words per codeword of the bit-packed received words in LDS
    const double* tab;      // n0 = 2, 3 without ones: the segment-state table (pcub_sc_deletion_build_table), or null
    unsigned long long* gate;     // null, or this launch's status word (a table the kernel rejected, sc_del.hip)
    unsigned long long gate_id;   // the value that marks the status word: this launch's table was rejected
    unsigned long long* wtiles = nullptr;  // k_sc_del_dense: codeword groups from this counter (zeroed per launch)
};

// Segment-state tables (n0 = 2 and 3, pcub_sc_deletion_build_table) start with a header that every
// kernel checks before it reads an entry: a magic word, n0 and pd (bit patterns), then the rows.
// A table built for another n0 or pd, or a buffer that holds no table, is never read as one (one
// uniform scalar load per workgroup; the n0 = 2 and n0 = 3 layouts cannot alias: the header is at
// the same place in both and records n0).
constexpr int kTabHdr = 8;  // doubles before the first row
constexpr unsigned long long kTabMagic = 0x7063756254616232ull;
PCUB_HD bool tab_ok(const double* tab, int n0, double pd) {
    return tab && (unsigned long long)as_bits(tab[0]) == kTabMagic && as_bits(tab[1]) == as_bits((double)n0) &&
           as_bits(tab[2]) == as_bits(pd);
}

// XSub (sc_bin_body.h) for the export mode: no rate-0 node is skipped and the two
// normalised leaves of every M = 2 node are written (by group position 0) at
// leaf[u * B] -- the xy marginals the genie reads (BinaryPolarEncoderDecoder.py:268-273).
template <int M, int UBASE>
struct XSubE {
    __device__ __forceinline__ static uint32_t run(double v, uint64_t& ub, uint64_t fm, uint64_t fv, int lane, double* leaf,
                                   long long B, bool store) {
        const double w = xor_shfl_c<M / 2>(v);
        const bool lo = (lane & (M / 2)) == 0;
        const double a = lo ? v : w, b = lo ? w : v;
        if constexpr (M == 2) {
            const double c0 = op_f(a, b);
            const uint32_t u0 = ((fm >> UBASE) & 1u) ? (uint32_t)((fv >> UBASE) & 1u) : leaf_v(c0);
            const double c1 = op_g(a, b, u0);
            const uint32_t u1 = ((fm >> (UBASE + 1)) & 1u) ? (uint32_t)((fv >> (UBASE + 1)) & 1u) : leaf_v(c1);
            if (store) {
                leaf[(long long)UBASE * B] = c0;
                leaf[(long long)(UBASE + 1) * B] = c1;
            }
            ub |= ((uint64_t)u0 << UBASE) | ((uint64_t)u1 << (UBASE + 1));
            return lo ? (u0 ^ u1) : u1;
        } else {
            constexpr int H = M / 2;
            const uint32_t ym = XSubE<H, UBASE>::run(op_f(a, b), ub, fm, fv, lane, leaf, B, store);
            const uint32_t yp = XSubE<H, UBASE + H>::run(op_g(a, b, ym), ub, fm, fv, lane, leaf, B, store);
            return lo ? (ym ^ yp) : yp;
        }
    }
};

// The wave-0 decode of a collapsed node of T > 64 rows (16 lanes per codeword, T/16
// values per lane): WinTree's split at the top nodes, each 64-position window decoded by
// one out-of-line copy of SubV<4, 0, 16> (the T = 64 decode).  Fully inlined, the node's
// code passes the 16-bit branch range, and LLVM's long branches in a device function go
// through the return-address registers s[30:31] (scripts/check_isa.py guards against it).
struct V4 {
    double v[4];
};

__device__ __attribute__((noinline)) uint32_t del_window(V4 x, uint64_t& ub, uint64_t fm, uint64_t fv, int lane) {
    return SubV<4, 0, 16>::run(x.v, ub, fm, fv, lane);
}

// (bits of L values a lane: 64 at T = 1024)
template <int L, int NWIN>
struct DelWin {
    using Bits = typename std::conditional<(L > 32), uint64_t, uint32_t>::type;
    static __device__ __forceinline__ Bits run(const double* v, uint64_t* ub, const uint64_t* fm,
                                               const uint64_t* fv, int lane) {
        if constexpr (NWIN == 1) {
            static_assert(L == 4, "one window = 4 values x 16 lanes");
            V4 x;
#pragma unroll
            for (int t = 0; t < 4; ++t) x.v[t] = v[t];
            return del_window(x, ub[0], fm[0], fv[0], lane);
        } else {
            constexpr int H = L / 2;
            constexpr int HW = NWIN / 2;
            double c[H];
            uint32_t ym, yp;
            if (WinTree<L, 16, NWIN>::frozen_windows(fm)) {
                ym = WinTree<H, 16, HW>::frozen(ub, fv, lane & 15);
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_f(v[t], v[t + H]);
                ym = DelWin<H, HW>::run(c, ub, fm, fv, lane);
            }
            if (WinTree<L, 16, NWIN>::frozen_windows(fm + HW)) {
                yp = WinTree<H, 16, HW>::frozen(ub + HW, fv + HW, lane & 15);
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_g(v[t], v[t + H], (ym >> t) & 1u);
                yp = DelWin<H, HW>::run(c, ub + HW, fm + HW, fv + HW, lane);
            }
            return (Bits)(ym ^ yp) | ((Bits)yp << H);
        }
    }
};

// Per-lane decoding context: frozen windows, decisions, information accumulator.
template <int T, bool EXP>
struct DelCtx {
    static constexpr int NW = T > 64 ? T / 64 : 1;  // 64-bit windows of a memoryless subtree
    static constexpr int CPB = del_block<T>() / T;  // codewords per workgroup
    static constexpr int GL = 16;                   // wave-0 lanes per codeword (T >= 64)
    static constexpr int LV = T >= 64 ? T / GL : 1;  // values per wave-0 lane (T >= 64)
    DelArgs A;  // by value: taking the kernel argument's address would force it to scratch
    long long cw;
    bool leader;  // group position 0 stores the information words and exported leaves
    int lane;
    int k;        // next memoryless subtree (u range [k*T, (k+1)*T))
    uint32_t acc;
    int nacc;
    int infow;
    // T >= 64, decode mode: exchange buffers in LDS (see subtree())
    double* xv;               // [256] collapsed values, codeword g's at [g*T, (g+1)*T)
    unsigned long long* xb;   // [LV] ballots of the encoding bits, one per local index
    unsigned long long* xub;  // [CPB][NW] decisions per codeword
    // T > 64, export mode: per-codeword SC levels and encodings in LDS (see export_wide())
    double* xe;               // [CPB][2T] node values, depth d at 2T - 2(T >> d)
    uint8_t* xeb;             // [CPB][2T] left-child encodings (depth d at T - 2(T >> d)), then the current one

    // bits [k*T + 64w, ...) of a bit vector whose word i is w[i * stride]
    PCUB_HD uint64_t window(const uint32_t* w, int wi, long long stride = 1) const {
        const int us = k * T + 64 * wi;
        if constexpr (T >= 64) {
            return (uint64_t)w[(us >> 5) * stride] | ((uint64_t)w[((us >> 5) + 1) * stride] << 32);
        } else {
            return (uint64_t)((w[(us >> 5) * stride] >> (us & 31)) & (uint32_t)((1ull << T) - 1ull));
        }
    }

    // SC over the collapsed memoryless node (one compact value per lane); returns
    // this lane's bit of the node's re-encoded vector (natural position = its trellis).
    __device__ __forceinline__ uint32_t subtree(double v) {
        uint64_t fm[NW], fv[NW], ub[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            fm[w] = window(A.fmask, w);
            fv[w] = A.fval_cw ? window(A.fval_cw + cw, w, A.B) : window(A.fval, w);
            ub[w] = 0;
        }
        uint32_t y;
        constexpr uint64_t WM = (T >= 64) ? ~0ull : ((1ull << T) - 1ull);
        bool rate0 = true;
#pragma unroll
        for (int w = 0; w < NW; ++w) rate0 = rate0 && (fm[w] == WM);
        if constexpr (EXP && T > 64) {
            y = export_wide(v, ub, fm, fv);
        } else if constexpr (EXP) {
            y = XSubE<T, 0>::run(v, ub[0], fm[0], fv[0], lane, A.leaf + (long long)k * T * A.B + cw, A.B, leader) & 1u;
        } else if (rate0) {  // rate-0 node: decisions are the frozen values
#pragma unroll
            for (int w = 0; w < NW; ++w) ub[w] = fv[w];
            const int p = threadIdx.x & (T - 1);
            if constexpr (T <= 64) y = frozen_local<1, T>(fv[0], p);
            else y = frozen_bit_wide(fv, p);
        } else if constexpr (T >= 64) {
            // One codeword per wave (or per workgroup) is the trellis stages' layout, but
            // a length-T subtree decoded across all those lanes spends a full wave op on
            // every node.  So the group's collapsed rows go through LDS to wave 0, which
            // decodes them all at once with GL = 16 lanes per codeword, LV = T/16 values
            // per lane (lane j of group c owns positions j + 16t: the binary kernel's
            // register subtree, WinTree<LV, 16, NW>), and hands back the encoding bits and
            // decisions.  With CPB < 4 codewords the other lanes decode a copy and store
            // nothing.  fm / fv are the same for the whole group (per-codeword frozen
            // values exist only in export mode), so every wave takes this branch together.
            const int wv = threadIdx.x >> 6;
            xv[threadIdx.x] = v;
            __syncthreads();
            // (measured at T = 64: wave 0 with four codewords beats two waves with two
            // each, and beats rotating the decoding wave over the group's waves)
            if (wv == 0) {
                const int c = lane / GL, j = lane % GL;
                const int cr = c < CPB ? c : CPB - 1;
                double vv[LV];
#pragma unroll
                for (int t = 0; t < LV; ++t) vv[t] = xv[cr * T + j + GL * t];
                uint64_t ubl[NW];
#pragma unroll
                for (int w = 0; w < NW; ++w) ubl[w] = 0;
                typename DelWin<LV, NW>::Bits bits;
                if constexpr (NW == 1) bits = WinTree<LV, GL, NW>::run(vv, ubl, fm, fv, lane);
                else bits = DelWin<LV, NW>::run(vv, ubl, fm, fv, lane);
#pragma unroll
                for (int t = 0; t < LV; ++t) {
                    const unsigned long long bal = __ballot((bits >> t) & 1u);
                    if (lane == 0) xb[t] = bal;
                }
                if (j == 0 && c < CPB)
#pragma unroll
                    for (int w = 0; w < NW; ++w) xub[c * NW + w] = ubl[w];
            }
            __syncthreads();
            // position p of codeword g is local index p / GL of wave-0 lane g*GL + p % GL
            const int p = threadIdx.x & (T - 1);
            const int g = threadIdx.x / T;
            y = (uint32_t)(xb[p / GL] >> (g * GL + p % GL)) & 1u;
#pragma unroll
            for (int w = 0; w < NW; ++w) ub[w] = xub[g * NW + w];
        } else {
            y = XSub<T, 0>::run(v, ub[0], fm[0], fv[0], lane) & 1u;
        }
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            for (uint64_t im = ~fm[w] & WM; im != 0ull; im &= im - 1ull) {
                acc |= (uint32_t)((ub[w] >> __builtin_ctzll(im)) & 1ull) << nacc;
                if (++nacc == 32) {
                    if (leader && A.info) A.info[(long long)infow * A.B + cw] = acc;
                    acc = 0;
                    nacc = 0;
                    ++infow;
                }
            }
        }
        ++k;
        return y;
    }

    // Export mode over T > 64 collapsed rows (the codeword's lanes span T/64 waves): SC over the
    // node in LDS, level by level across the codeword's lanes with a workgroup barrier per level
    // (every codeword of the group runs the same schedule), no node skipped, every leaf written
    // at leaf[u * B] by the leader (BinaryPolarEncoderDecoder.py:268-273).  Values keep the
    // half-split order of XSub: a node of length M at positions [0, M) has children
    // op(v[p], v[p + M/2]) at [0, M/2), and its encoding is [ym ^ yp | yp].  The genie path,
    // not the throughput path: ~3 barriers per leaf.
    __device__ __forceinline__ uint32_t export_wide(double v, uint64_t* ub, const uint64_t* fm, const uint64_t* fv) {
        constexpr int m = T == 128 ? 7 : 8;
        static_assert(T == 128 || T == 256, "wide export: 128 or 256 trellises");
        const int p = threadIdx.x & (T - 1);
        const int g = threadIdx.x / T;
        double* V = xe + g * 2 * T;
        uint8_t* E = xeb + g * 2 * T;
        uint8_t* C = E + T;
        auto voff = [](int d) { return 2 * T - 2 * (T >> d); };
        auto eoff = [](int d) { return T - 2 * (T >> d); };
        V[p] = v;
        __syncthreads();
#pragma unroll 1
        for (int i = 0; i < T; ++i) {
            const int ds = i == 0 ? 0 : m - 1 - __builtin_ctz((unsigned)i);
#pragma unroll 1
            for (int d = ds; d < m; ++d) {
                const int H = (T >> d) >> 1;
                if (p < H) {
                    const double a = V[voff(d) + p], b = V[voff(d) + p + H];
                    V[voff(d + 1) + p] = (d == ds && i != 0) ? op_g(a, b, E[eoff(d + 1) + p]) : op_f(a, b);
                }
                __syncthreads();
            }
            const double c = V[voff(m)];
            const int wi = i >> 6, bt = i & 63;
            uint64_t fmw = fm[0], fvw = fv[0];
#pragma unroll
            for (int w = 1; w < NW; ++w)
                if (wi == w) {
                    fmw = fm[w];
                    fvw = fv[w];
                }
            const uint32_t u = ((fmw >> bt) & 1ull) ? (uint32_t)((fvw >> bt) & 1ull) : leaf_v(c);
            if (leader) A.leaf[((long long)k * T + i) * A.B + cw] = c;
#pragma unroll
            for (int w = 0; w < NW; ++w)
                if (wi == w) ub[w] |= (uint64_t)u << bt;
            __syncthreads();  // every lane has read the leaf before C / V are rewritten
            if (p == 0) C[0] = (uint8_t)u;
            __syncthreads();
            int d = m;
#pragma unroll 1
            for (; d > 0 && ((i >> (m - d)) & 1); --d) {  // right child finished: combine into the parent
                const int M = T >> d;
                if (p < M) {
                    const uint8_t e = C[p];
                    C[p] = E[eoff(d) + p] ^ e;
                    C[p + M] = e;
                }
                __syncthreads();
            }
            if (d > 0) {  // a left child finished: keep its encoding for its sibling's plus transform
                if (p < (T >> d)) E[eoff(d) + p] = C[p];
                __syncthreads();
            }
        }
        const uint32_t y = C[p];
        __syncthreads();  // C is rewritten by the next node's first leaf
        return y;
    }

    // bit p of the polar transform (re-encoding) of NW*64 known bits fv (rate-0 node, T > 64)
    PCUB_HD uint32_t frozen_bit_wide(const uint64_t* fv, int p) const {
        // the encoding of a node is [enc(left) ^ enc(right) | enc(right)] over its halves:
        // fold the windows from the top
        uint64_t e[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) e[w] = polar_bits(fv[w]);
#pragma unroll
        for (int h = 1; h < NW; h <<= 1)
#pragma unroll
            for (int w = 0; w < NW; ++w)
                if ((w & h) == 0) e[w] ^= e[w + h];
        uint64_t sel = e[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) sel = ((p >> 6) == w) ? e[w] : sel;
        return (uint32_t)((sel >> (p & 63)) & 1ull);
    }
};

// The collapse of a length-2 trellis (CollectionOfBinaryTrellises.py:68-82) into the
// row of the memoryless node: without guard-band ones by trellis_collapse (no child
// built), with ones by building the length-1 child and taking its marginal.
template <int L, int OC, class PT>
PCUB_HD void del_collapse(const PT& t, const uint32_t* dec, int ones, double& m0, double& m1) {
    if constexpr (OC > 0) {
        if (ones > 0) {
            using Cap = DelCap<L, OC>;
            constexpr int d = (L == 2) ? 1 : (L == 4) ? 2 : (L == 8) ? 3 : 4;
            Trel<1, Cap::V, Cap::E(d)> c;
            trellis_transform<2>(t, c, dec);
            trellis_marginal(c, m0, m1);
            return;
        }
    }
    trellis_collapse(t, dec, m0, m1);
}

// One SC node of the trellis levels: trellis `t` of length LEN (this lane's
// slice of the collection).  Returns the node's re-encoded slice, natural order.
template <int L, int T, int LEN, bool EXP, int OC>
struct DelNode {
    template <class PT>
    __device__ __forceinline__ static uint32_t run(const PT& t, DelCtx<T, EXP>& cx) {
        using Cap = DelCap<L, OC>;
        if constexpr (LEN == 2) {
            // children are length-1 trellises collapsed to memoryless rows
            // (CollectionOfBinaryTrellises.py:68-82), then normalised by the decoder
            double m0, m1;
            del_collapse<L, OC>(t, nullptr, cx.A.op.ones, m0, m1);
            const uint32_t xm = cx.subtree(norm_pack(m0, m1));
            del_collapse<L, OC>(t, &xm, cx.A.op.ones, m0, m1);
            const uint32_t xp = cx.subtree(norm_pack(m0, m1));
            return (xm ^ xp) | (xp << 1);
        } else {
            constexpr int H = LEN / 2;
            constexpr int d = (L / H == 2) ? 1 : (L / H == 4) ? 2 : (L / H == 8) ? 3 : 4;  // child depth
            Trel<H, Cap::V, Cap::E(d)> c;
            trellis_transform<LEN>(t, c, nullptr);
            trellis_normalize<H>(c);
            const uint32_t ym = DelNode<L, T, H, EXP, OC>::run(c, cx);
            trellis_transform<LEN>(t, c, &ym);
            trellis_normalize<H>(c);
            const uint32_t yp = DelNode<L, T, H, EXP, OC>::run(c, cx);
            uint32_t x = 0;  // x[2h] = ym[h] ^ yp[h], x[2h+1] = yp[h]
#pragma unroll
            for (int h = 0; h < H; ++h)
                x |= ((((ym ^ yp) >> h) & 1u) << (2 * h)) | (((yp >> h) & 1u) << (2 * h + 1));
            return x;
        }
    }
};

// The top trellis level for n0 >= 3 without guard-band ones: the base trellis is implicit
// (BaseT, trellis_body.h), only its depth-1 children are materialised.
template <int L, int T, bool EXP>
struct DelBase {
    __device__ __forceinline__ static uint32_t run(const BaseT<L>& b, DelCtx<T, EXP>& cx) {
        using Cap = DelCap<L, 0>;
        constexpr int H = L / 2;
        Trel<H, Cap::V, Cap::E(1)> c;
        uint32_t y[2];
#pragma unroll 1
        for (int half = 0; half < 2; ++half) {
            trellis_transform_base<L>(b, c, half ? &y[0] : nullptr);
            trellis_normalize<H>(c);
            y[half] = DelNode<L, T, H, EXP, 0>::run(c, cx);
        }
        const uint32_t ym = y[0], yp = y[1];
        uint32_t x = 0;  // x[2h] = ym[h] ^ yp[h], x[2h+1] = yp[h]
#pragma unroll
        for (int h = 0; h < H; ++h) x |= ((((ym ^ yp) >> h) & 1u) << (2 * h)) | (((yp >> h) & 1u) << (2 * h + 1));
        return x;
    }
};

// n0 = 3 without guard-band ones: as for n0 = 2 (trellis_n02.h), every value a lane hands to the
// memoryless subtree is a function of its segment (m <= 8 received bits y, pd) and of the bits
// the subtree returned before it: the k-th of the walk's 8 values (k = 0..7) depends on the k
// earlier bits, so a segment state holds 1 + 2 + .. + 128 = 255 values, and there are 512 states
// (2^m - 1 + y for m <= 8, and "no edges" for m > 8).  The table (1 MB, global memory: built once
// per pd by pcub_sc_deletion_table, reused by every decode) replays DelBase / DelNode's walk with
// the same functions in the same order, so its entries are the per-lane values bit for bit.
constexpr int kN03States = 512;
constexpr int kN03Row = 256;  // 255 values per state, one pad

PCUB_HD int n03_state(int m, uint32_t y) { return (m >= 0 && m <= 8) ? (1 << m) - 1 + (int)y : kN03States - 1; }

// value k (history hist: the k bits returned before it, bit i = the i-th) of state st
PCUB_HD double n03_table_entry(int st, int k, uint32_t hist, double pd) {
    constexpr int L = 8;
    using Cap = DelCap<L, 0>;
    BaseT<L> b;
    if (st == kN03States - 1) {
        b.m = L + 1;
        b.y = 0;
    } else {
        int m = 0;
        while ((2 << m) <= st + 1) ++m;
        b.m = m;
        b.y = (uint32_t)(st + 1 - (1 << m));
    }
    b.d = L - b.m;
    b.pins = 0.5 * (1.0 - pd);
    b.pdel = 0.5 * pd;
    Trel<4, Cap::V, Cap::E(1)> c1;
    Trel<2, Cap::V, Cap::E(2)> c2;
    int idx = 0;
    uint32_t y1[2] = {0u, 0u};
    for (int half = 0; half < 2; ++half) {  // DelBase: the depth-1 minus child, then the plus child
        trellis_transform_base<L>(b, c1, half ? &y1[0] : nullptr);
        trellis_normalize<4>(c1);
        uint32_t y2[2] = {0u, 0u};
        for (int h2 = 0; h2 < 2; ++h2) {  // DelNode<8, T, 4>: its depth-2 children
            trellis_transform<4>(c1, c2, h2 ? &y2[0] : nullptr);
            trellis_normalize<2>(c2);
            double m0, m1;  // DelNode<8, T, 2>: the two collapses
            del_collapse<L, 0>(c2, nullptr, 0, m0, m1);
            if (idx == k) return norm_pack(m0, m1);
            const uint32_t xm = (hist >> idx++) & 1u;
            del_collapse<L, 0>(c2, &xm, 0, m0, m1);
            if (idx == k) return norm_pack(m0, m1);
            const uint32_t xp = (hist >> idx++) & 1u;
            y2[h2] = (xm ^ xp) | (xp << 1);
        }
        uint32_t x = 0;
        for (int h = 0; h < 2; ++h)
            x |= ((((y2[0] ^ y2[1]) >> h) & 1u) << (2 * h)) | (((y2[1] >> h) & 1u) << (2 * h + 1));
        y1[half] = x;
    }
    return 0.0;  // not reached: k < 8
}

// DelBase's walk through the table: the 8 subtree inputs in order (both candidates for the next
// one are loaded before the subtree call that picks between them, so the gather overlaps it),
// then DelBase / DelNode's re-encoding of the 8 returned bits
template <int T, bool EXP>
__device__ __forceinline__ uint32_t del_n03_tab(const double* tb, DelCtx<T, EXP>& cx) {
    uint32_t hist = 0;
    double v = tb[0];
#pragma unroll 1
    for (int k = 0; k < 8; ++k) {
        double v0 = 0.0, v1 = 0.0;
        if (k < 7) {
            const uint32_t nx = (2u << k) - 1u + hist;
            v0 = tb[nx];
            v1 = tb[nx + (1u << k)];
        }
        const uint32_t b = cx.subtree(v) & 1u;
        hist |= b << k;
        v = b ? v1 : v0;
    }
    uint32_t w[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        uint32_t z[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t b0 = (hist >> (4 * i + 2 * j)) & 1u, b1 = (hist >> (4 * i + 2 * j + 1)) & 1u;
            z[j] = (b0 ^ b1) | (b1 << 1);
        }
        uint32_t x = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) x |= ((((z[0] ^ z[1]) >> h) & 1u) << (2 * h)) | (((z[1] >> h) & 1u) << (2 * h + 1));
        w[i] = x;
    }
    uint32_t x = 0;
#pragma unroll
    for (int h = 0; h < 4; ++h) x |= ((((w[0] ^ w[1]) >> h) & 1u) << (2 * h)) | (((w[1] >> h) & 1u) << (2 * h + 1));
    return x;
}

// n0 = 2: the two trellis levels on the register-resident representation
// (trellis_n02.h); same recursion as DelNode.  Returns the 4-bit re-encoded slice.
// one depth-1 node: minus (dec == nullptr) or plus child of the base trellis
template <int T, bool EXP>
__device__ __forceinline__ uint32_t del_n02_half(const Base02& b, const uint32_t* dec, DelCtx<T, EXP>& cx) {
    Child02 c;
    n02_transform(b, dec, c);
    n02_normalize(c);
    Paths02 q;
    n02_paths(c, q);
    double m0, m1;
    n02_collapse_paths(q, nullptr, m0, m1);
    const uint32_t xm = cx.subtree(norm_pack(m0, m1));
    n02_collapse_paths(q, &xm, m0, m1);
    const uint32_t xp = cx.subtree(norm_pack(m0, m1));
    return (xm ^ xp) | (xp << 1);
}

// del_n02 through the workgroup's state table (trellis_n02.h: n02_table_entry): the same four
// subtree inputs in the same order, looked up instead of rebuilt per lane
template <int T, bool EXP>
__device__ __forceinline__ uint32_t del_n02_tab(const double* tb, DelCtx<T, EXP>& cx) {
    const uint32_t xm = cx.subtree(tb[0]);
    const uint32_t xp = cx.subtree(tb[1 + xm]);
    const uint32_t ym = (xm ^ xp) | (xp << 1);
    const uint32_t xm2 = cx.subtree(tb[3 + ym]);
    const uint32_t xp2 = cx.subtree(tb[7 + 2 * ym + xm2]);
    const uint32_t yp = (xm2 ^ xp2) | (xp2 << 1);
    uint32_t x = 0;  // x[2h] = ym[h] ^ yp[h], x[2h+1] = yp[h]
#pragma unroll
    for (int h = 0; h < 2; ++h) x |= ((((ym ^ yp) >> h) & 1u) << (2 * h)) | (((yp >> h) & 1u) << (2 * h + 1));
    return x;
}

template <int T, bool EXP>
__device__ __forceinline__ uint32_t del_n02(const Base02& b, DelCtx<T, EXP>& cx) {
    const uint32_t ym = del_n02_half(b, nullptr, cx);
    const uint32_t yp = del_n02_half(b, &ym, cx);
    uint32_t x = 0;  // x[2h] = ym[h] ^ yp[h], x[2h+1] = yp[h]
#pragma unroll
    for (int h = 0; h < 2; ++h) x |= ((((ym ^ yp) >> h) & 1u) << (2 * h)) | (((yp >> h) & 1u) << (2 * h + 1));
    return x;
}

// The group's received words, bit-packed into LDS (bit i of word i >> 5 of row gg = symbol i
// is 1): each wave packs whole rows with coalesced byte loads and a ballot per 64 symbols, kPackU
// loads in flight before the first ballot (one dependent HBM round trip per kPackU * 64
// symbols, not per 64).
constexpr int kPackU = 16;

template <int CPB, int BLK = kDelBlock>
__device__ __forceinline__ void pack_rows(const DelArgs& A, long long grp, uint32_t* rxb, int lane) {
    const int nch = (A.rw * 32 + 63) / 64;  // 64-symbol chunks per row
    for (int gg = threadIdx.x >> 6; gg < CPB; gg += BLK / 64) {
        long long cg = grp * CPB + gg;
        cg = cg < A.B ? cg : A.B - 1;
        const uint8_t* row = A.rx + cg * (long long)A.stride;
        int ln = A.rx_len[cg];
        ln = ln < 0 ? 0 : (ln > A.stride ? A.stride : ln);
        for (int c0 = 0; c0 < nch; c0 += kPackU) {
            uint32_t b[kPackU];
#pragma unroll
            for (int u = 0; u < kPackU; ++u) {
                const int i = (c0 + u) * 64 + lane;
                b[u] = i < ln ? (uint32_t)row[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kPackU; ++u) {
                const unsigned long long msk = __ballot(b[u] == 1u);
                const int wi = 2 * (c0 + u) + (lane & 1);
                if (lane < 2 && wi < A.rw) rxb[gg * A.rw + wi] = (uint32_t)(msk >> (32 * lane));
            }
        }
    }
}

template <int N0, int TB, bool EXP, int OC>
__device__ __forceinline__ void del_group(const DelArgs& A, long long grp, uint32_t* xs, const double* n02tab) {
    constexpr int L = 1 << N0;
    constexpr int T = 1 << TB;
    constexpr int BLK = del_block<T>();
    constexpr int CPB = BLK / T;             // codewords per workgroup
    constexpr int NB = T * L;                // code length N
    constexpr int WPC = (NB + 31) / 32;      // x_hat words per codeword
    using Cap = DelCap<L, OC>;
    constexpr bool TAB = N0 == 2 && OC == 0;
    const int lane = threadIdx.x & 63;
    const int p = threadIdx.x & (T - 1);
    const int g = threadIdx.x >> TB;
    const long long cw = grp * CPB + g;
    const bool valid = cw < A.B;
    const long long c = valid ? cw : A.B - 1;  // padding groups decode a duplicate, store nothing
    for (int i = threadIdx.x; i < CPB * WPC; i += BLK) xs[i] = 0;

    // Received words, bit-packed into LDS (rw > 0, the launcher's choice when the
    // group's words fit): each wave packs whole codewords with coalesced byte loads
    // and a ballot per 64 symbols, so the guard-band parse below probes 32 symbols
    // per LDS read instead of walking zero runs one dependent global load at a time.
    extern __shared__ uint32_t rxb[];
    const bool pk = A.rw > 0;
    if (pk) {
        pack_rows<CPB, BLK>(A, grp, rxb, lane);
        __syncthreads();
    }

    const uint8_t* w = A.rx + c * (long long)A.stride;
    const uint32_t* pw = rxb + (pk ? g * A.rw : 0);
    int len = A.rx_len[c];
    len = len < 0 ? 0 : (len > A.stride ? A.stride : len);
    auto bit = [w, pw, pk](int i) { return pk ? (int)((pw[i >> 5] >> (i & 31)) & 1u) : (int)w[i]; };
    const int t = (int)bitrev((uint32_t)p, TB);
    int s, m;
    if (pk) segment_of_packed(pw, len, TB, t, s, m);
    else segment_of(bit, len, TB, t, s, m);

    __shared__ double xv[(T >= 64 && !EXP) ? BLK : 1];
    __shared__ unsigned long long xb[(T >= 64 && !EXP) ? DelCtx<T, EXP>::LV : 1],
        xub[(T >= 64 && !EXP) ? CPB * DelCtx<T, EXP>::NW : 1];
    __shared__ double xe[(T > 64 && EXP) ? 2 * kDelBlock : 1];
    __shared__ uint8_t xeb[(T > 64 && EXP) ? 2 * kDelBlock : 1];
    DelCtx<T, EXP> cx;
    cx.xe = xe;
    cx.xeb = xeb;
    cx.xv = xv;
    cx.xb = xb;
    cx.xub = xub;
    cx.A = A;
    cx.cw = c;  // clamped: padding groups read fval_cw in bounds; stores are leader-only
    cx.leader = valid && p == 0;
    cx.lane = lane;
    cx.k = 0;
    cx.acc = 0;
    cx.nacc = 0;
    cx.infow = 0;
    uint32_t x;
    if constexpr (TAB) {
        // the segment's state indexes the workgroup's table (trellis_n02.h, n02_table_entry)
        uint32_t y = 0;
        if (m <= kN02L)
            for (int i = 0; i < m; ++i) y |= (uint32_t)(bit(s + i) & 1) << i;
        x = del_n02_tab(n02tab + n02_state(m, y) * kN02Row, cx);
    } else if constexpr (N0 == 3 && OC == 0) {
        // the segment-state table, when one was built for this n0 and pd (its header, tab_ok);
        // a wave-uniform branch, the header is a scalar load
        if (tab_ok(A.tab, 3, A.pd)) {
            uint32_t y = 0;
            if (m <= 8)
                for (int i = 0; i < m; ++i) y |= (uint32_t)(bit(s + i) & 1) << i;
            x = del_n03_tab(A.tab + kTabHdr + (long long)n03_state(m, y) * kN03Row, cx);
        } else {
            x = DelBase<L, T, EXP>::run(base_segment<L>(bit, s, m, A.pd), cx);
        }
    } else if constexpr (N0 >= 3 && OC == 0) {
        x = DelBase<L, T, EXP>::run(base_segment<L>(bit, s, m, A.pd), cx);
    } else {
        Trel<L, Cap::V, Cap::E0> base;
        trellis_build<L>(base, bit, s, m, A.pd, A.op);
        x = DelNode<L, T, L, EXP, OC>::run(base, cx);
    }
    if (cx.nacc && cx.leader && A.info) A.info[(long long)cx.infow * A.B + cw] = cx.acc;

    // x_hat: trellis t's slice is natural positions [t*L, (t+1)*L)
    __syncthreads();
    const int pos = t * L;
    atomicOr(&xs[g * WPC + (pos >> 5)], (x & (uint32_t)((1ull << L) - 1ull)) << (pos & 31));
    __syncthreads();
    if (A.xhat && valid)
        for (int i = p; i < WPC; i += T) A.xhat[(long long)i * A.B + cw] = xs[g * WPC + i];
    __syncthreads();  // xs / rxb / exchange buffers are reused by the workgroup's next group
}

template <int N0, int TB, bool EXP, int OC>
__global__ __launch_bounds__(del_block<(1 << TB)>()) void k_sc_del(DelArgs A) {
    constexpr int T = 1 << TB;
    constexpr int BLK = del_block<T>();
    constexpr int CPB = BLK / T;                      // codewords per workgroup
    constexpr int WPC = ((T << N0) + 31) / 32;        // x_hat words per codeword
    static_assert(T <= 1024, "at most one workgroup per codeword");
    static_assert(!EXP || T <= kDelBlock, "export mode: at most 256 trellises");
    constexpr bool TAB = N0 == 2 && OC == 0;  // the n0 = 2 stage through the state table
    __shared__ uint32_t xs[CPB * WPC];
    __shared__ double n02tab[TAB ? kN02States * kN02Row : 1];
    // a gated launch (the fallback behind a table-driven launch, sc_del.hip) runs only when that
    // launch rejected its table
    if (A.gate && *A.gate != A.gate_id) return;
    if constexpr (TAB) {
        // once per workgroup (the launch is persistent: a workgroup strides over codeword groups)
        for (int i = threadIdx.x; i < kN02States * 5; i += BLK)
            n02_table_entry(i / 5, i % 5, A.pd, n02tab + (i / 5) * kN02Row);
        __syncthreads();
    }
    const long long ngrp = (A.B + CPB - 1) / CPB;
    for (long long grp = blockIdx.x; grp < ngrp; grp += gridDim.x)
        del_group<N0, TB, EXP, OC>(A, grp, xs, n02tab);
}

typedef void (*DelKern)(DelArgs);

// the kernel for (n0, n - n0) trellis shape, export mode, guard-band-ones capacity (0 or 3); or
// nullptr.  Defined in sc_del_n<n0>.hip (decode, OC 0), sc_del_n<n0>o.hip (decode, OC 3) and
// sc_del_n<n0>x.hip (export).
#define PCUB_DEL_TABLE(n0)                     \
    DelKern del_kernel_n##n0##_d0(int tb);     \
    DelKern del_kernel_n##n0##_d3(int tb);     \
    DelKern del_kernel_n##n0##_x(int tb, int oc);
PCUB_DEL_TABLE(1)
PCUB_DEL_TABLE(2)
PCUB_DEL_TABLE(3)
PCUB_DEL_TABLE(4)
#undef PCUB_DEL_TABLE
// 512 and 1024 trellises of 2^4 inputs (a workgroup of T threads per codeword; main_deletion's
// n0 = n // 3 at n = 13, 14), decode without ones: sc_del_n4w.hip
DelKern del_kernel_n4_wide(int tb);
// 16-input trellises (n0 = 4) without ones, 64 .. 1024 trellises, decode: one wave a (trellis,
// depth-3 node) task, the trellises in LDS (trellis_wave.h): sc_del_w4.hip
DelKern del_kernel_w4(int tb, int alt = 0);

// Kernel tables, one per translation-unit group (decode without / with guard-band ones, export),
// so the large n0 = 3, 4 instantiations compile in parallel.  T up to 256 (one workgroup) in
// every mode; OC 0 or 3.
template <int N0, bool EXP, int OC>
DelKern del_kernel_t(int tb) {
    switch (tb) {
        case 1: return k_sc_del<N0, 1, EXP, OC>;
        case 2: return k_sc_del<N0, 2, EXP, OC>;
        case 3: return k_sc_del<N0, 3, EXP, OC>;
        case 4: return k_sc_del<N0, 4, EXP, OC>;
        case 5: return k_sc_del<N0, 5, EXP, OC>;
        case 6: return k_sc_del<N0, 6, EXP, OC>;
        case 7: return k_sc_del<N0, 7, EXP, OC>;
        case 8: return k_sc_del<N0, 8, EXP, OC>;
        default: return nullptr;
    }
}

}  // namespace pcub
