// sc_del.hip -- SC decoding over the deletion channel (collection of binary
// trellises), gfx950, + its C-ABI launcher.
//
// pcub_sc_decode_deletion replaces BinaryPolarEncoderDecoder.decode
// (BinaryPolarEncoderDecoder.py:71-99, recursion :223-325) when the xy vector
// distribution is the CollectionOfBinaryTrellises built by
// buildCollectionOfBinaryTrellises_uniformInput_deletion
// (VectorDistributions/CollectionOfBinaryTrellises.py:106-129) from a received
// word, for a batch of received words.
//
// Geometry.  T = 2^(n-n0) trellises per codeword -> T lanes per codeword (one
// trellis per lane), 256/T codewords per 256-thread workgroup.  Lane position p
// (lane & (T-1)) owns trellis bitrev(p): the collapsed memoryless node of length
// T is then held in half-split order, one value per lane, and its SC subtree is
// XSub<T> from sc_bin_body.h (cross-lane butterflies with __shfl_xor, the same
// compact-pair arithmetic as the memoryless kernel).  Everything above it -- the
// n0 trellis levels -- is lane-local: the plus transform of trellis t needs only
// t's slice of the minus child's re-encoded vector
// (CollectionOfBinaryTrellises.py:58-66), and the re-encoding combine
// (BinaryPolarEncoderDecoder.py:319-323) maps trellis t's slices onto itself.
//
// n0 = 2 (main_deletion.py's default shape at n = 8) runs on the register-resident
// representation of trellis_n02.h (no per-lane memory at all); other n0 keep one
// trellis per depth (the current SC path) in private memory (trellis_body.h).  The
// schedule is identical in every lane, only trip counts of the small edge loops
// differ.  Received words are read straight from HBM (u8, row per
// codeword, a few hundred bytes each, L1/L2-resident while a group works on them).
#include <hip/hip_runtime.h>

#include "polarcub_sc.h"
#include "sc_bin_body.h"
#include "trellis_body.h"
#include "trellis_n02.h"

using namespace pcub;

namespace {

constexpr int kBlock = 256;

struct DelArgs {
    const uint8_t* rx;      // [B][stride] received symbols (0/1)
    const int32_t* rx_len;  // [B]
    long long B;
    int stride;
    int n;
    double pd;
    const uint32_t* fmask;
    const uint32_t* fval;
    uint32_t* info;         // [ceil(K/32)][B] or null
    uint32_t* xhat;         // [ceil(N/32)][B] or null
    const uint32_t* fval_cw;  // [ceil(N/32)][B] per-codeword frozen values (export mode), or null
    double* leaf;           // [N][B] compact normalised leaves (export mode)
    int rw;                 // > 0: words per codeword of the bit-packed received words in LDS
};

// XSub (sc_bin_body.h) for the export mode: no rate-0 node is skipped and the two
// normalised leaves of every M = 2 node are written (by group position 0) at
// leaf[u * B] -- the xy marginals the genie reads (BinaryPolarEncoderDecoder.py:268-273).
template <int M, int UBASE>
struct XSubE {
    __device__ static uint32_t run(double v, uint64_t& ub, uint64_t fm, uint64_t fv, int lane, double* leaf,
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

// Per-lane decoding context: frozen windows, decisions, information accumulator.
template <int T, bool EXP>
struct DelCtx {
    DelArgs A;  // by value: taking the kernel argument's address would force it to scratch
    long long cw;
    bool leader;  // group position 0 stores the information words and exported leaves
    int lane;
    int k;        // next memoryless subtree (u range [k*T, (k+1)*T))
    uint32_t acc;
    int nacc;
    int infow;
    // T == 64, decode mode: the group's memoryless subtrees are decoded by wave 0 with
    // 16 lanes per codeword (see subtree()); exchange buffers in LDS
    double* xv;               // [4][64] collapsed values, one row per wave (= codeword)
    unsigned long long* xb;   // [4] ballots of the encoding bits, one per local index
    unsigned long long* xub;  // [4] decisions per codeword

    // bits [k*T, (k+1)*T) of a bit vector whose word i is w[i * stride]
    PCUB_HD uint64_t window(const uint32_t* w, long long stride = 1) const {
        const int us = k * T;
        if constexpr (T == 64) {
            return (uint64_t)w[(us >> 5) * stride] | ((uint64_t)w[((us >> 5) + 1) * stride] << 32);
        } else {
            return (uint64_t)((w[(us >> 5) * stride] >> (us & 31)) & (uint32_t)((1ull << T) - 1ull));
        }
    }

    // SC over the collapsed memoryless node (one compact value per lane); returns
    // this lane's bit of the node's re-encoded vector (natural position = its trellis).
    __device__ __forceinline__ uint32_t subtree(double v) {
        const uint64_t fm = window(A.fmask);
        const uint64_t fv = A.fval_cw ? window(A.fval_cw + cw, A.B) : window(A.fval);
        uint64_t ub = 0;
        uint32_t y;
        constexpr uint64_t WM = (T == 64) ? ~0ull : ((1ull << T) - 1ull);
        if constexpr (EXP) {
            y = XSubE<T, 0>::run(v, ub, fm, fv, lane, A.leaf + (long long)k * T * A.B + cw, A.B, leader) & 1u;
        } else if (fm == WM) {  // rate-0 node: decisions are the frozen values
            ub = fv;
            y = frozen_local<1, T>(fv, lane & (T - 1));
        } else if constexpr (T == 64) {
            // One codeword per wave is the trellis stages' layout, but a length-64
            // subtree decoded across one wave's lanes (XSub<64>) spends a full wave op
            // on every node.  So the four codewords' collapsed rows go through LDS to
            // one wave, which decodes all four at once with 16 lanes per codeword (lane
            // j of group c owns positions j + 16t, SubV<4, 0, 16>: the binary
            // kernel's schedule), and hands back the encoding bits and decisions.
            // fm / fv are the same for the whole group (per-codeword frozen values
            // exist only in export mode), so every wave takes this branch together.
            const int wv = threadIdx.x >> 6;
            xv[wv * 64 + lane] = v;
            __syncthreads();
            // (measured: wave 0 with four codewords beats two waves with two each, and
            // beats rotating the decoding wave over the group's waves)
            if (wv == 0) {
                const int c = lane >> 4, j = lane & 15;
                double vv[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) vv[t] = xv[c * 64 + j + 16 * t];
                uint64_t ubl = 0;
                const uint32_t bits = SubV<4, 0, 16>::run(vv, ubl, fm, fv, lane);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const unsigned long long bal = __ballot((bits >> t) & 1u);
                    if (lane == 0) xb[t] = bal;
                }
                if (j == 0) xub[c] = ubl;
            }
            __syncthreads();
            // position p = lane is local index p >> 4 of lane (wv * 16 + (p & 15))
            y = (uint32_t)(xb[lane >> 4] >> (wv * 16 + (lane & 15))) & 1u;
            ub = xub[wv];
        } else {
            y = XSub<T, 0>::run(v, ub, fm, fv, lane) & 1u;
        }
        for (uint64_t im = ~fm & WM; im != 0ull; im &= im - 1ull) {
            acc |= (uint32_t)((ub >> __builtin_ctzll(im)) & 1ull) << nacc;
            if (++nacc == 32) {
                if (leader && A.info) A.info[(long long)infow * A.B + cw] = acc;
                acc = 0;
                nacc = 0;
                ++infow;
            }
        }
        ++k;
        return y;
    }
};

template <int L>
struct DelCap {
    static constexpr int V = L / 2 + 1;
    static constexpr int E0 = 3 * V;      // base edge layer
    static constexpr int E1 = 2 * V * V;  // transformed edge layer
};

// One SC node of the trellis levels: trellis `t` of length LEN (this lane's
// slice of the collection).  Returns the node's re-encoded slice, natural order.
template <int L, int T, int LEN, bool EXP>
struct DelNode {
    template <class PT>
    __device__ static uint32_t run(const PT& t, DelCtx<T, EXP>& cx) {
        using Cap = DelCap<L>;
        if constexpr (LEN == 2) {
            // children are length-1 trellises collapsed to memoryless rows
            // (CollectionOfBinaryTrellises.py:68-82), then normalised by the decoder;
            // the collapse marginal is accumulated without building the child
            double m0, m1;
            trellis_collapse(t, nullptr, m0, m1);
            const uint32_t xm = cx.subtree(norm_pack(m0, m1));
            trellis_collapse(t, &xm, m0, m1);
            const uint32_t xp = cx.subtree(norm_pack(m0, m1));
            return (xm ^ xp) | (xp << 1);
        } else {
            constexpr int H = LEN / 2;
            Trel<H, Cap::V, Cap::E1> c;
            trellis_transform<LEN>(t, c, nullptr);
            trellis_normalize<H>(c);
            const uint32_t ym = DelNode<L, T, H, EXP>::run(c, cx);
            trellis_transform<LEN>(t, c, &ym);
            trellis_normalize<H>(c);
            const uint32_t yp = DelNode<L, T, H, EXP>::run(c, cx);
            uint32_t x = 0;  // x[2h] = ym[h] ^ yp[h], x[2h+1] = yp[h]
#pragma unroll
            for (int h = 0; h < H; ++h)
                x |= ((((ym ^ yp) >> h) & 1u) << (2 * h)) | (((yp >> h) & 1u) << (2 * h + 1));
            return x;
        }
    }
};

// n0 = 2: the two trellis levels on the register-resident representation
// (trellis_n02.h); same recursion as DelNode.  Returns the 4-bit re-encoded slice.
// one depth-1 node: minus (dec == nullptr) or plus child of the base trellis
template <int T, bool EXP>
__device__ __forceinline__ uint32_t del_n02_half(const Base02& b, const uint32_t* dec, DelCtx<T, EXP>& cx) {
    Child02 c;
    n02_transform(b, dec, c);
    n02_normalize(c);
    double m0, m1;
    n02_collapse(c, nullptr, m0, m1);
    const uint32_t xm = cx.subtree(norm_pack(m0, m1));
    n02_collapse(c, &xm, m0, m1);
    const uint32_t xp = cx.subtree(norm_pack(m0, m1));
    return (xm ^ xp) | (xp << 1);
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

template <int N0, int TB, bool EXP>
__global__ __launch_bounds__(kBlock) void k_sc_del(DelArgs A) {
    constexpr int L = 1 << N0;
    constexpr int T = 1 << TB;
    constexpr int CPB = kBlock / T;          // codewords per workgroup
    constexpr int NB = T * L;                // code length N
    constexpr int WPC = (NB + 31) / 32;      // x_hat words per codeword
    using Cap = DelCap<L>;
    __shared__ uint32_t xs[CPB * WPC];

    const int lane = threadIdx.x & 63;
    const int p = threadIdx.x & (T - 1);
    const int g = threadIdx.x >> TB;
    const long long cw = (long long)blockIdx.x * CPB + g;
    const bool valid = cw < A.B;
    const long long c = valid ? cw : A.B - 1;  // padding groups decode a duplicate, store nothing
    for (int i = threadIdx.x; i < CPB * WPC; i += kBlock) xs[i] = 0;

    // Received words, bit-packed into LDS (rw > 0, the launcher's choice when the
    // group's words fit): each wave packs whole codewords with coalesced byte loads
    // and a ballot per 64 symbols, so the guard-band parse below probes 32 symbols
    // per LDS read instead of walking zero runs one dependent global load at a time.
    extern __shared__ uint32_t rxb[];
    const bool pk = A.rw > 0;
    if (pk) {
        for (int gg = threadIdx.x >> 6; gg < CPB; gg += kBlock / 64) {
            long long cg = (long long)blockIdx.x * CPB + gg;
            cg = cg < A.B ? cg : A.B - 1;
            const uint8_t* row = A.rx + cg * (long long)A.stride;
            int ln = A.rx_len[cg];
            ln = ln < 0 ? 0 : (ln > A.stride ? A.stride : ln);
            for (int base = 0; base < A.rw * 32; base += 64) {
                const int i = base + lane;
                const unsigned long long msk = __ballot(i < ln && row[i] == 1);
                const int wi = (base >> 5) + (lane & 1);
                if (lane < 2 && wi < A.rw) rxb[gg * A.rw + wi] = (uint32_t)(msk >> (32 * lane));
            }
        }
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

    __shared__ double xv[(T == 64 && !EXP) ? 256 : 1];
    __shared__ unsigned long long xb[4], xub[4];
    DelCtx<T, EXP> cx;
    cx.xv = xv;
    cx.xb = xb;
    cx.xub = xub;
    cx.A = A;
    cx.cw = cw;
    cx.leader = valid && p == 0;
    cx.lane = lane;
    cx.k = 0;
    cx.acc = 0;
    cx.nacc = 0;
    cx.infow = 0;
    uint32_t x;
    if constexpr (N0 == 2) {
        // register-resident path (trellis_n02.h): the base trellis is implicit
        Base02 b;
        b.m = m;
        b.d = kN02L - m;
        b.y = 0;
        if (m <= kN02L)
            for (int i = 0; i < m; ++i) b.y |= (uint32_t)(bit(s + i) & 1) << i;
        b.pins = 0.5 * (1.0 - A.pd);
        b.pdel = 0.5 * A.pd;
        x = del_n02(b, cx);
    } else {
        Trel<L, Cap::V, Cap::E0> base;
        trellis_build<L>(base, bit, s, m, A.pd);
        x = DelNode<L, T, L, EXP>::run(base, cx);
    }
    if (cx.nacc && cx.leader && A.info) A.info[(long long)cx.infow * A.B + cw] = cx.acc;

    // x_hat: trellis t's slice is natural positions [t*L, (t+1)*L)
    __syncthreads();
    const int pos = t * L;
    atomicOr(&xs[g * WPC + (pos >> 5)], (x & ((1u << L) - 1u)) << (pos & 31));
    __syncthreads();
    if (A.xhat && valid)
        for (int i = p; i < WPC; i += T) A.xhat[(long long)i * A.B + cw] = xs[g * WPC + i];
}

typedef void (*DelKern)(DelArgs);

template <int N0, bool EXP>
DelKern del_kernel_tb(int tb) {
    switch (tb) {
        case 1: return k_sc_del<N0, 1, EXP>;
        case 2: return k_sc_del<N0, 2, EXP>;
        case 3: return k_sc_del<N0, 3, EXP>;
        case 4: return k_sc_del<N0, 4, EXP>;
        case 5: return k_sc_del<N0, 5, EXP>;
        case 6: return k_sc_del<N0, 6, EXP>;
        default: return nullptr;
    }
}

template <bool EXP>
DelKern del_kernel(int n0, int tb) {
    switch (n0) {
        case 1: return del_kernel_tb<1, EXP>(tb);
        case 2: return del_kernel_tb<2, EXP>(tb);
        case 3: return del_kernel_tb<3, EXP>(tb);
        default: return nullptr;
    }
}

}  // namespace

extern "C" int pcub_sc_deletion_supported(int32_t n, int32_t n0) { return del_kernel<false>(n0, n - n0) != nullptr; }

namespace {

int launch_del(bool exp, const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n, int32_t n0,
               double pd, const uint32_t* frozen_mask, const uint32_t* frozen_val, const uint32_t* frozen_val_cw,
               int32_t K, uint32_t* info_words, uint32_t* xhat_words, double* leaf, void* stream) {
    const DelKern kern = exp ? del_kernel<true>(n0, n - n0) : del_kernel<false>(n0, n - n0);
    if (!kern || B < 0 || stride < 0 || stride > 32767 || !frozen_mask || (!frozen_val && !frozen_val_cw))
        return PCUB_EINVAL;
    if (K < 0 || K > (1 << n) || (!exp && K > 0 && !info_words) || (B > 0 && (!rx || !rx_len))) return PCUB_EINVAL;
    if (exp && !leaf) return PCUB_EINVAL;
    if (!(pd >= 0.0 && pd <= 1.0)) return PCUB_EINVAL;
    if (B == 0) return 0;
    DelArgs A;
    A.rx = rx;
    A.rx_len = rx_len;
    A.B = B;
    A.stride = stride;
    A.n = n;
    A.pd = pd;
    A.fmask = frozen_mask;
    A.fval = frozen_val;
    A.fval_cw = frozen_val_cw;
    A.info = info_words;
    A.xhat = xhat_words;
    A.leaf = leaf;
    const long long cpb = kBlock >> (n - n0);
    const long long grid = (B + cpb - 1) / cpb;
    if (grid * kBlock > 0xffffffffLL) return PCUB_EINVAL;  // 32-bit dispatch grid (work-items)
    // bit-packed received words in LDS when the group's words fit in 32 KiB (always for
    // the 64-trellis shapes; very long padded rows of small codes parse from HBM)
    const long long rw = ((long long)stride + 31) / 32;
    A.rw = (cpb * rw * 4 <= 32768) ? (int)rw : 0;
    const size_t lds = A.rw ? (size_t)(cpb * rw * 4) : 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), lds, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" int pcub_sc_decode_deletion(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n,
                                       int32_t n0, double pd, const uint32_t* frozen_mask, const uint32_t* frozen_val,
                                       int32_t K, uint32_t* info_words, uint32_t* xhat_words, void* stream) {
    if (!frozen_val) return PCUB_EINVAL;
    return launch_del(false, rx, rx_len, B, stride, n, n0, pd, frozen_mask, frozen_val, nullptr, K, info_words,
                      xhat_words, nullptr, stream);
}

extern "C" int pcub_sc_leaf_deletion(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n,
                                     int32_t n0, double pd, const uint32_t* frozen_mask, const uint32_t* frozen_val,
                                     const uint32_t* frozen_val_cw, int32_t K, uint32_t* info_words,
                                     uint32_t* xhat_words, double* leaf, void* stream) {
    return launch_del(true, rx, rx_len, B, stride, n, n0, pd, frozen_mask, frozen_val, frozen_val_cw, K, info_words,
                      xhat_words, leaf, stream);
}
