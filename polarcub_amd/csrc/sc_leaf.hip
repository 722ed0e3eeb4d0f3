// sc_leaf.hip -- binary SC decode that also exports every leaf's distribution
// (LLR check, genie construction), gfx950, + C-ABI launchers.
//
// pcub_sc_leaf_bin decodes exactly like pcub_sc_decode_bin (same decisions,
// BinaryPolarEncoderDecoder.py:223-325) and additionally writes, for every u
// index i, the normalised xy leaf the reference hands to
// calcMarginalizedProbabilities (VectorDistributions/BinaryMemorylessVectorDistribution.py:52-69)
// -- what recursiveEncodeDecode collects into marginalizedUProbs (:268-273) and
// what the genie turns into Pe / H (genieSingleDecodeSimulatioan, :114-178).
// Frozen values may be given per codeword (the genie draws a fresh common
// randomness for every trial, :101-112), and no rate-0 subtree is skipped:
// every leaf is evaluated.
//
// This is the simple schedule (one codeword per lane, every stage level in a
// per-slot scratch, half-split node order as in sc_bin_body.h); it is the
// export path, not the throughput path.
#include <hip/hip_runtime.h>

#include "polarcub_sc.h"
#include "sc_common.h"

using namespace pcub;

namespace {

constexpr int kLBlock = 256;

struct LeafArgs {
    const double2* xy;          // [N][B] raw pairs
    long long B;
    int n;
    const uint32_t* fmask;      // ceil(N/32)
    const uint32_t* fval;       // ceil(N/32), or null when fval_cw is given
    const uint32_t* fval_cw;    // [ceil(N/32)][B] per-codeword frozen values, or null
    uint32_t* info;             // [ceil(K/32)][B] or null
    uint32_t* xhat;             // [ceil(N/32)][B] or null
    double* leaf;               // [N][B] compact normalised leaf values
    double* scratch;            // [N - 2][nslots]
    uint8_t* ybits;             // [N][nslots]
    long long nslots;
};

PCUB_HD uint32_t word_bit(const uint32_t* w, int i) { return (w[i >> 5] >> (i & 31)) & 1u; }

__device__ void leaf_cw(const LeafArgs& A, long long cw, long long slot, bool store) {
    const int n = A.n;
    const int N = 1 << n;
    const long long B = A.B, ns = A.nslots;
    double* scr = A.scratch + slot;
    uint8_t* Y = A.ybits + slot;
    auto fbit = [&](int i) -> uint32_t {
        return A.fval_cw ? ((A.fval_cw[(long long)(i >> 5) * B + cw] >> (i & 31)) & 1u) : word_bit(A.fval, i);
    };
    uint32_t acc = 0;
    int nacc = 0, infow = 0;
    auto put_info = [&](uint32_t u) {
        acc |= u << nacc;
        if (++nacc == 32) {
            if (store && A.info) A.info[(long long)(infow)*B + cw] = acc;
            ++infow;
            acc = 0;
            nacc = 0;
        }
    };
    const int D = n - 1;  // depth of the 2-value nodes
    for (int k = 0; k < (1 << D); ++k) {
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        double v0 = 0.0, v1 = 0.0;
        bool raw = false;  // N = 2: the 2-value node is the (never normalised) root
        double2 r0, r1;
        if (D == 0) {
            raw = true;
            r0 = A.xy[cw];
            r1 = A.xy[B + cw];
        }
        for (int d = d0; d <= D; ++d) {
            const bool gop = (d == d0) && (k != 0);
            const int Lo = N >> d;
            const int ystart = (k >> (D - d + 1)) * (N >> (d - 1));
            for (int p = 0; p < Lo; ++p) {
                const uint32_t u = gop ? Y[(long long)(ystart + p) * ns] : 0u;
                double o;
                if (d == 1) {
                    const long long q = (long long)bitrev((uint32_t)p, n - 1);
                    const double2 a = A.xy[(2 * q) * B + cw], b = A.xy[(2 * q + 1) * B + cw];
                    o = gop ? op_g_raw(a, b, u) : op_f_raw(a, b);
                } else {
                    const long long off = (long long)N - 2 * (N >> (d - 1));
                    const double a = scr[(off + p) * ns], b = scr[(off + p + Lo) * ns];
                    o = gop ? op_g(a, b, u) : op_f(a, b);
                }
                if (d == D) {
                    if (p == 0) v0 = o;
                    else v1 = o;
                } else {
                    scr[((long long)N - 2 * Lo + p) * ns] = o;
                }
            }
        }
        // the two leaves of this depth-D node: normalised minus / plus children
        const int i0 = 2 * k, i1 = 2 * k + 1;
        const double c0 = raw ? op_f_raw(r0, r1) : op_f(v0, v1);
        const uint32_t u0 = word_bit(A.fmask, i0) ? fbit(i0) : leaf_v(c0);
        const double c1 = raw ? op_g_raw(r0, r1, u0) : op_g(v0, v1, u0);
        const uint32_t u1 = word_bit(A.fmask, i1) ? fbit(i1) : leaf_v(c1);
        if (store) {
            A.leaf[(long long)i0 * B + cw] = c0;
            A.leaf[(long long)i1 * B + cw] = c1;
        }
        if (!word_bit(A.fmask, i0)) put_info(u0);
        if (!word_bit(A.fmask, i1)) put_info(u1);
        Y[(long long)i0 * ns] = (uint8_t)(u0 ^ u1);
        Y[(long long)i1 * ns] = (uint8_t)u1;
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = N >> d;
            const long long st = (long long)(k >> (D - d + 1)) * 2 * Lc;
            for (int p = 0; p < Lc; ++p) Y[(st + p) * ns] ^= Y[(st + Lc + p) * ns];
        }
    }
    if (store && nacc && A.info) A.info[(long long)infow * B + cw] = acc;
    if (store && A.xhat) {
        for (int w = 0; w < (N + 31) / 32; ++w) {
            uint32_t o = 0;
            for (int t = 0; t < 32 && 32 * w + t < N; ++t)
                o |= (uint32_t)Y[(long long)bitrev((uint32_t)(32 * w + t), n) * ns] << t;
            A.xhat[(long long)w * B + cw] = o;
        }
    }
}

__global__ __launch_bounds__(kLBlock) void k_sc_leaf(LeafArgs A) {
    const long long slot = (long long)blockIdx.x * kLBlock + threadIdx.x;
    const long long ntiles = (A.B + kLBlock - 1) / kLBlock;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * kLBlock + threadIdx.x;
        const bool valid = cw < A.B;
        leaf_cw(A, valid ? cw : A.B - 1, slot, valid);
    }
}

// ---------------------------------------------------------------------------------------------
// Two-tree SC: a non-uniform a-priori distribution (BinaryPolarEncoderDecoder.py:223-325 with
// xVectorDistribution not uniform).  The x tree (prior) runs beside the xy tree through the same
// minus / plus / normalise steps with the same decisions; a frozen u_i is 0 iff the x leaf's
// marginal m0 >= r_i (:258-262), an information u_i is the xy leaf's decision (decode, :249-252)
// or the given bit (encode: xy == null, :254).  Same simple schedule as k_sc_leaf, one stage
// scratch per tree.

struct PriorArgs {
    const double2* xy;       // [N][B] raw pairs, or null (encode)
    const double2* px;       // [N][PB] raw prior pairs, PB = 1 (shared) or B
    long long PB;
    long long B;
    int n;
    const uint32_t* fmask;   // ceil(N/32)
    const double* rnd;       // [N] common randomness r_i
    uint32_t* info;          // [ceil(K/32)][B]: output (decode) or input (encode)
    uint32_t* xhat;          // [ceil(N/32)][B] or null
    double* leaf;            // [N][B] compact leaves of the deciding tree (xy, or x when encoding), or null
    double* scratch;         // [2][N - 2][nslots]
    uint8_t* ybits;          // [N][nslots]
    long long nslots;
};

// the reference's marginal m0 of a compact normalised leaf (calcMarginalizedProbabilities, :52-69)
PCUB_HD double leaf_m0(double v) {
    const CV c = cv_load(v);
    double p0 = c.s ? c.r : 1.0, p1 = c.s ? 1.0 : c.r;
    if (c.r != c.r) p0 = p1 = 0.0;
    double s = 0.0;
    s += p0;
    s += p1;
    return s > 0.0 ? p0 / s : 0.5;
}

template <bool XY>
__device__ void prior_cw(const PriorArgs& A, long long cw, long long slot, bool store) {
    const int n = A.n;
    const int N = 1 << n;
    const long long B = A.B, ns = A.nslots;
    const long long pcw = A.PB == 1 ? 0 : cw;
    const long long tsz = (long long)(N > 2 ? N - 2 : 1) * ns;  // one tree's scratch
    double* scr = A.scratch + slot;          // xy tree
    double* scx = A.scratch + tsz + slot;    // x tree
    uint8_t* Y = A.ybits + slot;
    uint32_t acc = 0, inw = 0;
    int nacc = 0, infow = 0, ii = 0;
    auto info_bit = [&](uint32_t u) -> uint32_t {  // decode: collect u; encode: read the next bit
        if (XY) {
            acc |= u << nacc;
            if (++nacc == 32) {
                if (store) A.info[(long long)infow * B + cw] = acc;
                ++infow;
                acc = 0;
                nacc = 0;
            }
            return u;
        }
        if ((ii & 31) == 0) inw = A.info[(long long)(ii >> 5) * B + cw];
        return (inw >> (ii++ & 31)) & 1u;
    };
    const int D = n - 1;
    for (int k = 0; k < (1 << D); ++k) {
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        double v0 = 0.0, v1 = 0.0, w0 = 0.0, w1 = 0.0;
        for (int d = d0; d <= D; ++d) {
            const bool gop = (d == d0) && (k != 0);
            const int Lo = N >> d;
            const int ystart = (k >> (D - d + 1)) * (N >> (d - 1));
            for (int p = 0; p < Lo; ++p) {
                const uint32_t u = gop ? Y[(long long)(ystart + p) * ns] : 0u;
                double o = 0.0, ox;
                if (d == 1) {
                    const long long q = (long long)bitrev((uint32_t)p, n - 1);
                    if (XY) {
                        const double2 a = A.xy[(2 * q) * B + cw], b = A.xy[(2 * q + 1) * B + cw];
                        o = gop ? op_g_raw(a, b, u) : op_f_raw(a, b);
                    }
                    const double2 a = A.px[(2 * q) * A.PB + pcw], b = A.px[(2 * q + 1) * A.PB + pcw];
                    ox = gop ? op_g_raw(a, b, u) : op_f_raw(a, b);
                } else {
                    const long long off = (long long)N - 2 * (N >> (d - 1));
                    if (XY) {
                        const double a = scr[(off + p) * ns], b = scr[(off + p + Lo) * ns];
                        o = gop ? op_g(a, b, u) : op_f(a, b);
                    }
                    const double a = scx[(off + p) * ns], b = scx[(off + p + Lo) * ns];
                    ox = gop ? op_g(a, b, u) : op_f(a, b);
                }
                if (d == D) {
                    if (p == 0) v0 = o, w0 = ox;
                    else v1 = o, w1 = ox;
                } else {
                    if (XY) scr[((long long)N - 2 * Lo + p) * ns] = o;
                    scx[((long long)N - 2 * Lo + p) * ns] = ox;
                }
            }
        }
        const int i0 = 2 * k, i1 = 2 * k + 1;
        double c0 = 0.0, c1 = 0.0, x0, x1;
        uint32_t u0, u1;
        if (D == 0) {
            const double2 pa = A.px[pcw], pb = A.px[A.PB + pcw];
            double2 ra{0.0, 0.0}, rb{0.0, 0.0};
            if (XY) {
                ra = A.xy[cw];
                rb = A.xy[B + cw];
                c0 = op_f_raw(ra, rb);
            }
            x0 = op_f_raw(pa, pb);
            u0 = word_bit(A.fmask, i0) ? (leaf_m0(x0) >= A.rnd[i0] ? 0u : 1u) : info_bit(XY ? leaf_v(c0) : 0u);
            if (XY) c1 = op_g_raw(ra, rb, u0);
            x1 = op_g_raw(pa, pb, u0);
        } else {
            if (XY) c0 = op_f(v0, v1);
            x0 = op_f(w0, w1);
            u0 = word_bit(A.fmask, i0) ? (leaf_m0(x0) >= A.rnd[i0] ? 0u : 1u) : info_bit(XY ? leaf_v(c0) : 0u);
            if (XY) c1 = op_g(v0, v1, u0);
            x1 = op_g(w0, w1, u0);
        }
        u1 = word_bit(A.fmask, i1) ? (leaf_m0(x1) >= A.rnd[i1] ? 0u : 1u) : info_bit(XY ? leaf_v(c1) : 0u);
        if (store && A.leaf) {
            A.leaf[(long long)i0 * B + cw] = XY ? c0 : x0;
            A.leaf[(long long)i1 * B + cw] = XY ? c1 : x1;
        }
        Y[(long long)i0 * ns] = (uint8_t)(u0 ^ u1);
        Y[(long long)i1 * ns] = (uint8_t)u1;
        for (int d = D; d >= 1 && ((k >> (D - d)) & 1); --d) {
            const int Lc = N >> d;
            const long long st = (long long)(k >> (D - d + 1)) * 2 * Lc;
            for (int p = 0; p < Lc; ++p) Y[(st + p) * ns] ^= Y[(st + Lc + p) * ns];
        }
    }
    if (XY && store && nacc) A.info[(long long)infow * B + cw] = acc;
    if (store && A.xhat) {
        for (int w = 0; w < (N + 31) / 32; ++w) {
            uint32_t o = 0;
            for (int t = 0; t < 32 && 32 * w + t < N; ++t)
                o |= (uint32_t)Y[(long long)bitrev((uint32_t)(32 * w + t), n) * ns] << t;
            A.xhat[(long long)w * B + cw] = o;
        }
    }
}

template <bool XY>
__global__ __launch_bounds__(kLBlock) void k_sc_prior(PriorArgs A) {
    const long long slot = (long long)blockIdx.x * kLBlock + threadIdx.x;
    const long long ntiles = (A.B + kLBlock - 1) / kLBlock;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * kLBlock + threadIdx.x;
        const bool valid = cw < A.B;
        prior_cw<XY>(A, valid ? cw : A.B - 1, slot, valid);
    }
}

// compact leaf -> the reference's marginal: s = 0 + p0 + p1; m = p / s, or (0.5, 0.5)
__device__ void leaf_marginal(const double* leaf, long long i, double* m) {
    const CV c = cv_load(leaf[i]);
    double p0 = c.s ? c.r : 1.0, p1 = c.s ? 1.0 : c.r;
    if (c.r != c.r) p0 = p1 = 0.0;  // the (0, 0) sentinel
    double s = 0.0;
    s += p0;
    s += p1;
    m[2 * i] = s > 0.0 ? p0 / s : 0.5;
    m[2 * i + 1] = s > 0.0 ? p1 / s : 0.5;
}

// grid-stride: count = N * B can pass the 32-bit dispatch grid size
__global__ __launch_bounds__(kLBlock) void k_leaf_marginals(const double* leaf, long long count, double* m) {
    for (long long i = (long long)blockIdx.x * kLBlock + threadIdx.x; i < count; i += (long long)gridDim.x * kLBlock)
        leaf_marginal(leaf, i, m);
}

long long leaf_grid(long long B) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_sc_leaf, kLBlock, 0) != hipSuccess || occ < 1) occ = 1;
    const long long ntiles = (B + kLBlock - 1) / kLBlock;
    const long long g = (long long)cus * occ;
    return ntiles < g ? ntiles : g;
}

size_t leaf_slot_bytes(int n) {
    const size_t N = (size_t)1 << n;
    return (N > 2 ? N - 2 : 1) * sizeof(double) + N;
}

}  // namespace

extern "C" size_t pcub_sc_leaf_bin_workspace(int64_t B, int32_t log2N) {
    if (B <= 0 || log2N < 1 || log2N > 20) return 0;
    return (size_t)leaf_grid(B) * kLBlock * leaf_slot_bytes(log2N);
}

extern "C" int pcub_sc_leaf_bin(const double* xy, int64_t B, int32_t log2N, const uint32_t* frozen_mask,
                                const uint32_t* frozen_val, const uint32_t* frozen_val_cw, int32_t K,
                                uint32_t* info_words, uint32_t* xhat_words, double* leaf, void* workspace,
                                size_t workspace_bytes, void* stream) {
    if (B < 0 || log2N < 1 || log2N > 20 || !frozen_mask || (!frozen_val && !frozen_val_cw) || !leaf)
        return PCUB_EINVAL;
    if (K < 0 || K > (1 << log2N) || (B > 0 && !xy)) return PCUB_EINVAL;
    if (B == 0) return 0;
    long long g = leaf_grid(B);
    if (g <= 0) return (int)hipErrorNoDevice;
    const size_t per_block = (size_t)kLBlock * leaf_slot_bytes(log2N);
    if (!workspace) return PCUB_EINVAL;
    if ((size_t)g * per_block > workspace_bytes) g = (long long)(workspace_bytes / per_block);
    if (g <= 0) return PCUB_EINVAL;
    LeafArgs A;
    A.xy = (const double2*)xy;
    A.B = B;
    A.n = log2N;
    A.fmask = frozen_mask;
    A.fval = frozen_val;
    A.fval_cw = frozen_val_cw;
    A.info = info_words;
    A.xhat = xhat_words;
    A.leaf = leaf;
    A.nslots = g * kLBlock;
    const size_t N = (size_t)1 << log2N;
    A.scratch = (double*)workspace;
    A.ybits = (uint8_t*)workspace + (size_t)A.nslots * (N > 2 ? N - 2 : 1) * sizeof(double);
    hipLaunchKernelGGL(k_sc_leaf, dim3((unsigned)g), dim3(kLBlock), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}

namespace {

long long prior_grid(long long B, bool xy) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    const hipError_t e = xy ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_sc_prior<true>, kLBlock, 0)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_sc_prior<false>, kLBlock, 0);
    if (e != hipSuccess || occ < 1) occ = 1;
    const long long ntiles = (B + kLBlock - 1) / kLBlock;
    const long long g = (long long)cus * occ;
    return ntiles < g ? ntiles : g;
}

size_t prior_slot_bytes(int n) {
    const size_t N = (size_t)1 << n;
    return 2 * (N > 2 ? N - 2 : 1) * sizeof(double) + N;
}

}  // namespace

extern "C" size_t pcub_sc_prior_bin_workspace(int64_t B, int32_t log2N) {
    if (B <= 0 || log2N < 1 || log2N > 20) return 0;
    return (size_t)prior_grid(B, true) * kLBlock * prior_slot_bytes(log2N);
}

extern "C" int pcub_sc_prior_bin(const double* xy, const double* px, int64_t px_batch, int64_t B, int32_t log2N,
                                 const uint32_t* frozen_mask, const double* rnd, int32_t K, uint32_t* info_words,
                                 uint32_t* xhat_words, double* leaf, void* workspace, size_t workspace_bytes,
                                 void* stream) {
    if (B < 0 || log2N < 1 || log2N > 20 || !frozen_mask || !rnd || !px) return PCUB_EINVAL;
    if (px_batch != 1 && px_batch != B) return PCUB_EINVAL;
    if (K < 0 || K > (1 << log2N) || (K > 0 && !info_words)) return PCUB_EINVAL;
    if (B == 0) return 0;
    const bool dec = xy != nullptr;
    long long g = prior_grid(B, dec);
    if (g <= 0) return (int)hipErrorNoDevice;
    const size_t per_block = (size_t)kLBlock * prior_slot_bytes(log2N);
    if (!workspace) return PCUB_EINVAL;
    if ((size_t)g * per_block > workspace_bytes) g = (long long)(workspace_bytes / per_block);
    if (g <= 0) return PCUB_EINVAL;
    PriorArgs A;
    A.xy = (const double2*)xy;
    A.px = (const double2*)px;
    A.PB = px_batch;
    A.B = B;
    A.n = log2N;
    A.fmask = frozen_mask;
    A.rnd = rnd;
    A.info = info_words;
    A.xhat = xhat_words;
    A.leaf = leaf;
    A.nslots = g * kLBlock;
    const size_t N = (size_t)1 << log2N;
    A.scratch = (double*)workspace;
    A.ybits = (uint8_t*)workspace + 2 * (size_t)A.nslots * (N > 2 ? N - 2 : 1) * sizeof(double);
    if (dec) hipLaunchKernelGGL(k_sc_prior<true>, dim3((unsigned)g), dim3(kLBlock), 0, (hipStream_t)stream, A);
    else hipLaunchKernelGGL(k_sc_prior<false>, dim3((unsigned)g), dim3(kLBlock), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}

extern "C" int pcub_leaf_marginals(const double* leaf, int64_t count, double* marginals, void* stream) {
    if (count < 0 || (count > 0 && (!leaf || !marginals))) return PCUB_EINVAL;
    if (count == 0) return 0;
    const long long blocks = (count + kLBlock - 1) / kLBlock;
    hipLaunchKernelGGL(k_leaf_marginals, dim3((unsigned)(blocks < (1 << 20) ? blocks : (1 << 20))), dim3(kLBlock), 0,
                       (hipStream_t)stream, leaf, (long long)count, marginals);
    return (int)hipGetLastError();
}
