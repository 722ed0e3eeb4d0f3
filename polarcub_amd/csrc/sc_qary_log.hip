// sc_qary_log.hip -- q-ary SC decode in the log domain (use_log=True), gfx950, + C-ABI.
//
// QaryPolarEncoderDecoder(q, N, frozenSet, seed, use_log=True).decode
// (QaryPolarEncoderDecoder.py:318-401) over log-domain QaryMemorylessVectorDistribution
// (VectorDistributions/QaryMemorylessVectorDistribution.py):
//   minus  new[u] = -inf; new[(x1+x2)%q] = logaddexp(new, a[x1] + b[x2]), x1 outer, x2 inner (:31-42)
//   plus   new[u2] = logaddexp(-inf, a[(u1+u2)%q] + b[(q-u2)%q]) = a + b                 (:50-62)
//   normalise t = logsumexp(p); if t != -inf: p[x] -= t                                (:92-118)
//   leaf   s = logsumexp(p); m = p - s (or -log q each when s = -inf); u = first argmax  (:69-90, :342)
// logaddexp is numpy's npy_logaddexp (x == y: x + ln 2; else max + log1p(exp(-|x-y|)));
// logsumexp is scipy 1.15's (every maximal element taken out of the sum:
// log1p(sum_{x < max} exp(p_x - max) / m) + log(m) + max, m = their count).
// exp / log1p / log are the device's (ROCm ocml), not glibc's, so values agree with the
// reference to a few ulps, not bit for bit: the parity tests state their tolerance.
//
// The simple schedule of sc_leaf.hip (one codeword per lane, every stage level in a
// per-slot scratch, half-split node order): the log domain is an API variant off the
// throughput path, not the headline.
#include <hip/hip_runtime.h>
#include <math.h>

#include "polarcub_sc.h"
#include "sc_common.h"

using namespace pcub;

namespace {

constexpr int kLogBlock = 256;

struct QLArgs {
    const double* xy;        // [N][B][Q] log-probabilities
    long long B;
    int n;
    const uint32_t* fwords;  // ceil(N/32) frozen mask
    uint8_t* info;           // [K][B]
    uint8_t* xhat;           // [N][B] or null
    double* leaf;            // [N][B][Q] log marginals or null
    double* scratch;         // [(N - 2) * Q][nslots]
    uint8_t* ysym;           // [N][nslots]
    long long nslots;
};

constexpr double kLn2 = 0.693147180559945309417232121458176568;

__device__ double logaddexp_np(double x, double y) {
    if (x == y) return x + kLn2;
    const double t = x - y;
    if (t > 0) return x + log1p(exp(-t));
    if (t <= 0) return y + log1p(exp(t));
    return t;  // NaN
}

template <int Q>
__device__ double logsumexp_sp(const double* p) {
    double mx = p[0];
#pragma unroll
    for (int x = 1; x < Q; ++x) mx = p[x] > mx ? p[x] : mx;
    double m = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) m += (p[x] == mx) ? 1.0 : 0.0;
    const double shift = isfinite(mx) ? mx : 0.0;
    // numpy's sum of Q < 9 terms: the first term plus the sequential sum of the rest
    double e[Q];
#pragma unroll
    for (int x = 0; x < Q; ++x) e[x] = (p[x] == mx) ? 0.0 : exp(p[x] - shift);
    double rest = 0.0;
#pragma unroll
    for (int x = 1; x < Q; ++x) rest += e[x];
    double s = e[0] + rest;
    if (s != 0.0) s = s / m;
    return log1p(s) + log(m) + mx;
}

template <int Q>
__device__ void normalize_log(double* p) {
    const double t = logsumexp_sp<Q>(p);
    if (t != -INFINITY) {
#pragma unroll
        for (int x = 0; x < Q; ++x) p[x] -= t;
    }
}

template <int Q>
__device__ void minus_log(const double* a, const double* b, double* o) {
#pragma unroll
    for (int u = 0; u < Q; ++u) o[u] = -INFINITY;
#pragma unroll
    for (int x1 = 0; x1 < Q; ++x1)
#pragma unroll
        for (int x2 = 0; x2 < Q; ++x2) {
            const int u = (x1 + x2) % Q;
            o[u] = logaddexp_np(o[u], a[x1] + b[x2]);
        }
    normalize_log<Q>(o);
}

template <int Q>
__device__ void plus_log(const double* a, const double* b, int u1, double* o) {
#pragma unroll
    for (int u2 = 0; u2 < Q; ++u2) o[u2] = logaddexp_np(-INFINITY, a[(u1 + u2) % Q] + b[(Q - u2) % Q]);
    normalize_log<Q>(o);
}

// the marginal in place; returns the first argmax
template <int Q>
__device__ int leaf_log(double* p) {
    const double s = logsumexp_sp<Q>(p);
    if (s > -INFINITY) {
#pragma unroll
        for (int x = 0; x < Q; ++x) p[x] -= s;
    } else {
        const double d = -log((double)Q);
#pragma unroll
        for (int x = 0; x < Q; ++x) p[x] = d;
    }
    int arg = 0;
#pragma unroll
    for (int x = 1; x < Q; ++x)
        if (p[x] > p[arg]) arg = x;
    return arg;
}

template <int Q>
__device__ void log_cw(const QLArgs& A, long long cw, long long slot, bool store) {
    const int n = A.n;
    const int N = 1 << n;
    const long long B = A.B, ns = A.nslots;
    double* scr = A.scratch + slot;
    uint8_t* Y = A.ysym + slot;
    auto root = [&](long long row, int x) { return A.xy[(row * B + cw) * Q + x]; };
    auto sat = [&](long long pos, int x) -> double& { return scr[(pos * Q + x) * ns]; };
    int infow = 0;
    const int D = n - 1;
    for (int k = 0; k < (1 << D); ++k) {
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        double v0[Q], v1[Q];
        for (int d = d0; d <= D; ++d) {
            const bool gop = (d == d0) && (k != 0);
            const int Lo = N >> d;
            const int ystart = (k >> (D - d + 1)) * (N >> (d - 1));
            for (int p = 0; p < Lo; ++p) {
                const int u = gop ? (int)Y[(long long)(ystart + p) * ns] : 0;
                double a[Q], b[Q], o[Q];
                if (d == 1) {
                    const long long q0 = (long long)bitrev((uint32_t)p, n - 1);
#pragma unroll
                    for (int x = 0; x < Q; ++x) {
                        a[x] = root(2 * q0, x);
                        b[x] = root(2 * q0 + 1, x);
                    }
                } else {
                    const long long off = (long long)N - 2 * (N >> (d - 1));
#pragma unroll
                    for (int x = 0; x < Q; ++x) {
                        a[x] = sat(off + p, x);
                        b[x] = sat(off + p + Lo, x);
                    }
                }
                if (gop) plus_log<Q>(a, b, u, o);
                else minus_log<Q>(a, b, o);
                if (d == D) {
#pragma unroll
                    for (int x = 0; x < Q; ++x) (p == 0 ? v0 : v1)[x] = o[x];
                } else {
#pragma unroll
                    for (int x = 0; x < Q; ++x) sat((long long)N - 2 * Lo + p, x) = o[x];
                }
            }
        }
        if (D == 0) {  // N = 2: the 2-position node is the raw root
#pragma unroll
            for (int x = 0; x < Q; ++x) {
                v0[x] = root(0, x);
                v1[x] = root(1, x);
            }
        }
        const int i0 = 2 * k, i1 = 2 * k + 1;
        double c[Q];
        minus_log<Q>(v0, v1, c);
        const bool f0 = (A.fwords[i0 >> 5] >> (i0 & 31)) & 1u;
        int u0 = leaf_log<Q>(c);
        if (store && A.leaf)
            for (int x = 0; x < Q; ++x) A.leaf[((long long)i0 * B + cw) * Q + x] = c[x];
        if (f0) u0 = 0;
        else {
            if (store) A.info[(long long)infow * B + cw] = (uint8_t)u0;
            ++infow;
        }
        plus_log<Q>(v0, v1, u0, c);
        const bool f1 = (A.fwords[i1 >> 5] >> (i1 & 31)) & 1u;
        int u1 = leaf_log<Q>(c);
        if (store && A.leaf)
            for (int x = 0; x < Q; ++x) A.leaf[((long long)i1 * B + cw) * Q + x] = c[x];
        if (f1) u1 = 0;
        else {
            if (store) A.info[(long long)infow * B + cw] = (uint8_t)u1;
            ++infow;
        }
        Y[(long long)i0 * ns] = (uint8_t)((u0 + u1) % Q);
        Y[(long long)i1 * ns] = (uint8_t)((Q - u1) % Q);
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
    if (store && A.xhat)
        for (int i = 0; i < N; ++i) A.xhat[(long long)i * B + cw] = Y[(long long)bitrev((uint32_t)i, n) * ns];
}

template <int Q>
__global__ __launch_bounds__(kLogBlock) void k_sc_qary_log(QLArgs A) {
    const long long slot = (long long)blockIdx.x * kLogBlock + threadIdx.x;
    const long long ntiles = (A.B + kLogBlock - 1) / kLogBlock;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * kLogBlock + threadIdx.x;
        const bool valid = cw < A.B;
        log_cw<Q>(A, valid ? cw : A.B - 1, slot, valid);
    }
}

typedef void (*LogKern)(QLArgs);

LogKern log_kernel(int q) {
    switch (q) {
        case 2: return k_sc_qary_log<2>;
        case 3: return k_sc_qary_log<3>;
        case 4: return k_sc_qary_log<4>;
        case 5: return k_sc_qary_log<5>;
        case 6: return k_sc_qary_log<6>;
        case 7: return k_sc_qary_log<7>;
        case 8: return k_sc_qary_log<8>;
        default: return nullptr;
    }
}

long long log_grid(long long B, LogKern k) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kLogBlock, 0) != hipSuccess || occ < 1) occ = 1;
    const long long ntiles = (B + kLogBlock - 1) / kLogBlock;
    const long long g = (long long)cus * occ;
    return ntiles < g ? ntiles : g;
}

size_t log_slot_bytes(int n, int q) {
    const size_t N = (size_t)1 << n;
    return (N > 2 ? N - 2 : 1) * (size_t)q * sizeof(double) + N;
}

}  // namespace

extern "C" size_t pcub_sc_decode_qary_log_workspace(int64_t B, int32_t q, int32_t log2N) {
    LogKern k = log_kernel(q);
    if (B <= 0 || !k || log2N < 1 || log2N > 16) return 0;
    return (size_t)log_grid(B, k) * kLogBlock * log_slot_bytes(log2N, q);
}

extern "C" int pcub_sc_decode_qary_log(const double* xy, int64_t B, int32_t q, int32_t log2N,
                                      const uint32_t* frozen_mask, int32_t K, uint8_t* info, uint8_t* xhat,
                                      double* leaf, void* workspace, size_t workspace_bytes, void* stream) {
    LogKern k = log_kernel(q);
    if (!k || B < 0 || log2N < 1 || log2N > 16 || !frozen_mask || K < 0 || K > (1 << log2N)) return PCUB_EINVAL;
    if (B == 0) return 0;
    if (!xy || (K > 0 && !info) || !workspace) return PCUB_EINVAL;
    long long g = log_grid(B, k);
    if (g <= 0) return (int)hipErrorNoDevice;
    const size_t per_block = (size_t)kLogBlock * log_slot_bytes(log2N, q);
    if ((size_t)g * per_block > workspace_bytes) g = (long long)(workspace_bytes / per_block);
    if (g <= 0) return PCUB_EINVAL;
    QLArgs A;
    A.xy = xy;
    A.B = B;
    A.n = log2N;
    A.fwords = frozen_mask;
    A.info = info;
    A.xhat = xhat;
    A.leaf = leaf;
    A.nslots = g * kLogBlock;
    const size_t N = (size_t)1 << log2N;
    A.scratch = (double*)workspace;
    A.ysym = (uint8_t*)workspace + (size_t)A.nslots * (N > 2 ? N - 2 : 1) * (size_t)q * sizeof(double);
    hipLaunchKernelGGL(k, dim3((unsigned)g), dim3(kLogBlock), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}
