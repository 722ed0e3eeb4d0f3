// sc_qary.hip -- q-ary SC decode for gfx950 + C-ABI launcher.
//
// pcub_sc_decode_qary replaces QaryPolarEncoderDecoder.decode
// (QaryPolarEncoderDecoder.py:90-116, recursion :318-401) over
// QaryMemorylessVectorDistribution (VectorDistributions/QaryMemorylessVectorDistribution.py:26-118),
// linear (non-log) domain, for a batch of codewords.  Arithmetic contract:
//   minus  new[u] = 0.0, then new[(x1+x2)%q] += a[x1]*b[x2] with x1 outer, x2 inner (:36-42)
//   plus   new[u2] = 0.0 + a[(u1+u2)%q] * b[(q-u2)%q]                           (:55-62)
//   normalise t = ((0 + p0) + p1) + ... ; if t != 0: p[x] /= t                      (:92-118)
//   leaf   s = sum as above; m = p/s (or 1/q); u = first argmax(m)                  (:69-90, :342)
//   frozen symbols are 0 (:347-351); the a-priori tree is never consulted.
//   combine x[2h] = (xm+xp)%q, x[2h+1] = (q-xp)%q                                    (:397-399)
// Storage follows the binary kernel: half-split order inside each node, so
// children are op(in[p], in[p+L/2]) and the node's symbols are
// y = [(ym+yp)%q | (q-yp)%q]; one codeword per lane; levels 1..n-2 in a
// per-slot scratch (q doubles per position, slot-minor), the last node of two
// positions in registers; decided symbols in a per-slot byte array.
#include <hip/hip_runtime.h>

#include "polarcub_sc.h"
#include "sc_common.h"

using namespace pcub;

namespace {

constexpr int kQBlock = 256;

template <int Q>
struct QV {
    double p[Q];
};

template <int Q>
PCUB_HD QV<Q> q_normalize(QV<Q> v) {
    double t = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) t = t + v.p[x];
    if (t != 0.0) {
#pragma unroll
        for (int x = 0; x < Q; ++x) v.p[x] = v.p[x] / t;
    }
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
    QV<Q> o;
#pragma unroll
    for (int u2 = 0; u2 < Q; ++u2) {
        // a[(u1+u2)%Q] with a wave-divergent u1: select instead of indexing
        const int x1 = (u1 + u2) % Q;
        double ax = a.p[0];
#pragma unroll
        for (int x = 1; x < Q; ++x) ax = (x1 == x) ? a.p[x] : ax;
        o.p[u2] = 0.0 + ax * b.p[(Q - u2) % Q];
    }
    return q_normalize<Q>(o);
}

template <int Q>
PCUB_HD int q_leaf(const QV<Q>& v) {
    double s = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) s = s + v.p[x];
    int arg = 0;
    double best = 0.0;
#pragma unroll
    for (int x = 0; x < Q; ++x) {
        const double m = (s > 0.0) ? v.p[x] / s : 1.0 / (double)Q;
        if (x == 0 || m > best) {
            best = m;
            arg = x;
        }
    }
    return arg;
}

struct QArgs {
    const double* xy;       // [N][B][Q]
    long long B;
    int n;
    const uint8_t* frozen;  // [N] 0/1
    uint8_t* info;          // [K][B]
    uint8_t* xhat;          // [N][B] or null
    double* scratch;        // [(N - 2) positions][Q][nslots]
    uint8_t* ysym;          // [N][nslots]
    long long nslots;
};

template <int Q>
PCUB_HD QV<Q> load_q(const double* base, long long pos, long long stride) {
    QV<Q> v;
#pragma unroll
    for (int x = 0; x < Q; ++x) v.p[x] = base[(pos * Q + x) * stride];
    return v;
}

template <int Q>
PCUB_HD void store_q(double* base, long long pos, long long stride, const QV<Q>& v) {
#pragma unroll
    for (int x = 0; x < Q; ++x) base[(pos * Q + x) * stride] = v.p[x];
}

// depth-d node values at scratch positions [off(d), off(d) + (N >> d)), off(d) = N - 2*(N >> d) (d >= 1)
template <int Q>
PCUB_HD void decode_qary_cw(const QArgs& A, long long cw, long long slot, bool store) {
    const int n = A.n;
    const int N = 1 << n;
    const long long B = A.B, ns = A.nslots;
    const double* in = A.xy + cw * Q;  // element i, symbol x at in[(i*B)*Q + x]
    double* scr = A.scratch + slot;
    uint8_t* Y = A.ysym + slot;
    const int D = n - 1;  // depth of the 2-position nodes held in registers
    int infow = 0;
    for (int k = 0; k < (1 << D); ++k) {
        const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
        for (int d = d0; d <= D; ++d) {
            const bool gop = (d == d0) && (k != 0);
            const int Lo = N >> d;
            const int ystart = (k >> (D - d + 1)) * (N >> (d - 1));  // minus child's first u position
            for (int p = 0; p < Lo; ++p) {
                QV<Q> a, b;
                if (d == 1) {
                    const long long i0 = 2 * (long long)bitrev((uint32_t)p, n - 1);  // natural rows (2q, 2q+1)
                    a = load_q<Q>(in, i0 * B, 1);
                    b = load_q<Q>(in, (i0 + 1) * B, 1);
                } else {
                    const long long off = (long long)N - 2 * (N >> (d - 1));
                    a = load_q<Q>(scr, off + p, ns);
                    b = load_q<Q>(scr, off + p + Lo, ns);
                }
                const QV<Q> o = gop ? q_plus<Q>(a, b, Y[(long long)(ystart + p) * ns]) : q_minus<Q>(a, b);
                store_q<Q>(scr, (long long)N - 2 * Lo + p, ns, o);
            }
        }
        // node of length 2 at depth D (positions off(D), off(D)+1)
        const long long offD = (long long)N - 4;
        const QV<Q> a = load_q<Q>(scr, offD, ns), b = load_q<Q>(scr, offD + 1, ns);
        const int u0i = 2 * k, u1i = 2 * k + 1;
        const int u0 = A.frozen[u0i] ? 0 : q_leaf<Q>(q_minus<Q>(a, b));
        const int u1 = A.frozen[u1i] ? 0 : q_leaf<Q>(q_plus<Q>(a, b, u0));
        if (store) {
            if (!A.frozen[u0i]) A.info[(long long)(infow++) * B + cw] = (uint8_t)u0;
            if (!A.frozen[u1i]) A.info[(long long)(infow++) * B + cw] = (uint8_t)u1;
        } else {
            infow += (A.frozen[u0i] ? 0 : 1) + (A.frozen[u1i] ? 0 : 1);
        }
        Y[(long long)u0i * ns] = (uint8_t)((u0 + u1) % Q);
        Y[(long long)u1i * ns] = (uint8_t)((Q - u1) % Q);
        // combine completed plus children: [(ym+yp)%q | (q-yp)%q]
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
    if (A.xhat && store)
        for (int i = 0; i < N; ++i) A.xhat[(long long)i * B + cw] = Y[(long long)bitrev((uint32_t)i, n) * ns];
}

template <int Q>
__global__ __launch_bounds__(kQBlock) void k_sc_qary(QArgs A) {
    const long long slot = (long long)blockIdx.x * kQBlock + threadIdx.x;
    const long long ntiles = (A.B + kQBlock - 1) / kQBlock;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * kQBlock + threadIdx.x;
        const bool valid = cw < A.B;
        decode_qary_cw<Q>(A, valid ? cw : A.B - 1, slot, valid);
    }
}

// q-ary encoder: u (info symbols at information positions, 0 at frozen ones)
// -> y by in-place block combines -> x = bitrev(y).  Per-lane bytes in `work`.
__global__ __launch_bounds__(kQBlock) void k_encode_qary(const uint8_t* info, long long B, int n, int q,
                                                         const uint8_t* frozen, uint8_t* x) {
    const long long cw = (long long)blockIdx.x * kQBlock + threadIdx.x;
    if (cw >= B) return;
    const int N = 1 << n;
    // u written straight into x (natural u order), combined in place, then permuted in place
    int iw = 0;
    for (int i = 0; i < N; ++i) x[(long long)i * B + cw] = frozen[i] ? 0 : info[(long long)(iw++) * B + cw];
    for (int h = 1; h < N; h <<= 1)
        for (int b0 = 0; b0 < N; b0 += 2 * h)
            for (int p = 0; p < h; ++p) {
                const long long l = (long long)(b0 + p) * B + cw, r = (long long)(b0 + h + p) * B + cw;
                const int ym = x[l], yp = x[r];
                x[l] = (uint8_t)((ym + yp) % q);
                x[r] = (uint8_t)((q - yp) % q);
            }
    for (int i = 0; i < N; ++i) {
        const int j = (int)bitrev((uint32_t)i, n);
        if (j > i) {
            const uint8_t t = x[(long long)i * B + cw];
            x[(long long)i * B + cw] = x[(long long)j * B + cw];
            x[(long long)j * B + cw] = t;
        }
    }
}

typedef void (*QKern)(QArgs);
QKern qkernel(int q) {
    switch (q) {
        case 2: return k_sc_qary<2>;
        case 3: return k_sc_qary<3>;
        case 4: return k_sc_qary<4>;
        case 5: return k_sc_qary<5>;
        case 6: return k_sc_qary<6>;
        case 7: return k_sc_qary<7>;
        case 8: return k_sc_qary<8>;
        default: return nullptr;
    }
}

long long qgrid(long long B, int q) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, qkernel(q), kQBlock, 0) != hipSuccess || occ < 1) occ = 1;
    const long long ntiles = (B + kQBlock - 1) / kQBlock;
    const long long g = (long long)cus * occ;
    return ntiles < g ? ntiles : g;
}

size_t qslot_bytes(int n, int q) {
    const size_t N = (size_t)1 << n;
    return (N - 2) * q * sizeof(double) + N;
}

}  // namespace

extern "C" size_t pcub_sc_decode_qary_workspace(int64_t B, int32_t log2N, int32_t q) {
    if (B <= 0 || log2N < 2 || log2N > 20 || !qkernel(q)) return 0;
    return (size_t)qgrid(B, q) * kQBlock * qslot_bytes(log2N, q);
}

extern "C" int pcub_sc_decode_qary(const double* xy, int64_t B, int32_t log2N, int32_t q, const uint8_t* frozen,
                                   int32_t K, uint8_t* info, uint8_t* xhat, void* workspace, size_t workspace_bytes,
                                   void* stream) {
    if (B < 0 || log2N < 2 || log2N > 20 || !qkernel(q) || !frozen) return PCUB_EINVAL;
    if (K < 0 || K > (1 << log2N) || (K > 0 && !info) || (B > 0 && !xy)) return PCUB_EINVAL;
    if (B == 0) return 0;
    long long g = qgrid(B, q);
    if (g <= 0) return (int)hipErrorNoDevice;
    const size_t per_block = (size_t)kQBlock * qslot_bytes(log2N, q);
    if (!workspace) return PCUB_EINVAL;
    if ((size_t)g * per_block > workspace_bytes) g = (long long)(workspace_bytes / per_block);
    if (g <= 0) return PCUB_EINVAL;
    QArgs A;
    A.xy = xy;
    A.B = B;
    A.n = log2N;
    A.frozen = frozen;
    A.info = info;
    A.xhat = xhat;
    A.nslots = g * kQBlock;
    const size_t N = (size_t)1 << log2N;
    A.scratch = (double*)workspace;
    A.ysym = (uint8_t*)workspace + (size_t)A.nslots * (N - 2) * q * sizeof(double);
    hipLaunchKernelGGL(qkernel(q), dim3((unsigned)g), dim3(kQBlock), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}

extern "C" int pcub_polar_encode_qary(const uint8_t* info, int64_t B, int32_t log2N, int32_t q, const uint8_t* frozen,
                                      int32_t K, uint8_t* x, void* stream) {
    if (B < 0 || log2N < 0 || log2N > 20 || q < 2 || q > 255 || !frozen || !x) return PCUB_EINVAL;
    if (K < 0 || K > (1 << log2N) || (K > 0 && !info)) return PCUB_EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(k_encode_qary, dim3((unsigned)((B + kQBlock - 1) / kQBlock)), dim3(kQBlock), 0,
                       (hipStream_t)stream, info, (long long)B, log2N, q, frozen, x);
    return (int)hipGetLastError();
}
