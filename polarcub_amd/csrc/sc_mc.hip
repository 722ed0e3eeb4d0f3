// sc_mc.hip -- device Monte-Carlo: information bits and channel outputs keyed by the
// GLOBAL codeword index, and the error counters (gfx950) + C-ABI launchers.
//
// The reference's encodeDecodeSimulation (BinaryPolarEncoderDecoder.py:328-387)
// draws information bits (`0 if rng.random() < 0.5 else 1`, :350-358) and the
// channel from MT19937 streams, one trial after another.  On the GPU every
// codeword g gets its own Philox4x32-10 stream keyed by (seed, g): the batch
// [offset, offset + B) is the same whichever rank or chunk generates it, so a run
// sharded over G GPUs decodes exactly the codewords of the 1-GPU run and the
// summed counters match (tests/test_gpu_mc.py).  Statistically the draws follow
// the reference's laws (uniform bits; BSC flips with probability p; BI-AWGN
// y = (1 - 2x) + sigma z with z ~ N(0, 1) by Box-Muller); they are not
// MT19937-identical -- exact reproduction of a reference run uses the host
// driver (coding.encodeDecodeSimulation), which replays the reference's RNGs.
#include <hip/hip_runtime.h>

#include "polarcub_sc.h"
#include "sc_common.h"

using namespace pcub;

namespace {

constexpr int kMcBlock = 256;

// Philox4x32-10 (Salmon et al., SC'11): counter (c0..c3), key (k0, k1).
struct P4 {
    uint32_t v[4];
};

PCUB_HD P4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c0, p1 = (uint64_t)M1 * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += W0;
        k1 += W1;
    }
    return P4{{c0, c1, c2, c3}};
}

// streams inside one codeword's counter space
constexpr uint32_t kStreamInfo = 0, kStreamChannel = 1;

// uniform double in (0, 1] from 53 random bits
PCUB_HD double u01(uint32_t hi, uint32_t lo) {
    const uint64_t m = (((uint64_t)hi << 32) | lo) >> 11;
    return ((double)m + 1.0) * (1.0 / 9007199254740992.0);
}

struct McArgs {
    uint64_t seed;
    long long offset;  // global index of codeword 0 of this batch
    long long B;
    int n;
    int K;
    int channel;       // 0 = BI-AWGN (param = sigma^2), 1 = BSC (param = p)
    double param;
    double sigma;      // BI-AWGN: sqrt(sigma^2)
    double inv2s2;     //          1 / (2 sigma^2)
    double dens;       //          0.5 / sqrt(2 pi sigma^2) (uniform prior x Gaussian density)
    int tile;          // channel rows: 0 = [N][B]; T > 0 = [ceil(B/T)][N][T] (pcub_sc_decode_bin_tiled)
};

// element (row i, codeword b) of a batch of channel rows
PCUB_HD long long row_at(const McArgs& A, long long i, long long b) {
    if (A.tile <= 0) return i * A.B + b;
    return (b / A.tile) * ((long long)A.tile << A.n) + i * A.tile + b % A.tile;
}

// K uniform information bits per codeword: word w of codeword g is Philox
// output lane (w & 3) of counter (g, kStreamInfo, w >> 2).
__global__ __launch_bounds__(kMcBlock) void k_mc_info(McArgs A, uint32_t* info) {
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    if (b >= A.B) return;
    const uint64_t g = (uint64_t)(A.offset + b);
    const int W = (A.K + 31) / 32;
    for (int w = 0; w < W; w += 4) {
        const P4 r = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamInfo, (uint32_t)(w >> 2), (uint32_t)A.seed,
                            (uint32_t)(A.seed >> 32));
        for (int j = 0; j < 4 && w + j < W; ++j) {
            uint32_t v = r.v[j];
            if (w + j == W - 1 && (A.K & 31)) v &= (1u << (A.K & 31)) - 1u;
            info[(long long)(w + j) * A.B + b] = v;
        }
    }
}

// Channel outputs as joint pairs, native [N][B][2].  Elements 2j and 2j+1 of
// codeword g share Philox counter (g, kStreamChannel, j): words 0-1 and 2-3 are
// two 53-bit uniforms, and for BI-AWGN one Box-Muller transform yields both
// normals (cos and sin branches).  A thread owns one codeword and walks element
// pairs, so both of its stores are coalesced over the codeword-minor layout and
// no 64-bit index division is needed.  sigma, 1/(2 sigma^2) and the density
// constant come precomputed from the host.
__device__ __forceinline__ double2 awgn_pair(const McArgs& A, uint32_t xb, double z) {
    const double y = (xb ? -1.0 : 1.0) + A.sigma * z;
    double2 o;
    o.x = A.dens * exp(-((y - 1.0) * (y - 1.0)) * A.inv2s2);
    o.y = A.dens * exp(-((y + 1.0) * (y + 1.0)) * A.inv2s2);
    return o;
}

__device__ __forceinline__ double2 bsc_pair(const McArgs& A, uint32_t xb, double u) {
    // makeBSC table probs[y][x] = [[.5(1-p), .5p], [.5p, .5(1-p)]]
    const uint32_t yb = xb ^ (u <= A.param ? 1u : 0u);
    const double hi = 0.5 * (1.0 - A.param), lo = 0.5 * A.param;
    double2 o;
    o.x = yb ? lo : hi;
    o.y = yb ? hi : lo;
    return o;
}

// Two standard normals from two uniforms in (0, 1] (Box-Muller).  The transcendentals run in f32:
// the noise is a simulation draw, not a reference value, and the f32 forms (v_log_f32, v_sqrt_f32,
// sin / cos by pi-scaled reduction) are a few VALU each where the f64 log, sqrt and sincospi took
// ~150 of the channel kernel's ~190 f64 instructions a pair.  u0 keeps its 53-bit resolution down
// to the tail (u0 >= 2^-53 -> |z| <= 8.6), the 24-bit mantissa only rounds z (relative 6e-8).
__device__ __forceinline__ void box_muller(double u0, double u1, double& z0, double& z1) {
    const float rad = sqrtf(-2.0f * logf((float)u0));
    float sn, cs;
    sincospif(2.0f * (float)u1, &sn, &cs);
    z0 = (double)(rad * cs);
    z1 = (double)(rad * sn);
}

// grid: x over codewords, y strides over element pairs (a 2-D grid keeps every
// dimension far below the 32-bit dispatch limits at N = 2^24).
__global__ __launch_bounds__(kMcBlock) void k_mc_channel(McArgs A, const uint32_t* x, double2* xy) {
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    if (b >= A.B) return;
    const uint64_t g = (uint64_t)(A.offset + b);
    const long long N = 1LL << A.n;
    const long long pairs = (N + 1) / 2;
    for (long long j = blockIdx.y; j < pairs; j += gridDim.y) {
        const long long i0 = 2 * j;
        const uint32_t xw = x[(i0 >> 5) * A.B + b] >> (i0 & 31);  // bits i0, i0 + 1 (same word: i0 even)
        const P4 r = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamChannel, (uint32_t)j, (uint32_t)A.seed,
                            (uint32_t)(A.seed >> 32));
        const double u0 = u01(r.v[0], r.v[1]), u1 = u01(r.v[2], r.v[3]);
        double2 o0, o1;
        if (A.channel == 0) {
            double z0, z1;
            box_muller(u0, u1, z0, z1);
            o0 = awgn_pair(A, xw & 1u, z0);
            o1 = awgn_pair(A, (xw >> 1) & 1u, z1);
        } else {
            o0 = bsc_pair(A, xw & 1u, u0);
            o1 = bsc_pair(A, (xw >> 1) & 1u, u1);
        }
        xy[row_at(A, i0, b)] = o0;
        if (i0 + 1 < N) xy[row_at(A, i0 + 1, b)] = o1;
    }
}

// Normalised channel rows (each joint row divided by its larger entry: the same channel law, and
// no SC decision depends on a row's positive scale), as compact values (+r: (1, r), -r: (r, 1);
// COMPACT, [N][B] doubles) or as the pairs they stand for ([N][B][2]).  BI-AWGN: the likelihood
// ratio p0 / p1 = exp(2y / sigma^2), so the row is (1, exp(-2y/s2)) for y >= 0, else
// (exp(2y/s2), 1); BSC: makeBSC's row normalised (norm_pack).
//
// Draws (round 5).  BSC: elements 4j..4j+3 of codeword g take the four words of Philox counter
// (g, kStreamChannel, j) as 32-bit uniforms u = (r + 1) 2^-32 in (0, 1] and flip where u <= p.
// BI-AWGN: elements 4j..4j+3 take counters (g, kStreamChannel, 2j) and (g, kStreamChannel, 2j+1):
// the first gives two 53-bit uniforms (the Box-Muller radii, so the tail reaches |z| = 8.6 as with
// f64 draws; a 32-bit radius stops at 6.66, below which sigma ~ 0.15 could never flip a bit), the
// second two 32-bit uniforms for the angles.  The transforms run in f32 (v_log_f32, v_sqrt_f32, sin /
// cos by pi-scaled reduction), and so do y, l = 2y/s2 and exp(-|l|) while |l| < 80; past that the
// f32 exp would underflow (to 0 at |l| > ~103: a hard row the f64 reference never produces) and the
// row is exp(-|l|) in f64.  The noise is a simulation draw, not a reference value: f32 rounds a row
// to a relative 6e-8, far below anything a frame-error rate resolves, and the decode's arithmetic on
// the stored rows is the reference's in f64 (test_gpu_fer.py holds the FER to the reference's runs,
// test_gpu_mc.py the rows at 20 dB).
__device__ __forceinline__ float u01f(uint32_t r) { return ((float)r + 1.0f) * 2.3283064365386963e-10f; }

__device__ __forceinline__ double awgn_normf(const McArgs& A, uint32_t xb, float z) {
    const float y = (xb ? -1.0f : 1.0f) + (float)A.sigma * z;
    const float l = y * (float)(A.inv2s2 * 4.0);  // 2 y / sigma^2
    const float al = __builtin_fabsf(l);
    const double r = al < 80.0f ? (double)expf(-al) : exp(-(double)al);
    return l >= 0.0f ? r : -r;
}

__device__ __forceinline__ void put_norm(double* out, long long at, double c, bool compact) {
    if (compact) {
        out[at] = c;
    } else {
        const double r = __builtin_fabs(c);
        ((double2*)out)[at] = __builtin_signbit(c) ? double2{r, 1.0} : double2{1.0, r};
    }
}

template <bool COMPACT>
__global__ __launch_bounds__(kMcBlock) void k_mc_channel_norm(McArgs A, const uint32_t* x, double* out) {
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    if (b >= A.B) return;
    const uint64_t g = (uint64_t)(A.offset + b);
    const long long N = 1LL << A.n;
    const long long quads = (N + 3) / 4;
    const long long base = row_at(A, 0, b), stride = A.tile > 0 ? (long long)A.tile : A.B;
    const float pf = (float)A.param;
    for (long long j = blockIdx.y; j < quads; j += gridDim.y) {
        const long long i0 = 4 * j;
        const uint32_t xw = x[(i0 >> 5) * A.B + b] >> (i0 & 31);  // bits i0..i0+3 (one word: i0 % 4 == 0)
        double c[4];
        if (A.channel == 0) {
            const P4 ra = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamChannel, (uint32_t)(2 * j),
                                 (uint32_t)A.seed, (uint32_t)(A.seed >> 32));
            const P4 rb = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamChannel, (uint32_t)(2 * j + 1),
                                 (uint32_t)A.seed, (uint32_t)(A.seed >> 32));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float rad = sqrtf(-2.0f * logf((float)u01(ra.v[2 * h], ra.v[2 * h + 1])));
                float sn, cs;
                sincospif(2.0f * u01f(rb.v[h]), &sn, &cs);
                c[2 * h] = awgn_normf(A, (xw >> (2 * h)) & 1u, rad * cs);
                c[2 * h + 1] = awgn_normf(A, (xw >> (2 * h + 1)) & 1u, rad * sn);
            }
        } else {
            const P4 r = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamChannel, (uint32_t)j, (uint32_t)A.seed,
                                (uint32_t)(A.seed >> 32));
            const double hi = 0.5 * (1.0 - A.param), lo = 0.5 * A.param;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t yb = ((xw >> k) & 1u) ^ (u01f(r.v[k]) <= pf ? 1u : 0u);
                c[k] = yb ? norm_pack(lo, hi) : norm_pack(hi, lo);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i0 + k < N) put_norm(out, base + (i0 + k) * stride, c[k], COMPACT);
    }
}

// counters[0] += B, [1] += frame errors, [2] += bit errors (information bits)
__global__ __launch_bounds__(kMcBlock) void k_mc_count(const uint32_t* dec, const uint32_t* sent, long long B, int W,
                                                        unsigned long long* counters) {
    __shared__ unsigned long long fe[kMcBlock / 64], be[kMcBlock / 64];
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    unsigned long long f = 0, e = 0;
    if (b < B) {
        for (int w = 0; w < W; ++w) e += (unsigned long long)__builtin_popcount(dec[(long long)w * B + b] ^ sent[(long long)w * B + b]);
        f = e ? 1ull : 0ull;
    }
    for (int o = 32; o > 0; o >>= 1) {
        f += __shfl_xor(f, o);
        e += __shfl_xor(e, o);
    }
    if ((threadIdx.x & 63) == 0) {
        fe[threadIdx.x >> 6] = f;
        be[threadIdx.x >> 6] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tf = 0, tb = 0;
        for (int i = 0; i < kMcBlock / 64; ++i) {
            tf += fe[i];
            tb += be[i];
        }
        atomicAdd(&counters[1], tf);
        atomicAdd(&counters[2], tb);
        if (blockIdx.x == 0) atomicAdd(&counters[0], (unsigned long long)B);
    }
}

// q-ary: counters[0] += B, [1] += frame errors, [2] += symbol errors over [K][B] u8 symbols
__global__ __launch_bounds__(kMcBlock) void k_mc_count_sym(const uint8_t* dec, const uint8_t* sent, long long B, int K,
                                                            unsigned long long* counters) {
    __shared__ unsigned long long fe[kMcBlock / 64], se[kMcBlock / 64];
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    unsigned long long f = 0, e = 0;
    if (b < B) {
        for (int k = 0; k < K; ++k) e += dec[(long long)k * B + b] != sent[(long long)k * B + b] ? 1ull : 0ull;
        f = e ? 1ull : 0ull;
    }
    for (int o = 32; o > 0; o >>= 1) {
        f += __shfl_xor(f, o);
        e += __shfl_xor(e, o);
    }
    if ((threadIdx.x & 63) == 0) {
        fe[threadIdx.x >> 6] = f;
        se[threadIdx.x >> 6] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tf = 0, ts = 0;
        for (int i = 0; i < kMcBlock / 64; ++i) {
            tf += fe[i];
            ts += se[i];
        }
        atomicAdd(&counters[1], tf);
        atomicAdd(&counters[2], ts);
        if (blockIdx.x == 0) atomicAdd(&counters[0], (unsigned long long)B);
    }
}

unsigned grid_of(long long work) { return (unsigned)((work + kMcBlock - 1) / kMcBlock); }

// uniform symbol in [0, m) from 32 random bits (multiply-shift)
PCUB_HD uint32_t below(uint32_t r, uint32_t m) { return (uint32_t)(((uint64_t)r * m) >> 32); }

// q-ary information symbols [K][B] u8: symbol k of codeword g is below(q) of Philox output
// lane (k & 3) of counter (g, kStreamInfo, k >> 2)
__global__ __launch_bounds__(kMcBlock) void k_mc_info_qary(McArgs A, int q, uint8_t* info) {
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    if (b >= A.B) return;
    const uint64_t g = (uint64_t)(A.offset + b);
    for (int k = 0; k < A.K; k += 4) {
        const P4 r = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamInfo, (uint32_t)(k >> 2), (uint32_t)A.seed,
                            (uint32_t)(A.seed >> 32));
        for (int j = 0; j < 4 && k + j < A.K; ++j) info[(long long)(k + j) * A.B + b] = (uint8_t)below(r.v[j], q);
    }
}

// q-ary symmetric channel (makeQSC, ScalarDistributions/QaryMemorylessDistribution.py:780-784) as
// joint rows [N][B][q]: position i of codeword g draws counter (g, kStreamChannel, i): words 0-1
// a 53-bit uniform u (error iff u <= p), word 2 the shift s in [1, q) of an erroneous symbol;
// y = (x + s) % q, row[y'] = 1 - p if y' == y else p / (q - 1)
__global__ __launch_bounds__(kMcBlock) void k_mc_qsc(McArgs A, int q, const uint8_t* x, double* xy) {
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    if (b >= A.B) return;
    const uint64_t g = (uint64_t)(A.offset + b);
    const long long N = 1LL << A.n;
    const double hit = 1.0 - A.param, miss = A.param / (double)(q - 1);
    for (long long i = blockIdx.y; i < N; i += gridDim.y) {
        const P4 r = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamChannel, (uint32_t)i, (uint32_t)A.seed,
                            (uint32_t)(A.seed >> 32));
        const int xs = x[i * A.B + b];
        const bool err = u01(r.v[0], r.v[1]) <= A.param;
        const int y = err ? (xs + 1 + (int)below(r.v[2], q - 1)) % q : xs;
        double* row = xy + row_at(A, i, b) * q;
        for (int t = 0; t < q; ++t) row[t] = t == y ? hit : miss;
    }
}

// Guard bands + deletion channel (Guardbands.addDeletionGuardBands, Guardbands.py:4-44;
// BinaryTrellis.deletionChannelSimulation, BinaryTrellis.py:441-461): symbol j of the
// guard-banded word is tmpl[j] >= 0 ? codeword bit tmpl[j] : (tmpl[j] == -2 ? 1 : 0); it survives
// iff its uniform (32-bit lane (j & 3) of counter (g, kStreamChannel, j >> 2)) is >= pd.  One
// thread per codeword packs the survivors into its row of rx [B][W].
__global__ __launch_bounds__(kMcBlock) void k_mc_deletion(McArgs A, const int32_t* tmpl, int W, const uint32_t* x,
                                                           uint8_t* rx, int32_t* rx_len) {
    const long long b = (long long)blockIdx.x * kMcBlock + threadIdx.x;
    if (b >= A.B) return;
    const uint64_t g = (uint64_t)(A.offset + b);
    uint8_t* row = rx + b * (long long)W;
    int o = 0;
    P4 r{{0, 0, 0, 0}};
    for (int j = 0; j < W; ++j) {
        if ((j & 3) == 0)
            r = philox((uint32_t)g, (uint32_t)(g >> 32), kStreamChannel, (uint32_t)(j >> 2), (uint32_t)A.seed,
                       (uint32_t)(A.seed >> 32));
        const double u = ((double)r.v[j & 3] + 0.5) * (1.0 / 4294967296.0);
        const int t = tmpl[j];
        const uint8_t v = t >= 0 ? (uint8_t)((x[(long long)(t >> 5) * A.B + b] >> (t & 31)) & 1u) : (uint8_t)(t == -2);
        if (u >= A.param) row[o++] = v;
    }
    for (int j = o; j < W; ++j) row[j] = 0;
    rx_len[b] = o;
}

}  // namespace

extern "C" int pcub_mc_info(uint64_t seed, int64_t offset, int64_t B, int32_t K, uint32_t* info_words, void* stream) {
    if (B < 0 || offset < 0 || K < 0 || (K > 0 && B > 0 && !info_words)) return PCUB_EINVAL;
    if (B == 0 || K == 0) return 0;
    McArgs A{seed, offset, B, 0, K, 0, 0.0, 0.0, 0.0, 0.0, 0};
    hipLaunchKernelGGL(k_mc_info, dim3(grid_of(B)), dim3(kMcBlock), 0, (hipStream_t)stream, A, info_words);
    return (int)hipGetLastError();
}

extern "C" int pcub_mc_channel_tiled(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel,
                                     double param, const uint32_t* x_words, double* xy, int32_t tile, void* stream) {
    if (B < 0 || offset < 0 || log2N < 0 || log2N > 24 || (channel != 0 && channel != 1)) return PCUB_EINVAL;
    if (tile < 0 || tile > 4096) return PCUB_EINVAL;
    if (channel == 0 && !(param > 0.0)) return PCUB_EINVAL;
    if (channel == 1 && !(param >= 0.0 && param <= 1.0)) return PCUB_EINVAL;
    if (B == 0) return 0;
    if (!x_words || !xy) return PCUB_EINVAL;
    McArgs A{seed, offset, B, log2N, 0, channel, param, 0.0, 0.0, 0.0, tile};
    if (channel == 0) {
        A.sigma = sqrt(param);
        A.inv2s2 = 1.0 / (2.0 * param);
        A.dens = 0.5 / sqrt(6.283185307179586 * param);
    }
    // ~16 k workgroups in total, y capped by the number of element pairs
    const long long gx = (B + kMcBlock - 1) / kMcBlock;
    const long long pairs = (((long long)1 << log2N) + 1) / 2;
    long long gy = (16384 + gx - 1) / gx;
    if (gy > pairs) gy = pairs;
    if (gy > 65535) gy = 65535;
    if (gx > 0x7fffffffLL) return PCUB_EINVAL;
    hipLaunchKernelGGL(k_mc_channel, dim3((unsigned)gx, (unsigned)gy), dim3(kMcBlock), 0, (hipStream_t)stream, A,
                       x_words, (double2*)xy);
    return (int)hipGetLastError();
}

extern "C" int pcub_mc_channel(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel, double param,
                               const uint32_t* x_words, double* xy, void* stream) {
    return pcub_mc_channel_tiled(seed, offset, B, log2N, channel, param, x_words, xy, 0, stream);
}

extern "C" int pcub_mc_channel_norm_tiled(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel,
                                          double param, const uint32_t* x_words, double* out, int32_t compact,
                                          int32_t tile, void* stream) {
    if (B < 0 || offset < 0 || log2N < 0 || log2N > 24 || (channel != 0 && channel != 1)) return PCUB_EINVAL;
    if (tile < 0 || tile > 4096) return PCUB_EINVAL;
    if (channel == 0 && !(param > 0.0)) return PCUB_EINVAL;
    if (channel == 1 && !(param >= 0.0 && param <= 1.0)) return PCUB_EINVAL;
    if (B == 0) return 0;
    if (!x_words || !out) return PCUB_EINVAL;
    McArgs A{seed, offset, B, log2N, 0, channel, param, 0.0, 0.0, 0.0, tile};
    if (channel == 0) {
        A.sigma = sqrt(param);
        A.inv2s2 = 1.0 / (2.0 * param);
    }
    const long long gx = (B + kMcBlock - 1) / kMcBlock;
    const long long quads = (((long long)1 << log2N) + 3) / 4;
    long long gy = (16384 + gx - 1) / gx;
    if (gy > quads) gy = quads;
    if (gy > 65535) gy = 65535;
    if (gx > 0x7fffffffLL) return PCUB_EINVAL;
    if (compact)
        hipLaunchKernelGGL(k_mc_channel_norm<true>, dim3((unsigned)gx, (unsigned)gy), dim3(kMcBlock), 0,
                           (hipStream_t)stream, A, x_words, out);
    else
        hipLaunchKernelGGL(k_mc_channel_norm<false>, dim3((unsigned)gx, (unsigned)gy), dim3(kMcBlock), 0,
                           (hipStream_t)stream, A, x_words, out);
    return (int)hipGetLastError();
}

extern "C" int pcub_mc_channel_norm(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel,
                                    double param, const uint32_t* x_words, double* out, int32_t compact, void* stream) {
    return pcub_mc_channel_norm_tiled(seed, offset, B, log2N, channel, param, x_words, out, compact, 0, stream);
}

extern "C" int pcub_mc_info_qary(uint64_t seed, int64_t offset, int64_t B, int32_t K, int32_t q, uint8_t* info,
                                 void* stream) {
    if (B < 0 || offset < 0 || K < 0 || q < 2 || q > 255 || (K > 0 && B > 0 && !info)) return PCUB_EINVAL;
    if (B == 0 || K == 0) return 0;
    McArgs A{seed, offset, B, 0, K, 0, 0.0, 0.0, 0.0, 0.0, 0};
    hipLaunchKernelGGL(k_mc_info_qary, dim3(grid_of(B)), dim3(kMcBlock), 0, (hipStream_t)stream, A, (int)q, info);
    return (int)hipGetLastError();
}

extern "C" int pcub_mc_channel_qsc_tiled(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t q, double p,
                                         const uint8_t* x, double* xy, int32_t tile, void* stream) {
    if (B < 0 || offset < 0 || log2N < 0 || log2N > 24 || q < 2 || q > 255 || !(p >= 0.0 && p <= 1.0))
        return PCUB_EINVAL;
    if (tile < 0 || tile > 4096) return PCUB_EINVAL;
    if (B == 0) return 0;
    if (!x || !xy) return PCUB_EINVAL;
    McArgs A{seed, offset, B, log2N, 0, 2, p, 0.0, 0.0, 0.0, tile};
    const long long gx = (B + kMcBlock - 1) / kMcBlock;
    long long gy = (16384 + gx - 1) / gx;
    if (gy > ((long long)1 << log2N)) gy = (long long)1 << log2N;
    if (gy > 65535) gy = 65535;
    if (gx > 0x7fffffffLL) return PCUB_EINVAL;
    hipLaunchKernelGGL(k_mc_qsc, dim3((unsigned)gx, (unsigned)gy), dim3(kMcBlock), 0, (hipStream_t)stream, A, (int)q,
                       x, xy);
    return (int)hipGetLastError();
}

extern "C" int pcub_mc_channel_qsc(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t q, double p,
                                   const uint8_t* x, double* xy, void* stream) {
    return pcub_mc_channel_qsc_tiled(seed, offset, B, log2N, q, p, x, xy, 0, stream);
}

extern "C" int pcub_mc_deletion(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, const int32_t* tmpl,
                                int32_t W, double pd, const uint32_t* x_words, uint8_t* rx, int32_t* rx_len,
                                void* stream) {
    if (B < 0 || offset < 0 || log2N < 0 || log2N > 24 || W < 0 || !(pd >= 0.0 && pd <= 1.0)) return PCUB_EINVAL;
    if (B == 0) return 0;
    if (!tmpl || !x_words || !rx || !rx_len) return PCUB_EINVAL;
    McArgs A{seed, offset, B, log2N, 0, 3, pd, 0.0, 0.0, 0.0, 0};
    hipLaunchKernelGGL(k_mc_deletion, dim3(grid_of(B)), dim3(kMcBlock), 0, (hipStream_t)stream, A, tmpl, (int)W,
                       x_words, rx, rx_len);
    return (int)hipGetLastError();
}

extern "C" int pcub_mc_count_errors(const uint32_t* decoded_words, const uint32_t* sent_words, int64_t B, int32_t K,
                                    uint64_t* counters, void* stream) {
    if (B < 0 || K < 0 || !counters || (B > 0 && K > 0 && (!decoded_words || !sent_words))) return PCUB_EINVAL;
    if (B == 0) return 0;
    const int W = (K + 31) / 32;
    if (W == 0) {
        // no information bits: only the codeword count moves
        hipLaunchKernelGGL(k_mc_count, dim3(1), dim3(kMcBlock), 0, (hipStream_t)stream, decoded_words, sent_words,
                           (long long)B, 0, (unsigned long long*)counters);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(k_mc_count, dim3(grid_of(B)), dim3(kMcBlock), 0, (hipStream_t)stream, decoded_words, sent_words,
                       (long long)B, W, (unsigned long long*)counters);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// mc_run: the whole Monte-Carlo pipeline for codewords [offset, offset + count)
// in chunks -- information bits -> polar encoder -> channel (normalised rows, compact) ->
// SC decode (compact root) -> error counters -- all stream-ordered on the device.

namespace {

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// One generation slot (information words, channel rows), the codewords x and the decisions.  The
// chunks run back to back on the caller's stream: round 3 generated chunk i+1 on a side stream while
// chunk i decoded, and once the channel kernel got cheap that overlap measured slower than none
// (C2, 2^20 codewords in chunks of 2^18: 56.5 M cw/s overlapped, 65.3 M serial, median of 5;
// the decode holds the register file and the concurrent generation only takes its CUs).
struct McLayout {
    size_t info, x, xy, dec, dws, total;
};

// the compact-root decode exists for the variant this code length runs (sc_bin.hip); otherwise the
// pipeline generates normalised pair rows (16 bytes a position) for the pair decode instead of
// letting the compact entry expand them into a second chunk-sized buffer
bool mc_compact(int32_t log2N) { return pcub_sc_decode_bin_compact_direct(log2N) == 1; }

// the generation writes the rows in the decode kernel's tiles (pcub_sc_bin_tile: one wave's codewords
// contiguous), padded to whole tiles
int mc_tile(int32_t log2N) { return pcub_sc_bin_tile(log2N); }

McLayout mc_layout(int64_t chunk, int32_t log2N, int32_t K) {
    McLayout L;
    const size_t N = (size_t)1 << log2N;
    const size_t row = mc_compact(log2N) ? 8 : 16;  // bytes a position: compact row or pair
    const int T = mc_tile(log2N);
    const size_t cp = (size_t)((chunk + T - 1) / T) * T;  // the chunk padded to whole tiles
    const size_t iw = (size_t)((K + 31) / 32 > 0 ? (K + 31) / 32 : 1);
    const size_t nw = (N + 31) / 32;
    L.info = 0;
    L.x = L.info + align256(iw * chunk * 4);
    L.xy = L.x + align256(nw * chunk * 4);
    L.dec = L.xy + align256(N * cp * row);
    L.dws = L.dec + align256(iw * chunk * 4);
    L.total = L.dws + align256(mc_compact(log2N) ? pcub_sc_decode_bin_compact_workspace(chunk, log2N)
                                                 : pcub_sc_decode_bin_workspace(chunk, log2N));
    return L;
}

}  // namespace

extern "C" size_t pcub_mc_run_bin_workspace(int64_t chunk, int32_t log2N, int32_t K) {
    if (chunk <= 0 || log2N < 0 || log2N > 20 || K < 0 || K > (1 << log2N)) return 0;
    return mc_layout(chunk, log2N, K).total;
}

extern "C" int pcub_mc_run_bin(uint64_t seed, int64_t offset, int64_t count, int32_t log2N, int32_t channel,
                               double param, const uint32_t* frozen_mask, const uint32_t* frozen_val, int32_t K,
                               int64_t chunk, uint64_t* counters, void* workspace, size_t workspace_bytes, void* stream) {
    if (count < 0 || offset < 0 || chunk <= 0 || !counters || !frozen_mask || !frozen_val) return PCUB_EINVAL;
    if (log2N < 0 || log2N > 20) return PCUB_EINVAL;
    const McLayout L = mc_layout(chunk, log2N, K);
    if (!workspace || workspace_bytes < L.total) return PCUB_EINVAL;
    const bool compact = mc_compact(log2N);
    const int T = mc_tile(log2N);
    char* ws = (char*)workspace;
    uint32_t* x = (uint32_t*)(ws + L.x);
    uint32_t* dec = (uint32_t*)(ws + L.dec);
    const hipStream_t ms = (hipStream_t)stream;
    uint32_t* info = (uint32_t*)(ws + L.info);
    double* xy = (double*)(ws + L.xy);
    int rc = 0;
    for (int64_t c0 = 0; !rc && c0 < count; c0 += chunk) {
        const int64_t B = (count - c0) < chunk ? (count - c0) : chunk;
        if (K > 0 && (rc = pcub_mc_info(seed, offset + c0, B, K, info, ms))) break;
        if ((rc = pcub_polar_encode_bin(info, B, log2N, frozen_mask, frozen_val, K, x, ms))) break;
        // normalised rows in compact form (8 bytes a position) into the compact-root decode, or as
        // pairs where this code length has no compact-root kernel
        if ((rc = pcub_mc_channel_norm_tiled(seed, offset + c0, B, log2N, channel, param, x, xy, compact ? 1 : 0, T,
                                             ms)))
            break;
        if (compact)
            rc = pcub_sc_decode_bin_compact_tiled(xy, B, log2N, T, frozen_mask, frozen_val, K, dec, nullptr, nullptr,
                                                  ws + L.dws, L.total - L.dws, ms);
        else
            rc = pcub_sc_decode_bin_tiled(xy, B, log2N, T, frozen_mask, frozen_val, K, dec, nullptr, nullptr,
                                          ws + L.dws, L.total - L.dws, ms);
        if (rc) break;
        rc = pcub_mc_count_errors(dec, info, B, K, counters, ms);
    }
    return rc;
}

// ---------------------------------------------------------------------------
// mc_run for the q-ary and deletion workloads (mc_run(cfg, seed, cw_offset, count) ->
// counters): the same chunked, stream-ordered chain as pcub_mc_run_bin over the generators the
// parity tests use, so a run's counters are what composing those calls counts.

namespace {

struct QLayout {
    size_t info, x, xy, dec, dws, total;
};

QLayout q_layout(int64_t chunk, int32_t log2N, int32_t q, int32_t K) {
    QLayout L;
    const size_t N = (size_t)1 << log2N;
    const int T = pcub_sc_qary_tile(q, log2N);
    const size_t cp = (size_t)((chunk + T - 1) / T) * T;
    const size_t kk = (size_t)(K > 0 ? K : 1);
    L.info = 0;
    L.x = L.info + align256(kk * chunk);
    L.xy = L.x + align256(N * chunk);
    L.dec = L.xy + align256(N * cp * q * 8);
    L.dws = L.dec + align256(kk * chunk);
    L.total = L.dws + align256(pcub_sc_decode_qary_workspace((int64_t)cp, log2N, q));
    return L;
}

struct DLayout {
    size_t info, x, rx, len, dec, total;
};

DLayout d_layout(int64_t chunk, int32_t n, int32_t W, int32_t K) {
    DLayout L;
    const size_t iw = (size_t)((K + 31) / 32 > 0 ? (K + 31) / 32 : 1);
    const size_t nw = (((size_t)1 << n) + 31) / 32;
    L.info = 0;
    L.x = L.info + align256(iw * chunk * 4);
    L.rx = L.x + align256(nw * chunk * 4);
    L.len = L.rx + align256((size_t)W * chunk);
    L.dec = L.len + align256((size_t)chunk * 4);
    L.total = L.dec + align256(iw * chunk * 4);
    return L;
}

}  // namespace

extern "C" size_t pcub_mc_run_qary_workspace(int64_t chunk, int32_t log2N, int32_t q, int32_t K) {
    if (chunk <= 0 || pcub_sc_qary_tile(q, log2N) <= 0 || K < 0 || K > (1 << log2N)) return 0;
    return q_layout(chunk, log2N, q, K).total;
}

extern "C" int pcub_mc_run_qary(uint64_t seed, int64_t offset, int64_t count, int32_t log2N, int32_t q, double p,
                                const uint8_t* frozen, int32_t K, int64_t chunk, uint64_t* counters, void* workspace,
                                size_t workspace_bytes, void* stream) {
    if (count < 0 || offset < 0 || chunk <= 0 || !counters || !frozen) return PCUB_EINVAL;
    const int T = pcub_sc_qary_tile(q, log2N);
    if (T <= 0 || K < 0 || K > (1 << log2N) || !(p >= 0.0 && p <= 1.0)) return PCUB_EINVAL;
    const QLayout L = q_layout(chunk, log2N, q, K);
    if (!workspace || workspace_bytes < L.total) return PCUB_EINVAL;
    char* ws = (char*)workspace;
    uint8_t* info = (uint8_t*)(ws + L.info);
    uint8_t* x = (uint8_t*)(ws + L.x);
    double* xy = (double*)(ws + L.xy);
    uint8_t* dec = (uint8_t*)(ws + L.dec);
    const hipStream_t ms = (hipStream_t)stream;
    int rc = 0;
    for (int64_t c0 = 0; !rc && c0 < count; c0 += chunk) {
        const int64_t B = (count - c0) < chunk ? (count - c0) : chunk;
        if (K > 0 && (rc = pcub_mc_info_qary(seed, offset + c0, B, K, q, info, ms))) break;
        if ((rc = pcub_polar_encode_qary(info, B, log2N, q, frozen, K, x, ms))) break;
        if ((rc = pcub_mc_channel_qsc_tiled(seed, offset + c0, B, log2N, q, p, x, xy, T, ms))) break;
        if ((rc = pcub_sc_decode_qary_tiled(xy, B, log2N, q, T, frozen, K, dec, nullptr, ws + L.dws, L.total - L.dws,
                                            ms)))
            break;
        if (K == 0) {
            hipLaunchKernelGGL(k_mc_count_sym, dim3(1), dim3(kMcBlock), 0, ms, dec, info, (long long)B, 0,
                               (unsigned long long*)counters);
        } else {
            hipLaunchKernelGGL(k_mc_count_sym, dim3(grid_of(B)), dim3(kMcBlock), 0, ms, dec, info, (long long)B, (int)K,
                               (unsigned long long*)counters);
        }
        rc = (int)hipGetLastError();
    }
    return rc;
}

extern "C" size_t pcub_mc_run_deletion_workspace(int64_t chunk, int32_t n, int32_t W, int32_t K) {
    if (chunk <= 0 || n < 1 || n > 24 || W < 0 || K < 0 || K > (1 << n)) return 0;
    return d_layout(chunk, n, W, K).total;
}

extern "C" int pcub_mc_run_deletion(uint64_t seed, int64_t offset, int64_t count, int32_t n, int32_t n0,
                                    const int32_t* tmpl, int32_t W, int32_t ones, double pd,
                                    const uint32_t* frozen_mask, const uint32_t* frozen_val, int32_t K,
                                    const double* table, int64_t chunk, uint64_t* counters, void* workspace,
                                    size_t workspace_bytes, void* stream) {
    if (count < 0 || offset < 0 || chunk <= 0 || !counters || !frozen_mask || !frozen_val || !tmpl || W <= 0)
        return PCUB_EINVAL;
    if (!pcub_sc_deletion_supported(n, n0, ones) || K < 0 || K > (1 << n) || !(pd >= 0.0 && pd <= 1.0))
        return PCUB_EINVAL;
    const DLayout L = d_layout(chunk, n, W, K);
    if (!workspace || workspace_bytes < L.total) return PCUB_EINVAL;
    char* ws = (char*)workspace;
    uint32_t* info = (uint32_t*)(ws + L.info);
    uint32_t* x = (uint32_t*)(ws + L.x);
    uint8_t* rx = (uint8_t*)(ws + L.rx);
    int32_t* len = (int32_t*)(ws + L.len);
    uint32_t* dec = (uint32_t*)(ws + L.dec);
    const hipStream_t ms = (hipStream_t)stream;
    int rc = 0;
    for (int64_t c0 = 0; !rc && c0 < count; c0 += chunk) {
        const int64_t B = (count - c0) < chunk ? (count - c0) : chunk;
        if (K > 0 && (rc = pcub_mc_info(seed, offset + c0, B, K, info, ms))) break;
        if ((rc = pcub_polar_encode_bin(info, B, n, frozen_mask, frozen_val, K, x, ms))) break;
        if ((rc = pcub_mc_deletion(seed, offset + c0, B, n, tmpl, W, pd, x, rx, len, ms))) break;
        if ((rc = pcub_sc_decode_deletion_tab(rx, len, B, W, n, n0, ones, pd, frozen_mask, frozen_val, K, dec, nullptr,
                                              table, ms)))
            break;
        rc = pcub_mc_count_errors(dec, info, B, K, counters, ms);
    }
    return rc;
}
