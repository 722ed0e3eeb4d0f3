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
// The per-codeword schedule (register subtrees, fused chain passes, rate-0
// skipping, G lanes per codeword) is in sc_qary_body.h; this file owns the
// launch geometry: G lanes per codeword (default 4, fewer for short codes),
// 256-thread workgroups, a resident grid striding over 256/G-codeword tiles so
// the per-slot stage buffers are reused.
#include <hip/hip_runtime.h>

#include "polarcub_sc.h"
#include "sc_qary_kern.h"

using namespace pcub;

namespace {

constexpr int kQBlock = kQaryBlock;

// rate-0 table: frozen bytes -> words -> first all-frozen depth per register subtree
__global__ __launch_bounds__(kQBlock) void k_q_frozen_words(const uint8_t* frozen, int N, uint32_t* words) {
    const int w = blockIdx.x * kQBlock + threadIdx.x;
    if (w >= (N + 31) / 32) return;
    uint32_t o = 0;
    for (int t = 0; t < 32 && 32 * w + t < N; ++t) o |= (uint32_t)(frozen[32 * w + t] != 0) << t;
    words[w] = o;
}

__global__ __launch_bounds__(kQBlock) void k_q_ef(const uint32_t* words, int D, int S, uint8_t* ef,
                                                unsigned long long* wtiles) {
    const int k = blockIdx.x * kQBlock + threadIdx.x;
    if (k < (1 << D)) ef[k] = (uint8_t)first_frozen_depth(words, k, D, S);
    if (k == 0) *wtiles = 0;  // the decode's wave-tile counter (QArgs::wtiles), before it on the stream
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

// A/B experiments (sc_bin.hip's hook, scripts/exp_build.sh): a candidate split-level tiled-root
// kernel linked in as pcub_exp_qkernel, launched while pcub_sc_set_experiment selects it
extern "C" __attribute__((weak)) void* pcub_exp_qkernel(int e, int q, int S, int G);
extern "C" int pcub_sc_experiment(void);
extern "C" int pcub_sc_fixed_n(void);  // sc_bin.hip: the code-length-specialised twins allowed
extern "C" int pcub_sc_dynamic_tiles(void);  // sc_bin.hip: wave tiles from a counter

int g_qlanes = 4;  // requested lanes per codeword (pcub_sc_set_qary_lanes)
int g_qylds = 1;   // symbols in LDS where a twin kernel exists and fits (pcub_sc_set_qary_lds)
constexpr size_t kQLdsPerCu = 160 * 1024;
int g_qregs = 0;   // cap on register positions per lane (pcub_sc_set_qary_regs; 0 = the default)
int g_qhl = 1;     // split last level (HL twin) where one exists and fits (pcub_sc_set_qary_hl)
int g_qtr = 1;     // the uniform-base twin for rows in the wave's own tiles (pcub_sc_set_qary_tiled_root)

// register positions per lane S and lanes per codeword G for a code of 2^n:
// S = 8 (q <= 4) or 4, G = the requested lanes, both reduced until N >= 2*S*G
struct QGeom {
    int S, G;
    bool yl;  // symbols in LDS
    bool hl;  // split last level: 2S positions per lane at the chain's end, S of them in LDS
    int sr() const { return hl ? 2 * S : S; }
};

// symbols per 32-bit word (QPack): 16 two-bit fields at q = 4, else four bytes
int qsym_per_word(int q) { return q == 4 ? 16 : 4; }
// LDS bytes of a workgroup's symbols: ceil(Nv / per-word) words per thread
size_t qsym_lds_bytes(int n, int G, int q) {
    const size_t per = (size_t)qsym_per_word(q);
    return (size_t)kQBlock * ((((size_t)1 << n) / G + per - 1) / per) * sizeof(uint32_t);
}
// LDS bytes of the split level's LDS half: S positions x q doubles per thread
size_t qhl_lds_bytes(int q, int S) { return (size_t)kQBlock * S * q * sizeof(double); }
// the HL kernels' launch bounds: three workgroups a CU (q = 4: 4 KB of 2-bit symbols + 32 KB of the
// split level a workgroup would let four share the LDS, but the registers allow three)
// (S = 8, q = 4: 64 KB of split level a workgroup, two a CU)
int q_hl_waves(int q, int S) { return q * S >= 32 ? 2 : 3; }

QGeom q_geom(int q, int n) {
    QGeom c{4, g_qlanes, false, false};  // 8 register positions (q <= 4) via pcub_sc_set_qary_regs
    if (g_qregs > 0) c.S = (q <= 4 || g_qregs <= 4) ? g_qregs : 4;
    while (c.G > 1 && (1 << n) < 2 * c.S * c.G) c.G >>= 1;
    while (c.S > 1 && (1 << n) < 2 * c.S * c.G) c.S >>= 1;
    // G = 8, 16 are instantiated for some (q, S) only: otherwise four lanes
    if (c.G > 4 && !qary_kernel(q, c.S, c.G)) {
        c.G = 4;
        while (c.G > 1 && (1 << n) < 2 * c.S * c.G) c.G >>= 1;
    }
    // symbols in LDS while the resident workgroups' columns fit the CU's LDS (N <= 512 at G = 4)
    c.yl = g_qylds && qary_kernel_y(q, c.S, c.G) &&
           (size_t)qary_waves(q, c.S, c.G) * qsym_lds_bytes(n, c.G, q) <= kQLdsPerCu;
    // the split level (with the symbols in LDS) where its three workgroups fit a CU and the code
    // has an outer level above it (N >= 4 S G)
    c.hl = c.yl && g_qhl && qary_kernel_h(q, c.S, c.G) && (1 << n) >= 4 * c.S * c.G &&
           (size_t)q_hl_waves(q, c.S) * (qsym_lds_bytes(n, c.G, q) + qhl_lds_bytes(q, c.S)) <= kQLdsPerCu;
    return c;
}

QKern qkernel(int q, int n, int* waves = nullptr) {
    const QGeom c = q_geom(q, n);
    if (waves) *waves = c.hl ? q_hl_waves(q, c.S) : qary_waves(q, c.S, c.G);
    if (c.hl) return qary_kernel_h(q, c.S, c.G);
    return c.yl ? qary_kernel_y(q, c.S, c.G) : qary_kernel(q, c.S, c.G);
}

size_t qlaunch_lds(int q, int n) {
    const QGeom c = q_geom(q, n);
    return (c.yl ? qsym_lds_bytes(n, c.G, q) : 0) + (c.hl ? qhl_lds_bytes(q, c.S) : 0);
}

long long qgrid(long long B, int q, int n) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    int waves = 1;
    const QKern kern = qkernel(q, n, &waves);
    const size_t lds = qlaunch_lds(q, n);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kQBlock, lds) != hipSuccess || occ < 1) occ = 1;
    // the launch bounds guarantee `waves` resident workgroups per CU (the occupancy
    // query under-reports these kernels on ROCm 7.2)
    const QGeom cg = q_geom(q, n);
    if (occ < waves) occ = waves;
    if (lds > 0 && (size_t)occ * lds > kQLdsPerCu) occ = (int)(kQLdsPerCu / lds);
    const long long cwb = kQBlock / cg.G;
    const long long ntiles = (B + cwb - 1) / cwb;
    const long long g = (long long)cus * occ;
    if (ntiles <= g) return ntiles;
    const long long rounds = (ntiles + g - 1) / g;  // whole rounds (as the binary launcher)
    return (ntiles + rounds - 1) / rounds;
}

// per lane: virtual stage levels 1..D-1 (Nv - 2 SR positions as pairs, SR = the chain-end
// level's positions) + Nv symbol bytes in words (unless the symbols are in LDS)
size_t qslot_bytes(int n, int q) {
    const QGeom c = q_geom(q, n);
    const size_t Nv = ((size_t)1 << n) / c.G;
    const size_t per = (size_t)qsym_per_word(q);
    return (Nv - 2 * c.sr()) * (size_t)((q + 1) / 2) * sizeof(double2) + (c.yl ? 0 : (Nv + per - 1) / per * 4);
}

int q_depth(int n, int q) {
    const QGeom c = q_geom(q, n);
    return n - __builtin_ctz((unsigned)(c.sr() * c.G));
}

// rate-0 table + packed frozen words, ahead of the slots, and 256 bytes for the wave-tile counter
size_t qtable_bytes(int n, int q) {
    const int D = q_depth(n, q);
    return (((((size_t)1 << n) + 31) / 32 * 4 + ((size_t)1 << D) + 255) & ~(size_t)255) + 256;
}

}  // namespace

extern "C" size_t pcub_sc_decode_qary_workspace(int64_t B, int32_t log2N, int32_t q) {
    if (B <= 0 || log2N < 2 || log2N > 20 || !qkernel(q, log2N)) return 0;
    return qtable_bytes(log2N, q) + (size_t)qgrid(B, q, log2N) * kQBlock * qslot_bytes(log2N, q);
}

namespace {

int decode_qary_impl(const double* xy, int64_t B, int32_t log2N, int32_t q, int32_t tile, const uint8_t* frozen,
                     int32_t K, uint8_t* info, uint8_t* xhat, void* workspace, size_t workspace_bytes, void* stream) {
    if (B < 0 || log2N < 2 || log2N > 20 || !qkernel(q, log2N) || !frozen || tile < 0 || tile > 4096) return PCUB_EINVAL;
    if (K < 0 || K > (1 << log2N) || (K > 0 && !info) || (B > 0 && !xy)) return PCUB_EINVAL;
    if (B == 0) return 0;
    long long g = qgrid(B, q, log2N);
    if (g <= 0) return (int)hipErrorNoDevice;
    const size_t per_block = (size_t)kQBlock * qslot_bytes(log2N, q);
    const size_t tb = qtable_bytes(log2N, q);
    if (!workspace || workspace_bytes < tb + per_block) return PCUB_EINVAL;
    if ((size_t)g * per_block > workspace_bytes - tb) g = (long long)((workspace_bytes - tb) / per_block);
    const int N = 1 << log2N;
    const QGeom c = q_geom(q, log2N);
    const int D = q_depth(log2N, q);
    hipStream_t st = (hipStream_t)stream;
    uint32_t* words = (uint32_t*)workspace;
    uint8_t* ef = (uint8_t*)workspace + ((size_t)N + 31) / 32 * 4;
    hipLaunchKernelGGL(k_q_frozen_words, dim3((unsigned)(((N + 31) / 32 + kQBlock - 1) / kQBlock)), dim3(kQBlock), 0, st,
                       frozen, N, words);
    unsigned long long* wtiles = (unsigned long long*)((char*)workspace + tb - 256);
    hipLaunchKernelGGL(k_q_ef, dim3((unsigned)(((1 << D) + kQBlock - 1) / kQBlock)), dim3(kQBlock), 0, st, words, D,
                       c.sr() * c.G, ef, wtiles);
    QArgs A;
    A.xy = xy;
    A.B = B;
    A.n = log2N;
    A.fwords = words;
    A.ef = ef;
    A.info = info;
    A.xhat = xhat;
    A.nslots = g * kQBlock;
    A.ylds_words = c.yl ? (int)(qsym_lds_bytes(log2N, c.G, q) / kQBlock / sizeof(uint32_t)) : 0;
    A.tile = tile;
    A.wtiles = pcub_sc_dynamic_tiles() ? wtiles : nullptr;
    char* slots = (char*)workspace + tb;
    A.scratch = (double2*)slots;
    A.ysym = c.yl ? nullptr : (uint32_t*)(slots + (size_t)A.nslots * (N / c.G - 2 * c.sr()) * ((q + 1) / 2) * sizeof(double2));
    // rows in the wave's own tiles: the uniform-base twin where one is instantiated
    QKern kern = nullptr;
    if (pcub_exp_qkernel && pcub_sc_experiment() && c.hl && tile == 64 / c.G)
        kern = (QKern)pcub_exp_qkernel(pcub_sc_experiment(), q, c.S, c.G);
    if (!kern && g_qtr && c.hl && tile == 64 / c.G && q == 4 && pcub_sc_fixed_n())
        kern = qary_kernel_q4_h_tr_n(c.S, c.G, log2N);
    if (!kern && g_qtr && c.hl && tile == 64 / c.G) kern = qary_kernel_h_tr(q, c.S, c.G);
    if (!kern) kern = qkernel(q, log2N);
    hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(kQBlock), qlaunch_lds(q, log2N), st, A);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" int pcub_sc_decode_qary(const double* xy, int64_t B, int32_t log2N, int32_t q, const uint8_t* frozen,
                                   int32_t K, uint8_t* info, uint8_t* xhat, void* workspace, size_t workspace_bytes,
                                   void* stream) {
    return decode_qary_impl(xy, B, log2N, q, 0, frozen, K, info, xhat, workspace, workspace_bytes, stream);
}

// the codewords one wave of the q-ary kernel at (q, 2^log2N) decodes: the native tile width
extern "C" int pcub_sc_qary_tile(int32_t q, int32_t log2N) {
    if (log2N < 2 || log2N > 20 || !qkernel(q, log2N)) return PCUB_EINVAL;
    return 64 / q_geom(q, log2N).G;
}

extern "C" int pcub_sc_decode_qary_tiled(const double* xy, int64_t B, int32_t log2N, int32_t q, int32_t tile,
                                         const uint8_t* frozen, int32_t K, uint8_t* info, uint8_t* xhat,
                                         void* workspace, size_t workspace_bytes, void* stream) {
    return decode_qary_impl(xy, B, log2N, q, tile, frozen, K, info, xhat, workspace, workspace_bytes, stream);
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

// Tuning hook (not part of the stable ABI): lanes per codeword of the q-ary
// decode kernel (1, 2, 4, 8 or 16; reduced for short codes, 8 and 16 where instantiated).
// Returns the previous value.
extern "C" int pcub_sc_set_qary_lanes(int G) {
    if (G != 1 && G != 2 && G != 4 && G != 8 && G != 16) return PCUB_EINVAL;
    const int old = g_qlanes;
    g_qlanes = G;
    return old;
}

// Tuning hook (not part of the stable ABI): re-encoded symbols in LDS where a kernel for it
// exists and fits (1, the default) or in the per-slot workspace (0).  Returns the previous value.
extern "C" int pcub_sc_set_qary_lds(int on) {
    if (on != 0 && on != 1) return PCUB_EINVAL;
    const int old = g_qylds;
    g_qylds = on;
    return old;
}

// Tuning hook (not part of the stable ABI): the split last level (q = 4 HL kernel, three waves)
// where it exists and fits (1, the default) or not (0).  Returns the previous value.
extern "C" int pcub_sc_set_qary_hl(int on) {
    if (on != 0 && on != 1) return PCUB_EINVAL;
    const int old = g_qhl;
    g_qhl = on;
    return old;
}

// Tuning hook (not part of the stable ABI): cap on the register positions per lane of
// the q-ary decode kernel (0 = default: 8 for q <= 4, else 4; otherwise 2 or 4).
// Returns the previous value.
// Tuning hook (not part of the stable ABI): allow (1, the default) or forbid (0) the uniform-base
// twin for rows in the wave's own tiles.  Returns the previous value.
extern "C" int pcub_sc_set_qary_tiled_root(int on) {
    const int old = g_qtr;
    g_qtr = on ? 1 : 0;
    return old;
}

extern "C" int pcub_sc_set_qary_regs(int S) {
    if (S != 0 && S != 2 && S != 4 && S != 8) return PCUB_EINVAL;
    const int old = g_qregs;
    g_qregs = S;
    return old;
}
