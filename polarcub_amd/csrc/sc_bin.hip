// sc_bin.hip -- binary SC decode kernels for gfx950 + their C-ABI launchers.
//
// pcub_sc_decode_bin replaces BinaryPolarEncoderDecoder.decode
// (BinaryPolarEncoderDecoder.py:71-99) for a batch of codewords with a uniform
// a-priori distribution.  The schedule is in sc_bin_body.h; this file owns the
// launch geometry:
//   * 256-thread workgroups, one codeword per lane;
//   * a resident ("persistent") grid of CUs x occupancy workgroups that
//     strides over 256-codeword tiles, so the per-slot stage buffers are reused
//     and stay warm in L2 / Infinity Cache instead of being re-allocated per
//     codeword;
//   * padding lanes of the last tile decode a duplicate codeword and store
//     nothing, so every wave runs the same schedule.
#include <hip/hip_runtime.h>

#include <atomic>

#include "polarcub_sc.h"
#include "sc_bin_kern.h"

using namespace pcub;

// A/B experiments: a candidate kernel compiled outside the library build (its own translation unit,
// namespace and header copies; scripts/exp_build.sh) and linked in as pcub_exp_kernel, launched
// instead of the tiled-root twin while pcub_sc_set_experiment(e) selects it (scripts/ab_exp.py times
// both and compares their outputs).  Diagnostic hook, not the ABI: the shipped library has no
// pcub_exp_kernel (a weak reference, null), so the hook launches nothing.
extern "C" __attribute__((weak)) void* pcub_exp_kernel(int e, int v, int compact);
static BinKernFn exp_kernel(int e, int v, bool compact) {
    return pcub_exp_kernel ? (BinKernFn)pcub_exp_kernel(e, v, compact ? 1 : 0) : nullptr;
}
static std::atomic<int> g_experiment{0};
// the q-ary decode's twin compiled for its code length (sc_qary_q4.hip) where one exists (diagnostic
// A/B switch, not the ABI: pcub_sc_set_fixed_n(0) runs the generic kernels; identical outputs).  The
// binary tiled-root twins specialised the same way (N = 1024, 4096) measured slower -- 100.8 -> 99.6 M
// and 17.9 -> 16.1 M cw/s: SGPR spills 508 -> 20 but VGPR spills 50 -> 74 -- and were removed (round 6).
static std::atomic<int> g_fixed_n{1};
// the decode kernels' work tiles from a counter (BinArgs / QArgs / DelArgs::wtiles) instead of a static
// stride (diagnostic A/B switch, not the ABI: pcub_sc_set_dynamic_tiles(0) runs the static stride;
// identical outputs).  C2 98.5 -> 109.7 M cw/s, N = 4096 17.6 -> 18.9 M (round 6).
static std::atomic<int> g_dyn_tiles{1};
extern "C" int pcub_sc_set_dynamic_tiles(int on) { return g_dyn_tiles.exchange(on ? 1 : 0); }
extern "C" int pcub_sc_dynamic_tiles(void) { return g_dyn_tiles.load(std::memory_order_relaxed); }
extern "C" int pcub_sc_set_fixed_n(int on) { return g_fixed_n.exchange(on ? 1 : 0); }
extern "C" int pcub_sc_fixed_n(void) { return g_fixed_n.load(std::memory_order_relaxed); }
extern "C" int pcub_sc_set_experiment(int e) {
    const int old = g_experiment.exchange(e);
    return old;
}
// the selected experiment, for the q-ary launcher's hook (sc_qary.hip)
extern "C" int pcub_sc_experiment(void) { return g_experiment; }

namespace {

constexpr int kBlock = kBinBlock;

// rate-0 table: one byte per register subtree (first_frozen_depth); information-bit compress masks:
// eight words per frozen-mask word (compress_masks)
__global__ __launch_bounds__(kBlock) void k_ef_table(const uint32_t* fmask, int D, int SU, uint8_t* ef, int nwords,
                                                     uint32_t* cmask, unsigned long long* wtiles) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k < (1 << D)) ef[k] = (uint8_t)first_frozen_depth(fmask, k, D, SU);
    if (k < nwords) compress_masks(fmask[k], cmask + 8 * k);
    if (k == 0) *wtiles = 0;  // the decode's wave-tile counter (BinArgs::wtiles), before the decode on the stream
}

template <int NN>
__global__ __launch_bounds__(kBlock) void k_sc_bin_small(BinArgs A) {
    const long long cw = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (cw < A.B) decode_small<NN>(A, cw, true);
}

typedef BinKernFn KernFn;
KernFn variant_kernel(int v) {
    if (KernFn k = bin_kernel_part0(v)) return k;
    if (KernFn k = bin_kernel_part1(v)) return k;
    if (KernFn k = bin_kernel_part2(v)) return k;
    if (KernFn k = bin_kernel_part4(v)) return k;
    if (KernFn k = bin_kernel_part8(v)) return k;
    return bin_kernel_part5(v);
}

// {32, 4, 2, NT, re-encoded bits in LDS, split last level, prefetch 2}: at N=1024 one stored
// stage depth fewer than variant 24 (48.7 vs 68.6 KB/cw of HBM traffic) at 2 waves/SIMD,
// 76.3 vs 73.7 M cw/s (profiles/r3/); past its LDS budget (N > 1024 at G = 4) pick_variant
// falls back to 24 {32, 4, 3, NT, bits in LDS} (N = 4096: 13.3 M cw/s), then to 17
constexpr int kDefaultVariant = 26;
int g_variant = kDefaultVariant;
int g_tiled_root = 1;  // pcub_sc_set_tiled_root
int g_max_blocks = 0;  // workgroups per CU cap (0 = as many as fit)
constexpr size_t kLdsPerCu = 160 * 1024;

// dynamic LDS for variant v at code length 2^n: its stage level, its re-encoded bits, plus
// padding that caps residency at g_max_blocks
size_t launch_lds(int v, int n) {
    size_t b = bin_lds_bytes(v) + bin_ylds_bytes(v, n);
    if (g_max_blocks > 0) {
        const size_t cap = kLdsPerCu / (size_t)g_max_blocks;
        if (cap > b) b = cap - 256;
    }
    return b;
}

struct DevInfo {
    int dev = -1;
    int cus = 0;
    int occ[kNumVariants] = {};
};

DevInfo dev_info() {
    static thread_local DevInfo cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return DevInfo{};
    if (cache.dev == dev) return cache;
    DevInfo d;
    d.dev = dev;
    if (hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return DevInfo{};
    for (int v = 0; v < kNumVariants; ++v) {
        int occ = 0;
        const KernFn k = variant_kernel(v);
        if (!k || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kBlock, bin_lds_bytes(v)) != hipSuccess ||
            occ < 1)
            occ = 1;
        d.occ[v] = occ;
    }
    cache = d;
    return d;
}

// subtree depth D = log2(Nv / S) and the rate-0 table's bytes (256-aligned)
int tree_depth(int n, int v) {
    int g = 0;
    while ((1 << g) < kVar[v].G) ++g;
    int s = 0;
    while ((1 << s) < bin_sr(v)) ++s;
    return n - g - s;
}
size_t ef_only_bytes(int n, int v) { return (((size_t)1 << tree_depth(n, v)) + 255) & ~(size_t)255; }
size_t cmask_words(int n) { return n >= 5 ? ((size_t)1 << n) / 32 : 1; }
// + 256 bytes for the wave-tile counter at the end of the table area
size_t ef_bytes(int n, int v) { return ef_only_bytes(n, v) + ((cmask_words(n) * 32 + 255) & ~(size_t)255) + 256; }

// per-slot bytes: virtual levels 1..D-1 (Nv/2 - S pairs) + Nv local encoding bits (unless in LDS)
size_t slot_bytes(int n, int v) {
    const size_t Nv = ((size_t)1 << n) / kVar[v].G;
    return (Nv / 2 - bin_sr(v)) * sizeof(double2) + (kVar[v].Y ? 0 : (Nv / 32) * sizeof(uint32_t));
}

long long grid_for(long long B, int v, int n) {
    const DevInfo d = dev_info();
    if (d.cus <= 0) return 0;
    const long long cwb = kBlock / kVar[v].G;
    const long long ntiles = (B + cwb - 1) / cwb;
    int occ = d.occ[v];
    const size_t lds = launch_lds(v, n);
    if (lds > 0 && (size_t)occ * lds > kLdsPerCu) occ = (int)(kLdsPerCu / lds);
    if (occ < 1) occ = 1;
    if (g_max_blocks > 0 && g_max_blocks < occ) occ = g_max_blocks;
    long long g = (long long)d.cus * occ;
    return ntiles < g ? ntiles : g;
}

// a variant needs at least one outer level (N >= 2*S*G) and whole-word x_hat
// segments (N >= 32*G); otherwise fall back to the first variant of a
// decreasing-subtree list that fits (v1 = {8, 1} fits every N >= 64).
// A Y variant fits while its W workgroups' re-encoded bits fit the CU's LDS
// (N <= 4096 at G = 4); beyond that its non-LDS twin takes over.
bool fits(int v, int n) {
    const long long N = 1LL << n;
    if (kVar[v].Y && (size_t)kVar[v].W * launch_lds(v, n) > kLdsPerCu) return false;
    return N >= 2LL * bin_sr(v) * kVar[v].G && N >= 32LL * kVar[v].G;
}
int pick_variant(int n) {
    if (fits(g_variant, n)) return g_variant;
    // past the split level's LDS budget with the bits in LDS (N = 4096, 8192): the split level at G = 8
    // lanes a codeword (a node of 512 positions: one stored depth fewer than G = 4), with its bits in
    // LDS at N = 4096 (variant 30: 15.5 -> 17.8 M cw/s, 362 -> 314 KB/cw) and in the slot scratch at
    // N = 8192, 16384 (33: 6.1 -> 6.6 M; 2.28 -> 2.68 M over 17), round 6; before them the G = 4 split
    // level with the bits in scratch
    // (31: N = 4096 13.1 -> 14.1 M cw/s, N = 8192 5.2 -> 5.7 M over variant 24; equal to 17 at
    // N = 16384); N >= 32768 keeps variant 17 (not measured against 33)
    if (g_variant == kDefaultVariant) {
        if (n == 12 && fits(30, n)) return 30;
        if ((n == 13 || n == 14) && fits(33, n)) return 33;
        if (n <= 13 && fits(31, n)) return 31;
    }
    constexpr int kFallback[] = {24, 17, 13, 14, 10, 0, 1};
    for (int v : kFallback)
        if (fits(v, n)) return v;
    return 1;
}

}  // namespace

extern "C" int pcub_abi_version(void) { return 4; }

// Tuning hooks (not part of the stable ABI): choose / describe the decode kernel variant.
extern "C" int pcub_sc_num_variants(void) { return kNumVariants; }
extern "C" int pcub_sc_variant_info(int v, int* S, int* G, int* W) {
    if (v < 0 || v >= kNumVariants) return PCUB_EINVAL;
    *S = kVar[v].S;
    *G = kVar[v].G;
    *W = kVar[v].W * (kVar[v].L ? -1 : 1);  // negative: deepest stage level in LDS
    return 0;
}
extern "C" int pcub_sc_set_max_blocks_per_cu(int b) {
    if (b < 0 || b > 8) return PCUB_EINVAL;
    g_max_blocks = b;
    return 0;
}

extern "C" int pcub_sc_default_variant(void) { return kDefaultVariant; }
// Tuning hook (not part of the stable ABI): allow (1, the default) or forbid (0) the uniform-base
// twins for rows in the wave's own tiles (bin_kernel_tiled_root); returns the previous setting.
extern "C" int pcub_sc_set_tiled_root(int on) {
    const int old = g_tiled_root;
    g_tiled_root = on ? 1 : 0;
    return old;
}
// the variant a decode of code length 2^log2N launches (the selected one, or its fallback)
extern "C" int pcub_sc_variant_for(int32_t log2N) {
    if (log2N < 6 || log2N > 24) return PCUB_EINVAL;
    return pick_variant(log2N);
}
extern "C" int pcub_sc_set_variant(int v) {
    if (v < 0 || v >= kNumVariants || !variant_kernel(v)) return PCUB_EINVAL;  // not built: EINVAL
    g_variant = v;
    return 0;
}

extern "C" size_t pcub_sc_decode_bin_workspace(int64_t B, int32_t log2N) {
    if (B <= 0 || log2N < 0 || log2N > 24) return 0;
    if (log2N < 6) return 0;
    const int v = pick_variant(log2N);
    const long long g = grid_for(B, v, log2N);
    return ef_bytes(log2N, v) + (size_t)g * kBlock * slot_bytes(log2N, v);
}

namespace {

// raw pairs xy, or compact rows xc through a variant's compact-root twin (the caller checks one exists)
int decode_bin_impl(const double* xy, const double* xc, int64_t B, int32_t log2N, int32_t tile,
                    const uint32_t* frozen_mask, const uint32_t* frozen_val, int32_t K, uint32_t* info_words,
                    uint32_t* xhat_words, uint32_t* u_words, void* workspace, size_t workspace_bytes, void* stream) {
    if (B < 0 || log2N < 0 || log2N > 24 || tile < 0 || tile > 4096 || !frozen_mask || !frozen_val) return PCUB_EINVAL;
    if (K < 0 || K > (1 << log2N) || (K > 0 && !info_words) || (B > 0 && !xy && !xc)) return PCUB_EINVAL;
    if (B == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    BinArgs A;
    A.xy = (const double2*)xy;
    A.xc = xc;
    A.B = B;
    A.n = log2N;
    A.fmask = frozen_mask;
    A.fval = frozen_val;
    A.info = info_words;
    A.xhat = xhat_words;
    A.uout = u_words;
    A.scratch = nullptr;
    A.ybits = nullptr;
    A.nslots = 0;
    A.ef = nullptr;
    A.cmask = nullptr;
    A.tile = tile;
    if (log2N <= 5) {
        const dim3 grid((unsigned)((B + kBlock - 1) / kBlock));
        switch (log2N) {
            case 0: hipLaunchKernelGGL(k_sc_bin_small<1>, grid, dim3(kBlock), 0, st, A); break;
            case 1: hipLaunchKernelGGL(k_sc_bin_small<2>, grid, dim3(kBlock), 0, st, A); break;
            case 2: hipLaunchKernelGGL(k_sc_bin_small<4>, grid, dim3(kBlock), 0, st, A); break;
            case 3: hipLaunchKernelGGL(k_sc_bin_small<8>, grid, dim3(kBlock), 0, st, A); break;
            case 4: hipLaunchKernelGGL(k_sc_bin_small<16>, grid, dim3(kBlock), 0, st, A); break;
            default: hipLaunchKernelGGL(k_sc_bin_small<32>, grid, dim3(kBlock), 0, st, A); break;
        }
        return (int)hipGetLastError();
    }
    const int v = pick_variant(log2N);
    long long g = grid_for(B, v, log2N);
    if (g <= 0) return (int)hipErrorNoDevice;
    const size_t per_block = (size_t)kBlock * slot_bytes(log2N, v);
    if (!workspace) return PCUB_EINVAL;
    const size_t efb = ef_bytes(log2N, v);
    if (workspace_bytes < efb + per_block) return PCUB_EINVAL;
    if ((size_t)g * per_block > workspace_bytes - efb) g = (long long)((workspace_bytes - efb) / per_block);
    const long long nslots = g * kBlock;
    const size_t Nv = ((size_t)1 << log2N) / kVar[v].G;
    const int D = tree_depth(log2N, v);
    uint8_t* ef = (uint8_t*)workspace;
    uint32_t* cmask = (uint32_t*)((char*)workspace + ef_only_bytes(log2N, v));
    char* slots = (char*)workspace + efb;
    const int nw = (int)cmask_words(log2N);
    const int eft = (1 << D) > nw ? (1 << D) : nw;
    unsigned long long* wtiles = (unsigned long long*)((char*)workspace + efb - 256);
    hipLaunchKernelGGL(k_ef_table, dim3((unsigned)((eft + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, frozen_mask,
                       D, bin_sr(v) * kVar[v].G, ef, nw, cmask, wtiles);
    A.wtiles = g_dyn_tiles.load(std::memory_order_relaxed) ? wtiles : nullptr;
    A.ef = ef;
    A.cmask = cmask;
    A.nslots = nslots;
    A.scratch = (double2*)slots;
    A.ybits = kVar[v].Y ? nullptr : (uint32_t*)(slots + (size_t)nslots * (Nv / 2 - bin_sr(v)) * sizeof(double2));
    // rows in the wave's own tiles: the uniform-base twin where one is instantiated
    BinKernFn kern = nullptr;
    if (g_experiment && tile == 64 / kVar[v].G) kern = exp_kernel(g_experiment, v, xc != nullptr);
    if (!kern && g_tiled_root && tile == 64 / kVar[v].G) kern = bin_kernel_tiled_root(v, xc != nullptr);
    if (!kern && g_tiled_root && tile == 64 / kVar[v].G) kern = bin_kernel_tiled_root2(v, xc != nullptr);
    if (!kern) kern = xc ? bin_kernel_compact(v) : variant_kernel(v);
    if (!kern) return PCUB_EINVAL;
    hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(kBlock), launch_lds(v, log2N), st, A);
    return (int)hipGetLastError();
}

// compact normalised rows -> (1, r) / (r, 1) pairs; NaN -> (0, 0).  Grid-stride over a capped grid:
// B * N reaches past 2^32 work items (a 1-D dispatch's limit) at N >= 2^14 with 2^18-codeword chunks.
__global__ __launch_bounds__(kBlock) void k_expand_compact(const double* xc, long long count, double2* xy) {
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < count; i += (long long)gridDim.x * kBlock) {
        const double v = xc[i];
        const double r = __builtin_fabs(v);
        double2 o;
        if (v != v) o = double2{0.0, 0.0};
        else if (__builtin_signbit(v)) o = double2{r, 1.0};
        else o = double2{1.0, r};
        xy[i] = o;
    }
}

// the compact path runs a compact-root kernel when the variant picked for 2^n has one (and the
// code is past the small-code kernels); otherwise the rows are expanded into the workspace
bool compact_direct(int n) { return n > 5 && bin_kernel_compact(pick_variant(n)) != nullptr; }

}  // namespace

extern "C" int pcub_sc_decode_bin(const double* xy, int64_t B, int32_t log2N, const uint32_t* frozen_mask,
                                  const uint32_t* frozen_val, int32_t K, uint32_t* info_words, uint32_t* xhat_words,
                                  uint32_t* u_words, void* workspace, size_t workspace_bytes, void* stream) {
    if (!xy && B > 0) return PCUB_EINVAL;
    return decode_bin_impl(xy, nullptr, B, log2N, 0, frozen_mask, frozen_val, K, info_words, xhat_words, u_words,
                           workspace, workspace_bytes, stream);
}

// the codewords one wave of the kernel that runs at 2^log2N decodes (64 / lanes per codeword): the
// tile width whose root rows a wave reads as one contiguous block
extern "C" int pcub_sc_bin_tile(int32_t log2N) {
    if (log2N < 0 || log2N > 24) return PCUB_EINVAL;
    if (log2N <= 5) return 64;
    return 64 / kVar[pick_variant(log2N)].G;
}

extern "C" int pcub_sc_decode_bin_tiled(const double* xy, int64_t B, int32_t log2N, int32_t tile,
                                        const uint32_t* frozen_mask, const uint32_t* frozen_val, int32_t K,
                                        uint32_t* info_words, uint32_t* xhat_words, uint32_t* u_words, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    if (!xy && B > 0) return PCUB_EINVAL;
    return decode_bin_impl(xy, nullptr, B, log2N, tile, frozen_mask, frozen_val, K, info_words, xhat_words, u_words,
                           workspace, workspace_bytes, stream);
}

extern "C" int pcub_sc_decode_bin_compact_direct(int32_t log2N) {
    if (log2N < 0 || log2N > 24) return PCUB_EINVAL;
    return compact_direct(log2N) ? 1 : 0;
}

extern "C" size_t pcub_sc_decode_bin_compact_workspace(int64_t B, int32_t log2N) {
    if (B <= 0 || log2N < 0 || log2N > 24) return 0;
    const size_t w = pcub_sc_decode_bin_workspace(B, log2N);
    if (compact_direct(log2N)) return w;
    return ((w + 255) & ~(size_t)255) + (size_t)B * ((size_t)1 << log2N) * sizeof(double2);
}

namespace {

int decode_compact(const double* xc, int64_t B, int32_t log2N, int32_t tile, const uint32_t* frozen_mask,
                   const uint32_t* frozen_val, int32_t K, uint32_t* info_words, uint32_t* xhat_words,
                   uint32_t* u_words, void* workspace, size_t workspace_bytes, void* stream) {
    if (B < 0 || log2N < 0 || log2N > 24) return PCUB_EINVAL;
    if (B == 0) return 0;
    if (!xc || !workspace) return PCUB_EINVAL;
    if (compact_direct(log2N))
        return decode_bin_impl(nullptr, xc, B, log2N, tile, frozen_mask, frozen_val, K, info_words, xhat_words,
                               u_words, workspace, workspace_bytes, stream);
    const size_t w = pcub_sc_decode_bin_workspace(B, log2N);
    const size_t off = (w + 255) & ~(size_t)255;
    // element-wise: the pairs keep the rows' layout; a tiled layout spans whole tiles (the caller
    // sizes the workspace for the padded batch, pcub_sc_decode_bin_compact_workspace(ceil(B/T) T, n))
    const long long Bp = tile > 0 ? (B + tile - 1) / tile * tile : B;
    const long long count = Bp * (1LL << log2N);
    if (workspace_bytes < off + (size_t)count * sizeof(double2)) return PCUB_EINVAL;
    double2* xy = (double2*)((char*)workspace + off);
    const long long eb = (count + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_expand_compact, dim3((unsigned)(eb < 65536 ? eb : 65536)), dim3(kBlock), 0,
                       (hipStream_t)stream, xc, count, xy);
    if (hipGetLastError() != hipSuccess) return (int)hipErrorLaunchFailure;
    return decode_bin_impl((const double*)xy, nullptr, B, log2N, tile, frozen_mask, frozen_val, K, info_words,
                           xhat_words, u_words, workspace, w, stream);
}

}  // namespace

extern "C" int pcub_sc_decode_bin_compact(const double* xc, int64_t B, int32_t log2N, const uint32_t* frozen_mask,
                                          const uint32_t* frozen_val, int32_t K, uint32_t* info_words,
                                          uint32_t* xhat_words, uint32_t* u_words, void* workspace,
                                          size_t workspace_bytes, void* stream) {
    return decode_compact(xc, B, log2N, 0, frozen_mask, frozen_val, K, info_words, xhat_words, u_words, workspace,
                          workspace_bytes, stream);
}

extern "C" int pcub_sc_decode_bin_compact_tiled(const double* xc, int64_t B, int32_t log2N, int32_t tile,
                                                const uint32_t* frozen_mask, const uint32_t* frozen_val, int32_t K,
                                                uint32_t* info_words, uint32_t* xhat_words, uint32_t* u_words,
                                                void* workspace, size_t workspace_bytes, void* stream) {
    if (tile < 0 || tile > 4096) return PCUB_EINVAL;
    return decode_compact(xc, B, log2N, tile, frozen_mask, frozen_val, K, info_words, xhat_words, u_words, workspace,
                          workspace_bytes, stream);
}
