// sc_bin_kern.h -- the binary SC decode kernel template and its variant table.
//
// The variants are instantiated in several translation units (sc_bin_k*.hip) so
// the library builds in parallel; sc_bin.hip owns the launch code.
#pragma once
#include <hip/hip_runtime.h>

#include "sc_bin_sched.h"

namespace pcub {

constexpr int kBinBlock = 256;

// Decode kernel variants: virtual register subtree S (values per lane), lanes
// per codeword G, and the minimum waves/SIMD the register allocation must allow.
// Variant fields: S = register subtree values per lane, G = lanes per codeword,
// W = minimum waves/SIMD for register allocation, L = deepest stage level in
// LDS, T = non-temporal loads for the (once-streamed) input rows, Y = the re-encoded bits
// in LDS (Nv/32 words per thread; only where W workgroups still fit a CU's LDS).
// H = the chain's last level has 2S values per lane, the first S in LDS (HL; hl_run).
// P = prefetch distance of the final passes, in column pairs (chain_final).
struct Variant {
    int S, G, W, L, T, Y, H, P;
};
constexpr int kNumVariants = 34;
constexpr Variant kVar[kNumVariants] = {
    {16, 1, 2, 0, 0}, {8, 1, 4, 0, 0}, {32, 1, 1, 0, 0}, {16, 4, 2, 0, 0}, {8, 4, 4, 0, 0}, {16, 2, 2, 0, 0},
    {32, 2, 1, 0, 0}, {8, 8, 4, 0, 0}, {16, 2, 2, 0, 1}, {8, 8, 4, 0, 1}, {16, 4, 2, 0, 1}, {8, 4, 4, 1, 0},
    {16, 2, 4, 0, 1}, {16, 4, 4, 0, 1}, {8, 4, 4, 0, 1}, {32, 4, 2, 0, 1}, {32, 2, 2, 0, 1},
    {32, 4, 3, 0, 1}, {32, 2, 3, 0, 1}, {32, 8, 2, 0, 1}, {32, 8, 3, 0, 1},
    {32, 16, 2, 0, 1}, {32, 16, 3, 0, 1}, {16, 16, 3, 0, 1},
    {32, 4, 3, 0, 1, 1}, {32, 8, 3, 0, 1, 1},
    {32, 4, 2, 0, 1, 1, 1, 2}, {32, 4, 2, 0, 1, 1, 1, 1}, {32, 4, 2, 0, 1, 1, 1, 3}, {32, 4, 3, 0, 1, 1, 0, 2},
    {32, 8, 2, 0, 1, 1, 1, 2}, {32, 4, 2, 0, 1, 0, 1, 2}, {16, 8, 3, 0, 1, 1, 1, 2},
    {32, 8, 2, 0, 1, 0, 1, 2},
};

// LDS bytes of the stage level (L: S pairs per thread) or of the split level's LDS half (H: S doubles)
inline size_t bin_lds_bytes(int v) {
    if (kVar[v].H) return (size_t)kVar[v].S * kBinBlock * sizeof(double);
    return kVar[v].L ? (size_t)kVar[v].S * kBinBlock * sizeof(double2) : 0;
}

// values per lane at the end of a chain (the register level; 2S for the split-level variants)
inline int bin_sr(int v) { return kVar[v].S << kVar[v].H; }

// LDS bytes of the re-encoded bits of variant v at code length 2^n (0 unless Y)
inline size_t bin_ylds_bytes(int v, int n) {
    return kVar[v].Y ? (size_t)kBinBlock * (((size_t)1 << n) / kVar[v].G / 32) * sizeof(uint32_t) : 0;
}

template <int S, int G, int W, bool LDS, int NT, bool YL = false, bool HL = false, int PF = 0, bool CR = false,
          bool TR = false>
__global__ __launch_bounds__(kBinBlock, W) void k_sc_bin(BinArgs A) {
    // [S pairs][kBinBlock] when LDS (HL: [S doubles][kBinBlock]), then [Nv/32 words][kBinBlock]
    // when YL (plus occupancy padding)
    extern __shared__ double2 lds_last[];
    constexpr int LDS2 = LDS ? S * kBinBlock : HL ? S / 2 * kBinBlock : 0;  // double2 units before Y
    constexpr int CWB = kBinBlock / G;  // codewords per workgroup tile
    const long long slot = (long long)blockIdx.x * kBinBlock + threadIdx.x;
    const int j = threadIdx.x & (G - 1);
    const int lane = threadIdx.x & 63;
    const Lvl last = LDS ? Lvl{lds_last + threadIdx.x, kBinBlock} : Lvl{nullptr, 0};
    // wave tiles: a wave decodes 64 / G codewords at a time (its lanes' codewords are independent of the
    // other waves', whose LDS columns are their own), either the static stride of the workgroup tiles
    // (wave wv of workgroup b takes wave tiles (b + i * grid) * WPB + wv) or the next tile of a counter
    constexpr int WPB = kBinBlock / 64, CWW = 64 / G;
    static_assert(CWB == WPB * CWW, "workgroup tile = its waves' tiles");
    const long long nwt = (A.B + CWW - 1) / CWW;
    const int wv = threadIdx.x >> 6;
    long long wt = A.wtiles ? next_wave_tile(A.wtiles, lane) : (long long)blockIdx.x * WPB + wv;
    while (wt < nwt) {
        const long long cw = wt * CWW + lane / G;
        const bool valid = cw < A.B;
        decode_codeword<S, G, LDS, NT, YL, HL, PF, CR, -1, TR>(A, valid ? cw : A.B - 1, j, lane, slot, valid, last,
                                               YL ? (uint32_t*)(lds_last + LDS2) + threadIdx.x : nullptr, kBinBlock,
                                               HL ? (double*)lds_last + threadIdx.x : nullptr);
        wt = A.wtiles ? next_wave_tile(A.wtiles, lane) : wt + (long long)gridDim.x * WPB;
    }
}

typedef void (*BinKernFn)(BinArgs);

// The kernel of variant v if this translation unit instantiates it, else nullptr.  The shipped library
// builds the variants pick_variant can launch (0, 1, 10, 13, 14, 17, 24, 26, 31); the rest of kVar
// are the round 1-3 sweep's geometries, measured slower, kept as table rows so the
// variant numbers in profiles/ stay meaningful; pcub_sc_set_variant rejects them.
BinKernFn bin_kernel_part0(int v);
BinKernFn bin_kernel_part1(int v);
BinKernFn bin_kernel_part2(int v);
BinKernFn bin_kernel_part4(int v);
BinKernFn bin_kernel_part5(int v);
BinKernFn bin_kernel_part8(int v);
// the compact-root twin of variant v (CR: root rows as compact normalised doubles), or nullptr
BinKernFn bin_kernel_compact(int v);
// variant v reading its root in the wave's own tiles (TR: tile = 64 / G, a wave-uniform base and
// 32-bit lane offsets), pairs or compact rows; nullptr where not instantiated (sc_bin_k7.hip)
BinKernFn bin_kernel_tiled_root(int v, bool compact);
BinKernFn bin_kernel_tiled_root2(int v, bool compact);  // sc_bin_k9.hip: the N >= 4096 variants' twins

}  // namespace pcub
