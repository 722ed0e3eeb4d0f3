// sc_bin_kern.h -- the binary SC decode kernel template and its variant table.
//
// The variants are instantiated in several translation units (sc_bin_k*.hip) so
// the library builds in parallel; sc_bin.hip owns the launch code.
#pragma once
#include <hip/hip_runtime.h>

#include "sc_bin_body.h"

namespace pcub {

constexpr int kBinBlock = 256;

// Decode kernel variants: virtual register subtree S (values per lane), lanes
// per codeword G, and the minimum waves/SIMD the register allocation must allow.
// Variant fields: S = register subtree values per lane, G = lanes per codeword,
// W = minimum waves/SIMD for register allocation, L = deepest stage level in
// LDS, T = non-temporal loads for the (once-streamed) input rows, Y = the re-encoded bits
// in LDS (Nv/32 words per thread; only where W workgroups still fit a CU's LDS).
struct Variant {
    int S, G, W, L, T, Y;
};
constexpr int kNumVariants = 26;
constexpr Variant kVar[kNumVariants] = {
    {16, 1, 2, 0, 0}, {8, 1, 4, 0, 0}, {32, 1, 1, 0, 0}, {16, 4, 2, 0, 0}, {8, 4, 4, 0, 0}, {16, 2, 2, 0, 0},
    {32, 2, 1, 0, 0}, {8, 8, 4, 0, 0}, {16, 2, 2, 0, 1}, {8, 8, 4, 0, 1}, {16, 4, 2, 0, 1}, {8, 4, 4, 1, 0},
    {16, 2, 4, 0, 1}, {16, 4, 4, 0, 1}, {8, 4, 4, 0, 1}, {32, 4, 2, 0, 1}, {32, 2, 2, 0, 1},
    {32, 4, 3, 0, 1}, {32, 2, 3, 0, 1}, {32, 8, 2, 0, 1}, {32, 8, 3, 0, 1},
    {32, 16, 2, 0, 1}, {32, 16, 3, 0, 1}, {16, 16, 3, 0, 1},
    {32, 4, 3, 0, 1, 1}, {32, 8, 3, 0, 1, 1},
};

inline size_t bin_lds_bytes(int v) { return kVar[v].L ? (size_t)kVar[v].S * kBinBlock * sizeof(double2) : 0; }

// LDS bytes of the re-encoded bits of variant v at code length 2^n (0 unless Y)
inline size_t bin_ylds_bytes(int v, int n) {
    return kVar[v].Y ? (size_t)kBinBlock * (((size_t)1 << n) / kVar[v].G / 32) * sizeof(uint32_t) : 0;
}

template <int S, int G, int W, bool LDS, int NT, bool YL = false>
__global__ __launch_bounds__(kBinBlock, W) void k_sc_bin(BinArgs A) {
    // [S pairs][kBinBlock] when LDS, then [Nv/32 words][kBinBlock] when YL (plus occupancy padding)
    extern __shared__ double2 lds_last[];
    constexpr int CWB = kBinBlock / G;  // codewords per workgroup tile
    const long long slot = (long long)blockIdx.x * kBinBlock + threadIdx.x;
    const int j = threadIdx.x & (G - 1);
    const int lane = threadIdx.x & 63;
    const Lvl last = LDS ? Lvl{lds_last + threadIdx.x, kBinBlock} : Lvl{nullptr, 0};
    const long long ntiles = (A.B + CWB - 1) / CWB;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long cw = t * CWB + threadIdx.x / G;
        const bool valid = cw < A.B;
        decode_codeword<S, G, LDS, NT, YL>(A, valid ? cw : A.B - 1, j, lane, slot, valid, last,
                                           YL ? (uint32_t*)(lds_last + (LDS ? S * kBinBlock : 0)) + threadIdx.x : nullptr,
                                           kBinBlock);
    }
}

typedef void (*BinKernFn)(BinArgs);

// The kernel of variant v if this translation unit instantiates it, else nullptr.
BinKernFn bin_kernel_part0(int v);
BinKernFn bin_kernel_part1(int v);
BinKernFn bin_kernel_part2(int v);
BinKernFn bin_kernel_part3(int v);

}  // namespace pcub
