// sc_qary_kern.h -- the q-ary SC decode kernel template and its instantiation table.
//
// Instantiated per alphabet size in sc_qary_q*.hip (the q-ary schedules are large
// templates: one translation unit per q keeps the parallel build short); sc_qary.hip
// owns the launch code.  Geometries: S register positions per lane x G lanes per
// codeword, only those q_geom() can pick (S = 8 for q <= 4 else 4, G = 4, both
// reduced for short codes).
#pragma once
#include <hip/hip_runtime.h>

#include "sc_qary_body.h"

namespace pcub {

constexpr int kQaryBlock = 256;

// waves per SIMD the register allocation must allow: the S*q doubles of the register
// level (and q >= 6 vectors in the transforms) need two waves' worth of registers at
// 32; up to 16 the kernel runs at four (the fastest q = 4 geometry, S = 4, G = 4:
// 73.4M cw/s at 4 waves vs 71.0M at 3, profiles/r2/qary_*)
// (G >= 8 with q * S = 32: three, the cross-lane leaves keep fewer vectors live)
constexpr int qary_waves(int q, int S, int G = 4) {
    return (G >= 8 && q * S == 32 && q < 6) ? 3 : (q * S >= 32 || q >= 6) ? 2 : (q * S <= 16 ? 4 : 3);
}

// YL: the re-encoded symbols in dynamic LDS ([Nv/4 words][kQaryBlock]) instead of the slot
// HL: the split last level's LDS half after them ([S * Q doubles][kQaryBlock], decode_qary_cw)
template <int Q, int S, int G, int W = qary_waves(Q, S, G), int U = 1, bool YL = false, bool HL = false,
          bool TR = false, int NC = -1>
__global__ __launch_bounds__(kQaryBlock, W) void k_sc_qary(QArgs A) {
    static_assert(kQaryBlock == kQHlStride, "split-level LDS column stride");
    extern __shared__ uint32_t qsym_lds[];
    double* hl = HL ? (double*)(qsym_lds + A.ylds_words * kQaryBlock) + threadIdx.x : nullptr;
    const long long slot = (long long)blockIdx.x * kQaryBlock + threadIdx.x;
    const int j = threadIdx.x & (G - 1);
    const int lane = threadIdx.x & 63;
    // wave tiles of 64 / G codewords (k_sc_bin's): the static stride of the workgroup tiles, or the
    // next tile of the launch's counter so the waves finish together (round 6)
    constexpr int WPB = kQaryBlock / 64, CWW = 64 / G;
    const long long nwt = (A.B + CWW - 1) / CWW;
    long long wt = A.wtiles ? next_wave_tile(A.wtiles, lane) : (long long)blockIdx.x * WPB + (threadIdx.x >> 6);
    while (wt < nwt) {
        const long long cw = wt * CWW + lane / G;
        const bool valid = cw < A.B;
        decode_qary_cw<Q, S, G, U, YL, HL, TR, NC>(A, valid ? cw : A.B - 1, slot, valid, j, lane,
                                           YL ? qsym_lds + threadIdx.x : nullptr, kQaryBlock, hl);
        wt = A.wtiles ? next_wave_tile(A.wtiles, lane) : wt + (long long)gridDim.x * WPB;
    }
}

typedef void (*QKern)(QArgs);

// the kernel for (q, S, G), or nullptr
QKern qary_kernel_q2(int S, int G);
QKern qary_kernel_q3(int S, int G);
QKern qary_kernel_q4(int S, int G);
QKern qary_kernel_q56(int q, int S, int G);
QKern qary_kernel_q78(int q, int S, int G);

// the symbols-in-LDS twin of the kernel for (q, S, G), or nullptr (q = 4, S = 4, G = 4 only)
QKern qary_kernel_q4_y(int S, int G);
// its split-level twin (2S positions per lane at the chain's end, S of them in LDS; three waves)
QKern qary_kernel_q4_h(int S, int G);
inline QKern qary_kernel_h(int q, int S, int G) { return q == 4 ? qary_kernel_q4_h(S, G) : nullptr; }
// the split-level kernel reading its root in the wave's own tiles (decode_qary_cw's TR), or nullptr
QKern qary_kernel_q4_h_tr(int S, int G);
// ... compiled for code length 2^n alone (NC = n; the C4 shape, n = 8), or nullptr
QKern qary_kernel_q4_h_tr_n(int S, int G, int n);
inline QKern qary_kernel_h_tr(int q, int S, int G) { return q == 4 ? qary_kernel_q4_h_tr(S, G) : nullptr; }
inline QKern qary_kernel_y(int q, int S, int G) { return q == 4 ? qary_kernel_q4_y(S, G) : nullptr; }

inline QKern qary_kernel(int q, int S, int G) {
    switch (q) {
        case 2: return qary_kernel_q2(S, G);
        case 3: return qary_kernel_q3(S, G);
        case 4: return qary_kernel_q4(S, G);
        case 5:
        case 6: return qary_kernel_q56(q, S, G);
        case 7:
        case 8: return qary_kernel_q78(q, S, G);
        default: return nullptr;
    }
}

// geometries q_geom() can produce for a large S0 (8 or 4): S in {S0, S0/2} with
// G = 4, 2, 1, and smaller S with G = 1 (short codes)
template <int Q, int S0>
QKern qary_kernel_geom(int S, int G) {
    constexpr int S1 = S0 / 2;
    if (S == S0 || S == S1) {
        if (S == S0) {
            if (G == 4) return k_sc_qary<Q, S0, 4>;
            if (G == 2) return k_sc_qary<Q, S0, 2>;
            if (G == 1) return k_sc_qary<Q, S0, 1>;
        } else {
            if (G == 4) return k_sc_qary<Q, S1, 4>;
            if (G == 2) return k_sc_qary<Q, S1, 2>;
            if (G == 1) return k_sc_qary<Q, S1, 1>;
        }
        return nullptr;
    }
    if (G != 1) return nullptr;
    if constexpr (S1 > 2) {
        if (S == S1 / 2) return k_sc_qary<Q, S1 / 2, 1>;
    }
    if constexpr (S1 > 1) {
        if (S == 1) return k_sc_qary<Q, 1, 1>;
    }
    return nullptr;
}

}  // namespace pcub
