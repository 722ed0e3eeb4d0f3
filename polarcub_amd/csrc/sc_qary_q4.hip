// sc_qary_q4.hip -- q-ary SC decode kernels for q = 4 (see sc_qary_kern.h).
#include "sc_qary_kern.h"

namespace pcub {

// G = 8, 16 (one or two stored stage levels fewer, q-ary DESIGN 3.4) for the C4 alphabet
QKern qary_kernel_q4(int S, int G) {
    if (G == 8) {
        if (S == 8) return k_sc_qary<4, 8, 8>;
        if (S == 4) return k_sc_qary<4, 4, 8>;
        if (S == 2) return k_sc_qary<4, 2, 8>;
        return nullptr;
    }
    if (G == 16) {
        if (S == 4) return k_sc_qary<4, 4, 16>;
        if (S == 2) return k_sc_qary<4, 2, 16>;
        return nullptr;
    }
    return qary_kernel_geom<4, 8>(S, G);
}

// the C4 geometry with its symbols in LDS (4 words of 2-bit symbols a thread at N = 256)
QKern qary_kernel_q4_y(int S, int G) {
    if (S == 4 && G == 4) return k_sc_qary<4, 4, 4, qary_waves(4, 4, 4), 1, true>;
    return nullptr;
}

// the split-level twin: 2S = 8 positions per lane at a chain's end, 4 of them in LDS (36 KB a
// workgroup with the 2-bit symbols; three workgroups a CU: the kernel needs ~168 VGPRs, and at the
// 128 of four workgroups it spilled 119 VGPRs and ran 2 % slower, 88.3 vs 90.0 M cw/s)
QKern qary_kernel_q4_h(int S, int G) {
    if (S == 4 && G == 4) return k_sc_qary<4, 4, 4, 3, 1, true, true>;
    return nullptr;
}

// ... reading its root rows in the wave's own tiles (TR: tile = 16, a wave-uniform base)
QKern qary_kernel_q4_h_tr(int S, int G) {
    if (S == 4 && G == 4) return k_sc_qary<4, 4, 4, 3, 1, true, true, true>;
    return nullptr;
}

// ... specialised on the C4 code length (N = 256): the per-position offsets fold (round 6)
QKern qary_kernel_q4_h_tr_n(int S, int G, int n) {
    if (S == 4 && G == 4 && n == 8) return k_sc_qary<4, 4, 4, 3, 1, true, true, true, 8>;
    return nullptr;
}

}  // namespace pcub
