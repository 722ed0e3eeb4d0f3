// sc_bin_k9.hip -- tiled-root twins (TR: the wave's tile base in SGPRs, 32-bit lane offsets; see
// sc_bin_k7.hip) of the N >= 4096 variants 31 (G = 4) and 30, 33 (G = 8), pairs and compact rows.
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_tiled_root2(int v, bool compact) {
    switch (v) {
        case 31: return compact ? k_sc_bin<32, 4, 2, false, 1, false, true, 2, true, true>
                                : k_sc_bin<32, 4, 2, false, 1, false, true, 2, false, true>;
        case 30: return compact ? k_sc_bin<32, 8, 2, false, 1, true, true, 2, true, true>
                                : k_sc_bin<32, 8, 2, false, 1, true, true, 2, false, true>;
        case 33: return compact ? k_sc_bin<32, 8, 2, false, 1, false, true, 2, true, true>
                                : k_sc_bin<32, 8, 2, false, 1, false, true, 2, false, true>;
        default: return nullptr;
    }
}

}  // namespace pcub
