// sc_bin_k6.hip -- compact-root twins of the default binary decode variants (the end-to-end
// Monte-Carlo pipeline's normalised channel rows, 8 bytes a position instead of a 16-byte pair).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_compact(int v) {
    switch (v) {
        case 24: return k_sc_bin<32, 4, 3, false, 1, true, false, 0, true>;
        case 26: return k_sc_bin<32, 4, 2, false, 1, true, true, 2, true>;
        case 31: return k_sc_bin<32, 4, 2, false, 1, false, true, 2, true>;
        case 30: return k_sc_bin<32, 8, 2, false, 1, true, true, 2, true>;
        case 33: return k_sc_bin<32, 8, 2, false, 1, false, true, 2, true>;
        default: return nullptr;
    }
}

}  // namespace pcub
