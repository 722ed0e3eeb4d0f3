// sc_bin_k0.hip -- instantiations of the binary SC decode kernel (part 0 of 4).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part0(int v) {
    switch (v) {
        case 0: return k_sc_bin<16, 1, 2, false, 0>;
        case 4: return k_sc_bin<8, 4, 4, false, 0>;
        case 8: return k_sc_bin<16, 2, 2, false, 1>;
        case 12: return k_sc_bin<16, 2, 4, false, 1>;
        case 16: return k_sc_bin<32, 2, 2, false, 1>;
        case 20: return k_sc_bin<32, 8, 3, false, 1>;
        case 24: return k_sc_bin<32, 4, 3, false, 1, true>;
        default: return nullptr;
    }
}

}  // namespace pcub
