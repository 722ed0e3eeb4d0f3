// sc_bin_k3.hip -- instantiations of the binary SC decode kernel (part 3 of 4).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part3(int v) {
    switch (v) {
        case 3: return k_sc_bin<16, 4, 2, false, 0>;
        case 7: return k_sc_bin<8, 8, 4, false, 0>;
        case 11: return k_sc_bin<8, 4, 4, true, 0>;
        case 15: return k_sc_bin<32, 4, 2, false, 1>;
        case 19: return k_sc_bin<32, 8, 2, false, 1>;
        case 23: return k_sc_bin<16, 16, 3, false, 1>;
        default: return nullptr;
    }
}

}  // namespace pcub
