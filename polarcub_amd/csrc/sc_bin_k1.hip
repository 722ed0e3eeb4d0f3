// sc_bin_k1.hip -- instantiations of the binary SC decode kernel (part 1 of 4).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part1(int v) {
    switch (v) {
        case 1: return k_sc_bin<8, 1, 4, false, 0>;
        case 5: return k_sc_bin<16, 2, 2, false, 0>;
        case 9: return k_sc_bin<8, 8, 4, false, 1>;
        case 13: return k_sc_bin<16, 4, 4, false, 1>;
        case 17: return k_sc_bin<32, 4, 3, false, 1>;
        case 21: return k_sc_bin<32, 16, 2, false, 1>;
        case 25: return k_sc_bin<32, 8, 3, false, 1, true>;
        default: return nullptr;
    }
}

}  // namespace pcub
