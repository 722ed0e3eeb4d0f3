// sc_bin_k2.hip -- instantiations of the binary SC decode kernel (part 2 of 4).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part2(int v) {
    switch (v) {
        case 2: return k_sc_bin<32, 1, 1, false, 0>;
        case 6: return k_sc_bin<32, 2, 1, false, 0>;
        case 10: return k_sc_bin<16, 4, 2, false, 1>;
        case 14: return k_sc_bin<8, 4, 4, false, 1>;
        case 18: return k_sc_bin<32, 2, 3, false, 1>;
        case 22: return k_sc_bin<32, 16, 3, false, 1>;
        default: return nullptr;
    }
}

}  // namespace pcub
