// sc_bin_k1.hip -- instantiations of the binary SC decode kernel (part 1).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part1(int v) {
    switch (v) {
        case 1: return k_sc_bin<8, 1, 4, false, 0>;
        case 13: return k_sc_bin<16, 4, 4, false, 1>;
        case 17: return k_sc_bin<32, 4, 3, false, 1>;
        default: return nullptr;
    }
}

}  // namespace pcub
