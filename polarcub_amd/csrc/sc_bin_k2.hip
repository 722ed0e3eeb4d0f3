// sc_bin_k2.hip -- instantiations of the binary SC decode kernel (part 2).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part2(int v) {
    switch (v) {
        case 10: return k_sc_bin<16, 4, 2, false, 1>;
        case 14: return k_sc_bin<8, 4, 4, false, 1>;
        default: return nullptr;
    }
}

}  // namespace pcub
