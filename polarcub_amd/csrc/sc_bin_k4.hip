// sc_bin_k4.hip -- instantiations of the binary SC decode kernel (part 4: split-level variants).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part4(int v) {
    switch (v) {
        case 26: return k_sc_bin<32, 4, 2, false, 1, true, true, 2>;
        case 27: return k_sc_bin<32, 4, 2, false, 1, true, true, 1>;
        case 28: return k_sc_bin<32, 4, 2, false, 1, true, true, 3>;
        case 29: return k_sc_bin<32, 4, 3, false, 1, true, false, 2>;
        default: return nullptr;
    }
}

}  // namespace pcub
