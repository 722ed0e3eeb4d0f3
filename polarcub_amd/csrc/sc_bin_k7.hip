// sc_bin_k7.hip -- instantiations of the binary SC decode kernel (part 7: the split-level variant
// 26 with speculative plus transforms, op_g2, from the cross-lane leaves up to the split level).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part6(int v) {
    switch (v) {
        case 33: return k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, 1, false>;
        case 34: return k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, 4, false>;
        case 35: return k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, 16, false>;
        case 36: return k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, 32, false>;
        case 37: return k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, 32, true>;
        default: return nullptr;
    }
}

}  // namespace pcub
