// sc_bin_k0.hip -- instantiations of the binary SC decode kernel (part 0).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part0(int v) {
    switch (v) {
        case 0: return k_sc_bin<16, 1, 2, false, 0>;
        case 24: return k_sc_bin<32, 4, 3, false, 1, true>;
        default: return nullptr;
    }
}

}  // namespace pcub
