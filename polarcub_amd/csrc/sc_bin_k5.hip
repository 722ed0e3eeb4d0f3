// sc_bin_k5.hip -- instantiations of the binary SC decode kernel (part 5: split-level variants at
// G = 8, and with the re-encoded bits in the slot scratch for N = 4096).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part5(int v) {
    switch (v) {
        case 30: return k_sc_bin<32, 8, 2, false, 1, true, true, 2>;
        case 31: return k_sc_bin<32, 4, 2, false, 1, false, true, 2>;
        case 32: return k_sc_bin<16, 8, 3, false, 1, true, true, 2>;
        default: return nullptr;
    }
}

}  // namespace pcub
