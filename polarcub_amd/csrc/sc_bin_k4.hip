// sc_bin_k4.hip -- instantiations of the binary SC decode kernel (part 4: the split-level default).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part4(int v) {
    switch (v) {
        case 26: return k_sc_bin<32, 4, 2, false, 1, true, true, 2>;
        default: return nullptr;
    }
}

}  // namespace pcub
