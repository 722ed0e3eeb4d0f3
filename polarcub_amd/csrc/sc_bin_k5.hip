// sc_bin_k5.hip -- instantiations of the binary SC decode kernel (part 5: the split-level variant with
// the re-encoded bits in the slot scratch, N = 4096 and 8192).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part5(int v) {
    switch (v) {
        case 31: return k_sc_bin<32, 4, 2, false, 1, false, true, 2>;
        default: return nullptr;
    }
}

}  // namespace pcub
