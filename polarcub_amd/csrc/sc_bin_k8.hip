// sc_bin_k8.hip -- binary decode variants 30 and 33: the split level at G = 8 lanes a codeword
// (S = 32: 64 values a lane, a node of 512 positions), the re-encoded bits in LDS (30) or in the
// slot scratch (33).  At N = 4096 the split level is depth 3, so only levels 1 and 2 are stored
// (variant 31, G = 4, stores three): the C3 shape's candidates.
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_part8(int v) {
    switch (v) {
        case 30: return k_sc_bin<32, 8, 2, false, 1, true, true, 2>;
        case 33: return k_sc_bin<32, 8, 2, false, 1, false, true, 2>;
        default: return nullptr;
    }
}

}  // namespace pcub
