// sc_del_n4w.hip -- deletion-channel SC decode kernels for 512 and 1024 trellises of 2^4 inputs
// (n = 13, 14 at main_deletion's n0 = n // 3), no guard-band ones: one codeword per workgroup of
// T threads (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n4_wide(int tb) {
    if (tb == 9) return k_sc_del<4, 9, false, 0>;
    if (tb == 10) return k_sc_del<4, 10, false, 0>;
    return nullptr;
}

}  // namespace pcub
