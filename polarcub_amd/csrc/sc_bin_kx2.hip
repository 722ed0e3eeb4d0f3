// sc_bin_kx2.hip -- EXPERIMENT (A/B only): kx1 (div_den12 in the minus transform, one comparison in
// the plus transform's orientation) + the information bits packed by compress masks and x_hat by
// bit-matrix transposes (PCUB_R5).  Its own namespace so the kernel symbols differ from the shipped ones.
#define PCUB_FAST_F 1
#define PCUB_R5 1
#define pcub pcubx2
#include "sc_bin_kern.h"

namespace pcubx2 {
BinKernFn bin_kernel_x(int v, bool compact) {
    if (v != 26) return nullptr;
    return compact ? k_sc_bin<32, 4, 2, false, 1, true, true, 2, true, true>
                   : k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, true>;
}
}  // namespace pcubx2
#undef pcub
