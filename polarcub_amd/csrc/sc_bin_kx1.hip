// sc_bin_kx1.hip -- EXPERIMENT (A/B only): the shipped tiled-root variant 26 with the minus
// transform's division as div_den12 (no v_div_scale / v_div_fixup).  Its own namespace so the
// kernel symbols differ from the shipped ones.
#define PCUB_FAST_F 1
#define pcub pcubx1
#include "sc_bin_kern.h"

namespace pcubx1 {
BinKernFn bin_kernel_x(int v, bool compact) {
    if (v != 26) return nullptr;
    return compact ? k_sc_bin<32, 4, 2, false, 1, true, true, 2, true, true>
                   : k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, true>;
}
}  // namespace pcubx1
#undef pcub
