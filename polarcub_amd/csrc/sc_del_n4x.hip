// sc_del_n4x.hip -- leaf-export (genie) deletion kernels for 2^4-input trellises, with and
// without guard-band ones (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n4_x(int tb, int oc) {
    return oc == 0 ? del_kernel_t<4, true, 0>(tb) : oc == 3 ? del_kernel_t<4, true, 3>(tb) : nullptr;
}

}  // namespace pcub
