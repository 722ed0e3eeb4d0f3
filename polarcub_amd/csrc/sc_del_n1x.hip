// sc_del_n1x.hip -- leaf-export (genie) deletion kernels for 2^1-input trellises, with and
// without guard-band ones (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n1_x(int tb, int oc) {
    return oc == 0 ? del_kernel_t<1, true, 0>(tb) : oc == 3 ? del_kernel_t<1, true, 3>(tb) : nullptr;
}

}  // namespace pcub
