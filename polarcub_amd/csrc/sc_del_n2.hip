// sc_del_n2.hip -- deletion-channel SC decode kernels for 2^2-input trellises (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n2(int tb, bool exp, int oc) { return del_kernel_tb<2>(tb, exp, oc); }

}  // namespace pcub
