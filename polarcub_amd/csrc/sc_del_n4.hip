// sc_del_n4.hip -- deletion-channel SC decode kernels for 2^4-input trellises (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n4(int tb, bool exp, int oc) { return del_kernel_tb<4>(tb, exp, oc); }

}  // namespace pcub
