// sc_del_n1.hip -- deletion-channel SC decode kernels for 2^1-input trellises (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n1(int tb, bool exp, int oc) { return del_kernel_tb<1>(tb, exp, oc); }

}  // namespace pcub
