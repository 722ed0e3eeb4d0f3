// sc_del_n3.hip -- deletion-channel SC decode kernels for 2^3-input trellises (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n3(int tb, bool exp, int oc) { return del_kernel_tb<3>(tb, exp, oc); }

}  // namespace pcub
