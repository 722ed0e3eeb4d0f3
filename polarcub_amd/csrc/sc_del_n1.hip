// sc_del_n1.hip -- deletion-channel SC decode kernels for 2^1-input trellises, no guard-band
// ones (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n1_d0(int tb) { return del_kernel_t<1, false, 0>(tb); }

}  // namespace pcub
