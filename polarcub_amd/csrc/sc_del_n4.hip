// sc_del_n4.hip -- deletion-channel SC decode kernels for 2^4-input trellises, no guard-band
// ones (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n4_d0(int tb) { return del_kernel_t<4, false, 0>(tb); }

}  // namespace pcub
