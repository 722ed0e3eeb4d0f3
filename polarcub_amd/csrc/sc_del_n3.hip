// sc_del_n3.hip -- deletion-channel SC decode kernels for 2^3-input trellises, no guard-band
// ones (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n3_d0(int tb) { return del_kernel_t<3, false, 0>(tb); }

}  // namespace pcub
