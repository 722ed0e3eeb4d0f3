// sc_del_n3o.hip -- deletion-channel SC decode kernels for 2^3-input trellises with up to
// 3 guard-band ones (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n3_d3(int tb) { return del_kernel_t<3, false, 3>(tb); }

}  // namespace pcub
