// sc_del_n1o.hip -- deletion-channel SC decode kernels for 2^1-input trellises with up to
// 3 guard-band ones (see sc_del_kern.h).
#include "sc_del_kern.h"

namespace pcub {

DelKern del_kernel_n1_d3(int tb) { return del_kernel_t<1, false, 3>(tb); }

}  // namespace pcub
