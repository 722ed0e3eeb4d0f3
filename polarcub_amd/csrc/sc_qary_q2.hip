// sc_qary_q2.hip -- q-ary SC decode kernels for q = 2 (see sc_qary_kern.h).
#include "sc_qary_kern.h"

namespace pcub {

QKern qary_kernel_q2(int S, int G) { return qary_kernel_geom<2, 8>(S, G); }

}  // namespace pcub
