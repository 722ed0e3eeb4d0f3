// sc_qary_q3.hip -- q-ary SC decode kernels for q = 3 (see sc_qary_kern.h).
#include "sc_qary_kern.h"

namespace pcub {

QKern qary_kernel_q3(int S, int G) { return qary_kernel_geom<3, 8>(S, G); }

}  // namespace pcub
