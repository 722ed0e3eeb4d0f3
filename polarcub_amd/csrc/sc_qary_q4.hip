// sc_qary_q4.hip -- q-ary SC decode kernels for q = 4 (see sc_qary_kern.h).
#include "sc_qary_kern.h"

namespace pcub {

QKern qary_kernel_q4(int S, int G) { return qary_kernel_geom<4, 8>(S, G); }

}  // namespace pcub
