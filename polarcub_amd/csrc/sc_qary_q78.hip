// sc_qary_q78.hip -- q-ary SC decode kernels for q = 7, 8 (see sc_qary_kern.h).
#include "sc_qary_kern.h"

namespace pcub {

QKern qary_kernel_q78(int q, int S, int G) {
    switch (q) {
        case 7: return qary_kernel_geom<7, 4>(S, G);
        case 8: return qary_kernel_geom<8, 4>(S, G);
        default: return nullptr;
    }
}

}  // namespace pcub
