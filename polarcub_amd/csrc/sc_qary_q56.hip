// sc_qary_q56.hip -- q-ary SC decode kernels for q = 5, 6 (see sc_qary_kern.h).
#include "sc_qary_kern.h"

namespace pcub {

QKern qary_kernel_q56(int q, int S, int G) {
    switch (q) {
        case 5: return qary_kernel_geom<5, 4>(S, G);
        case 6: return qary_kernel_geom<6, 4>(S, G);
        default: return nullptr;
    }
}

}  // namespace pcub
