// sc_del_dense.hip -- instantiations of the table-driven deletion decoder (sc_del_dense.h).
#include "sc_del_dense.h"

namespace pcub {

DelKern del_kernel_dense(int n0, int tb, bool gt) {
#define PCUB_DENSE(N0, GT)                             \
    switch (tb) {                                      \
        case 4: return k_sc_del_dense<N0, 4, GT>;      \
        case 5: return k_sc_del_dense<N0, 5, GT>;      \
        case 6: return k_sc_del_dense<N0, 6, GT>;      \
        case 7: return k_sc_del_dense<N0, 7, GT>;      \
        case 8: return k_sc_del_dense<N0, 8, GT>;      \
        default: return nullptr;                       \
    }
    if (n0 == 2 && gt) PCUB_DENSE(2, true)
    if (n0 == 2) PCUB_DENSE(2, false)
    if (n0 == 3) PCUB_DENSE(3, false)
#undef PCUB_DENSE
    return nullptr;
}

}  // namespace pcub
