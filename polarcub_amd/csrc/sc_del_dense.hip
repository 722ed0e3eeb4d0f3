// sc_del_dense.hip -- instantiations of the table-driven deletion decoder (sc_del_dense.h).
#include "sc_del_dense.h"

namespace pcub {

DelKern del_kernel_dense(int n0, int tb) {
#define PCUB_DENSE(N0)                                 \
    switch (tb) {                                      \
        case 4: return k_sc_del_dense<N0, 4>;          \
        case 5: return k_sc_del_dense<N0, 5>;          \
        case 6: return k_sc_del_dense<N0, 6>;          \
        case 7: return k_sc_del_dense<N0, 7>;          \
        case 8: return k_sc_del_dense<N0, 8>;          \
        default: return nullptr;                       \
    }
    if (n0 == 2) PCUB_DENSE(2)
    if (n0 == 3) PCUB_DENSE(3)
#undef PCUB_DENSE
    return nullptr;
}

}  // namespace pcub
