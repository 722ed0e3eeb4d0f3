// sc_del_dense.hip -- instantiations of the table-driven deletion decoder (sc_del_dense.h).
#include "sc_del_dense.h"

namespace pcub {

DelKern del_kernel_dense(int n0, int tb, bool gt, int g, bool r1) {
#define PCUB_DENSE(N0, GT)                             \
    switch (tb) {                                      \
        case 4: return k_sc_del_dense<N0, 4, GT>;      \
        case 5: return k_sc_del_dense<N0, 5, GT>;      \
        case 6: return k_sc_del_dense<N0, 6, GT>;      \
        case 7: return k_sc_del_dense<N0, 7, GT>;      \
        case 8: return k_sc_del_dense<N0, 8, GT>;      \
        default: return nullptr;                       \
    }
#define PCUB_DENSE_G(N0, GT, G)                        \
    switch (tb) {                                      \
        case 4: return k_sc_del_dense<N0, 4, GT, G>;   \
        case 5: return k_sc_del_dense<N0, 5, GT, G>;   \
        case 6: return k_sc_del_dense<N0, 6, GT, G>;   \
        default: return nullptr;                       \
    }
#define PCUB_DENSE_8(N0, GT)                           \
    switch (tb) {                                      \
        case 4: return k_sc_del_dense<N0, 4, GT, 8>;   \
        case 5: return k_sc_del_dense<N0, 5, GT, 8>;   \
        case 6: return k_sc_del_dense<N0, 6, GT, 8>;   \
        case 7: return k_sc_del_dense<N0, 7, GT, 8>;   \
        case 8: return k_sc_del_dense<N0, 8, GT, 8>;   \
        default: return nullptr;                       \
    }
    if (g == 8 && !r1) {  // the rate-1 A/B (pcub_sc_set_deletion_rate1, a diagnostic)
        if (n0 == 2 && gt) {
            switch (tb) {
                case 6: return k_sc_del_dense<2, 6, true, 8, false>;
                case 8: return k_sc_del_dense<2, 8, true, 8, false>;
                default: return nullptr;
            }
        }
        return nullptr;
    }
    if (g == 8) {
        if (n0 == 2 && gt) PCUB_DENSE_8(2, true)
        if (n0 == 2) PCUB_DENSE_8(2, false)
        if (n0 == 3) PCUB_DENSE_8(3, false)
        return nullptr;
    }
    if (g == 4) {
        if (n0 == 2 && gt) PCUB_DENSE_G(2, true, 4)
        if (n0 == 2) PCUB_DENSE_G(2, false, 4)
        if (n0 == 3) PCUB_DENSE_G(3, false, 4)
        return nullptr;
    }
    if (g != 16) return nullptr;
    if (n0 == 2 && gt) PCUB_DENSE(2, true)
    if (n0 == 2) PCUB_DENSE(2, false)
    if (n0 == 3) PCUB_DENSE(3, false)
#undef PCUB_DENSE
#undef PCUB_DENSE_G
#undef PCUB_DENSE_8
    return nullptr;
}

}  // namespace pcub
