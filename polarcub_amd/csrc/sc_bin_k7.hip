// sc_bin_k7.hip -- the default binary decode variants reading their root in the wave's own tiles
// (decode_codeword's TR: tile = 64 / G codewords, the rows addressed from a wave-uniform base).
#include "sc_bin_kern.h"

namespace pcub {

BinKernFn bin_kernel_tiled_root(int v, bool compact) {
    switch (v) {
        case 26: return compact ? k_sc_bin<32, 4, 2, false, 1, true, true, 2, true, true>
                                : k_sc_bin<32, 4, 2, false, 1, true, true, 2, false, true>;
        default: return nullptr;
    }
}

}  // namespace pcub
