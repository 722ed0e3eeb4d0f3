// dpp_check.hip -- GPU check of the DPP lane exchanges of sc_bin_body.h (xor_shfl_c<1,2,4,8>).
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Iinclude -Ipolarcub_amd/csrc -o build/dpptest tests/emu/dpp_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "sc_bin_body.h"
using namespace pcub;
template <int M> __global__ void k(double* o) {
    const int l = threadIdx.x;
    o[blockIdx.x * 64 + l] = xor_shfl_c<M>((double)(l + 1000 * blockIdx.x));
}
int main() {
    double* d; hipMalloc(&d, 4 * 64 * sizeof(double));
    hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, d);
    hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, d + 64);
    hipLaunchKernelGGL(k<4>, 1, 64, 0, 0, d + 128);
    hipLaunchKernelGGL(k<8>, 1, 64, 0, 0, d + 192);
    double h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0; const int m[4] = {1, 2, 4, 8};
    for (int t = 0; t < 4; ++t) for (int l = 0; l < 64; ++l) if (h[t * 64 + l] != (double)(l ^ m[t])) { ++bad; if (bad < 10) printf("mask %d lane %d got %g\n", m[t], l, h[t*64+l]); }
    printf("dpp xor check: %d bad\n", bad);
    return bad != 0;
}
