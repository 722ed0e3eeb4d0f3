// valu_peak.hip -- measured fp64 VALU ceilings of the MI355X (the guides quote no fp64 figure).
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/valu_peak scripts/valu_peak.hip
//   ./build/valu_peak            -> one JSON line
//
// Three kernels, each a long loop of independent chains per lane (8 in flight, no memory in
// the loop; one store at the end keeps the work live):
//   fma   v_fma_f64 (2 flop)            -> fp64 vector FLOP/s and wave-instructions/s
//   add   v_add_f64                     -> issue rate of a plain fp64 VALU op
//   div   a / b, correctly rounded      -> IEEE divisions/s (v_div_scale, v_rcp_f64, 5 fma,
//                                          v_div_fmas, v_div_fixup: the sequence the decoders use)
// Grid: 256 CUs x 8 waves x 64 lanes x 16 blocks.  Clock: the kernel's s_memrealtime is not the
// shader clock, so rates are per second (HIP events), and instructions/cycle follow from the
// nominal 2.4 GHz.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr int CH = 8;

__global__ __launch_bounds__(256) void k_fma(double* out, int iters, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int c = 0; c < CH; ++c) x[c] = __builtin_fma(x[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(double* out, int iters, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int c = 0; c < CH; ++c) x[c] = x[c] + a;
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + b;
}

__global__ __launch_bounds__(256) void k_div(double* out, int iters, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = 1.0 + threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < CH; ++c) x[c] = a / x[c] + b;  // one division + one add per step
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
static double time_ms(K kern, double* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);  // warm
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 5.0;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 8 * 4;  // 8 waves/CU resident x 4 rounds
    double* out;
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(double)));
    const double lanes = (double)blocks * 256;
    const int it_f = 4096, it_d = 2048;
    const double t_fma = time_ms(k_fma, out, blocks, it_f);
    const double t_add = time_ms(k_add, out, blocks, it_f);
    const double t_div = time_ms(k_div, out, blocks, it_d);
    const double fma_ops = lanes * it_f * 16 * CH;  // lane-FMAs
    const double div_ops = lanes * it_d * 2 * CH;   // lane-divisions
    const double ghz = 2.4, simds = 4.0 * cus;
    printf("{\"cus\": %d, \"fp64_fma_tflops\": %.2f, \"fp64_fma_lane_ops_per_clk_per_simd\": %.2f, "
           "\"fp64_add_lane_ops_per_clk_per_simd\": %.2f, \"fp64_div_per_s\": %.4g, "
           "\"fp64_div_lane_per_clk_per_simd\": %.3f, \"ms\": [%.3f, %.3f, %.3f], \"nominal_ghz\": %.1f}\n",
           cus, 2.0 * fma_ops / (t_fma * 1e-3) / 1e12, fma_ops / (t_fma * 1e-3) / (ghz * 1e9) / simds,
           fma_ops / (t_add * 1e-3) / (ghz * 1e9) / simds, div_ops / (t_div * 1e-3),
           div_ops / (t_div * 1e-3) / (ghz * 1e9) / simds, t_fma, t_add, t_div, ghz);
    CHECK(hipFree(out));
    return 0;
}
