// Diagnostic (round 3): does an out-of-line device function see its caller's private
// (scratch) array correctly through a generic pointer, at full occupancy with large frames?
// Each lane fills a 4 KiB private array with lane-unique values and hands it to a noinline
// callee that reads it at data-dependent indices and writes some entries back; the caller then
// re-reads it.  Any lane whose result differs from the host's recomputation is counted.
// Build: hipcc --offload-arch=gfx950 -O3 flat_private.hip -o flat_private
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kLen = 512;

__device__ __attribute__((noinline)) double touch(double* a, unsigned seed, int lane) {
    double s = 0.0;
    unsigned h = seed;
    for (int i = 0; i < 64; ++i) {
        h = h * 1664525u + 1013904223u;
        const int k = (int)(h >> 23) & (kLen - 1);
        s += a[k];
        a[(k * 7 + i) & (kLen - 1)] += 1.0;
    }
    // a lane exchange inside the callee, as the deletion subtree does
    s += __shfl_xor(s, 1) * 0.0;
    return s + lane * 0.0;
}

__global__ __launch_bounds__(256) void k(double* out, long long n) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double a[kLen];
    for (int i = 0; i < kLen; ++i) a[i] = (double)((t * 131 + i * 7) % 1000003);
    const double s = touch(a, (unsigned)(t * 2654435761u), threadIdx.x & 63);
    double c = 0.0;
    for (int i = 0; i < kLen; ++i) c += a[i] * (double)(i + 1);
    if (t < n) {
        out[2 * t] = s;
        out[2 * t + 1] = c;
    }
}

int main() {
    const long long n = 1LL << 20;
    double* d;
    if (hipMalloc(&d, 2 * n * sizeof(double)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3((unsigned)(n / 256)), dim3(256), 0, 0, d, n);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    double* h = (double*)malloc(2 * n * sizeof(double));
    hipMemcpy(h, d, 2 * n * sizeof(double), hipMemcpyDeviceToHost);
    long long bad = 0;
    static double a[kLen];
    for (long long t = 0; t < n; ++t) {
        for (int i = 0; i < kLen; ++i) a[i] = (double)((t * 131 + i * 7) % 1000003);
        double s = 0.0;
        unsigned hh = (unsigned)(t * 2654435761u);
        for (int i = 0; i < 64; ++i) {
            hh = hh * 1664525u + 1013904223u;
            const int k2 = (int)(hh >> 23) & (kLen - 1);
            s += a[k2];
            a[(k2 * 7 + i) & (kLen - 1)] += 1.0;
        }
        double c = 0.0;
        for (int i = 0; i < kLen; ++i) c += a[i] * (double)(i + 1);
        if (h[2 * t] != s || h[2 * t + 1] != c) ++bad;
    }
    printf("flat_private: %lld of %lld lanes differ\n", bad, n);
    return bad ? 1 : 0;
}
