// Microbenchmark of the n0 = 4 wave-per-task trellis stage alone (trellis_wave.h), test-only: random
// segments with n = 12's length distribution (pd = 0.1, xi = 0.1), random decision histories, all 8
// depth-3 nodes; tasks a second for several launch shapes.  Build: hipcc --offload-arch=gfx950 -O3
// -ffp-contract=off -std=c++17 -I polarcub_amd/csrc -I include scripts/dbg/w4_tasks.hip -o w4_tasks
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "sc_del_kern.h"
#include "trellis_wave.h"

using namespace pcub;

struct WR {
    int lane;
    template <class F>
    __device__ __forceinline__ void operator()(F&& f) const {
        f(lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
};

// w4_task up to a stage: 1 = depth-1 edges, 2 = depth 1 complete, 3 = + depth-2 edges, 4 = depth 2
// complete, 5 = + depth-3 edges, 6 = + the middle-vertex order and layer 0's normaliser, 7 = everything
template <int STOP, class Run>
__device__ __forceinline__ void w4_task_upto(const Run& run, W4Buf& b, const W4Dims& D, int k, uint32_t hist) {
    if (D.m > kW4L) {
        run([&](int lane) { if (lane < 3) b.out[lane] = norm_pack(0.0, 0.0); });
        return;
    }
    const W4View A = w4_view_a(b), B = w4_view_b(b);
    const bool p1 = (k >> 2) & 1, p2 = (k >> 1) & 1, p3 = k & 1;
    const uint32_t d1 = p1 ? w4_enc8(hist, 0) : 0u;
    const uint32_t d2 = p2 ? w4_enc4(hist, (k >> 1) - 1) : 0u;
    const uint32_t d3 = p3 ? w4_enc2(hist, k - 1) : 0u;
    run([&](int lane) { w4_ph_edges(D, 0, A, A, d1, p1, lane); });
    if (STOP == 1) return;
    run([&](int lane) { w4_ph_rank(D, 1, A, b, lane); });
    run([&](int lane) { w4_ph_vkey(D, 1, A, b, lane); });
    run([&](int lane) { w4_ph_vrank(D, 1, A, b, lane); });
    run([&](int lane) { w4_ph_norder(D, 1, A, b, lane); });
    run([&](int lane) { w4_ph_nsum(D, 1, A, b, lane); });
    run([&](int lane) { w4_ph_ndiv(D, 1, A, b, lane); });
    if (STOP == 2) return;
    run([&](int lane) { w4_ph_edges(D, 1, A, B, d2, p2, lane); });
    if (STOP == 3) return;
    run([&](int lane) { w4_ph_rank(D, 2, B, b, lane); });
    run([&](int lane) { w4_ph_vkey(D, 2, B, b, lane); });
    run([&](int lane) { w4_ph_vrank(D, 2, B, b, lane); });
    run([&](int lane) { w4_ph_norder(D, 2, B, b, lane); });
    run([&](int lane) { w4_ph_nsum(D, 2, B, b, lane); });
    run([&](int lane) { w4_ph_ndiv(D, 2, B, b, lane); });
    if (STOP == 4) return;
    run([&](int lane) { w4_ph_edges(D, 2, B, A, d3, p3, lane); });
    if (STOP == 5) return;
    run([&](int lane) { w4_ph_f1(D, A, b, lane); });
    run([&](int lane) { w4_ph_f2(D, A, b, lane); });
    if (STOP == 6) return;
    run([&](int lane) { w4_ph_f3(D, A, b, lane); });
}

template <int STOP>
__global__ __launch_bounds__(64) void k_stage(const uint32_t* seg, const uint16_t* hist, double* rows, long long n, int k,
                                              double pd) {
    __shared__ W4Buf wb;
    const int lane = threadIdx.x & 63;
    for (long long t = blockIdx.x; t < n; t += gridDim.x) {
        const uint32_t sg = (uint32_t)__builtin_amdgcn_readfirstlane((int)seg[t]);
        W4Dims D;
        D.set((int)(sg >> 16), sg & 0xffffu, pd);
        w4_task_upto<STOP>(WR{lane}, wb, D, k, (uint32_t)__builtin_amdgcn_readfirstlane((int)hist[t]));
        if (lane < 3) rows[t * 3 + lane] = wb.out[lane];
    }
}

template <int STOP>
static void stage(const uint32_t* seg, const uint16_t* hist, double* rows, long long n) {
    int cus = 0, occ = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_stage<STOP>, 64, 0);
    const long long grid = (long long)cus * occ;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int k = 0; k < 8; ++k) hipLaunchKernelGGL((k_stage<STOP>), dim3(grid), dim3(64), 0, 0, seg, hist, rows, n, k, 0.1);
    hipEventRecord(a);
    for (int k = 0; k < 8; ++k) hipLaunchKernelGGL((k_stage<STOP>), dim3(grid), dim3(64), 0, 0, seg, hist, rows, n, k, 0.1);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::printf("stage %d: %8.2f ms for %lld tasks (%.1f ns a task on the GPU)\n", STOP, ms, 8 * n, ms * 1e6 / (8.0 * n));
}

template <int WPB, int MINB>
__global__ __launch_bounds__(WPB * 64, MINB) void k_tasks(const uint32_t* seg, const uint16_t* hist, double* rows,
                                                         long long n, int k, double pd) {
    __shared__ W4Buf wb[WPB];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (long long t = (long long)blockIdx.x * WPB + wv; t < n; t += (long long)gridDim.x * WPB) {
        const uint32_t sg = (uint32_t)__builtin_amdgcn_readfirstlane((int)seg[t]);
        W4Dims D;
        D.set((int)(sg >> 16), sg & 0xffffu, pd);
        w4_task(WR{lane}, wb[wv], D, k, (uint32_t)__builtin_amdgcn_readfirstlane((int)hist[t]));
        if (lane < 3) rows[t * 3 + lane] = wb[wv].out[lane];
    }
}

template <int WPB, int MINB>
static void run(const char* name, const uint32_t* seg, const uint16_t* hist, double* rows, long long n, int cap = 0) {
    int cus = 0, occ = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_tasks<WPB, MINB>, WPB * 64, 0);
    if (cap > 0 && cap < occ) occ = cap;
    const long long grid = (long long)cus * occ;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int k = 0; k < 8; ++k) hipLaunchKernelGGL((k_tasks<WPB, MINB>), dim3(grid), dim3(WPB * 64), 0, 0, seg, hist, rows, n, k, 0.1);
    hipEventRecord(a);
    for (int rep = 0; rep < 2; ++rep)
        for (int k = 0; k < 8; ++k)
            hipLaunchKernelGGL((k_tasks<WPB, MINB>), dim3(grid), dim3(WPB * 64), 0, 0, seg, hist, rows, n, k, 0.1);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double tasks = 2.0 * 8.0 * (double)n;
    std::printf("%-22s blocks/CU %2d  %8.2f ms  %8.2f M tasks/s  (n = 12: %.1f k cw/s at 2048 tasks a codeword)\n", name, occ,
                ms, tasks / (ms * 1e-3) / 1e6, tasks / (ms * 1e-3) / 2048.0 / 1e3);
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? std::atoll(argv[1]) : (1 << 20);
    // segment lengths at n = 12 (measured from the reference's guard bands + channel, pd = 0.1)
    const double pm[17] = {0.0, 0.0008, 0.0007, 0.0013, 0.0025, 0.0038, 0.0089, 0.0171, 0.027, 0.0473,
                           0.0736, 0.1125, 0.1497, 0.1929, 0.1845, 0.1282, 0.0493};
    std::mt19937_64 rng(5);
    std::discrete_distribution<int> dm(pm, pm + 17);
    std::vector<uint32_t> seg(n);
    std::vector<uint16_t> hist(n);
    for (long long i = 0; i < n; ++i) {
        const int m = dm(rng);
        const uint32_t y = (uint32_t)(rng() & ((1u << m) - 1u));
        seg[i] = ((uint32_t)m << 16) | y;
        hist[i] = (uint16_t)rng();
    }
    uint32_t* dseg;
    uint16_t* dhist;
    double* drows;
    hipMalloc(&dseg, n * 4);
    hipMalloc(&dhist, n * 2);
    hipMalloc(&drows, n * 24);
    hipMemcpy(dseg, seg.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dhist, hist.data(), n * 2, hipMemcpyHostToDevice);
    run<1, 1>("1 wave/WG", dseg, dhist, drows, n);
    run<1, 1>("1 wave/WG, 4 a CU", dseg, dhist, drows, n, 4);
    run<1, 1>("1 wave/WG, 8 a CU", dseg, dhist, drows, n, 8);
    run<1, 1>("1 wave/WG, 10 a CU", dseg, dhist, drows, n, 10);
    stage<1>(dseg, dhist, drows, n);
    stage<2>(dseg, dhist, drows, n);
    stage<3>(dseg, dhist, drows, n);
    stage<4>(dseg, dhist, drows, n);
    stage<5>(dseg, dhist, drows, n);
    stage<6>(dseg, dhist, drows, n);
    stage<7>(dseg, dhist, drows, n);
    std::printf("sizeof(W4Buf) = %zu\n", sizeof(W4Buf));
    return (int)hipGetLastError();
}
