// sc_del_w4.hip -- deletion-channel SC decode for 16-input trellises (n0 = 4, no guard-band ones):
// main_deletion.py's n0 = n // 3 at n = 12 .. 14 (:100), 64 .. 1024 trellises a codeword.
//
// Replaces BinaryPolarEncoderDecoder.decode (BinaryPolarEncoderDecoder.py:71-99, recursion
// :223-325) over the CollectionOfBinaryTrellises of a received word
// (VectorDistributions/CollectionOfBinaryTrellises.py:55-82, 106-129) for those shapes, with the
// trellis levels of trellis_wave.h: one wave a (trellis, depth-3 node) task, its trellises in the
// wave's LDS, instead of k_sc_del's one lane a trellis with 22.6 KB of private memory.
//
// Workgroup: 256 threads, one codeword at a time (codewords from a per-launch counter).  For each of
// the 8 depth-3 nodes k, the four waves take the codeword's trellises in turn and leave each one's
// three rows (minus; plus after decision 0 / 1) in LDS at its half-split position bitrev(t); wave 0
// then decodes the memoryless node of the minus rows (16 lanes, T / 16 values a lane: the binary
// kernel's register subtree, as k_sc_del's T >= 64 path), every trellis picks its plus row by its
// decision, and wave 0 decodes that node.  A node whose two memoryless subtrees are both rate-0 skips
// its tasks (its decisions are the frozen values whatever the rows).  The 16 decisions of a trellis
// re-encode to its 16 x_hat bits (w4_enc16).
#include <hip/hip_runtime.h>

#include "sc_del_kern.h"
#include "trellis_wave.h"

namespace pcub {

namespace {

// run a phase on one lane of the wave, then make its LDS writes visible to the wave's other lanes
struct W4WaveRun {
    int lane;
    template <class F>
    __device__ __forceinline__ void operator()(F&& f) const {
        f(lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
};

template <int T>
__device__ __forceinline__ uint64_t w4_window(const uint32_t* w, int kk, int wi) {
    const int us = kk * T + 64 * wi;
    return (uint64_t)w[us >> 5] | ((uint64_t)w[(us >> 5) + 1] << 32);
}

// collapse point kk's memoryless node: all frozen?
template <int T>
__device__ __forceinline__ bool w4_rate0(const uint32_t* fmask, int kk) {
    bool r = true;
    for (int i = 0; i < T / 32; ++i) r = r && fmask[kk * (T / 32) + i] == 0xffffffffu;
    return r;
}

// SC over collapse point kk's memoryless node of the T rows vals[p] (half-split positions): wave 0,
// 16 lanes (the other groups decode copies); bits to xb[p / 16] bit p % 16, decisions to xub
template <int TB>
__device__ __forceinline__ void w4_subtree(const DelArgs& A, const double* vals, int kk, unsigned long long* xb,
                                           unsigned long long* xub) {
    constexpr int T = 1 << TB, NW = T / 64, LV = T / 16;
    const int lane = threadIdx.x & 63;
    if ((threadIdx.x >> 6) == 0) {
        uint64_t fm[NW], fv[NW], ubl[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            fm[w] = w4_window<T>(A.fmask, kk, w);
            fv[w] = w4_window<T>(A.fval, kk, w);
            ubl[w] = 0;
        }
        const int j = lane & 15;
        double vv[LV];
#pragma unroll
        for (int t = 0; t < LV; ++t) vv[t] = vals[j + 16 * t];
        typename DelWin<LV, NW>::Bits bits;
        if constexpr (NW == 1) bits = WinTree<LV, 16, 1>::run(vv, ubl, fm, fv, lane);
        else bits = DelWin<LV, NW>::run(vv, ubl, fm, fv, lane);
#pragma unroll
        for (int t = 0; t < LV; ++t) {
            const unsigned long long bal = __ballot((bits >> t) & 1u);
            if (lane == 0) xb[t] = bal;
        }
        if (lane == 0)
#pragma unroll
            for (int w = 0; w < NW; ++w) xub[w] = ubl[w];
    }
    __syncthreads();
}

// collapse point kk's information bits (its decisions at the unfrozen positions, in order) into the
// codeword's bit buffer at offset ib; returns the count
template <int T>
__device__ __forceinline__ int w4_info(const DelArgs& A, int kk, const unsigned long long* xub, uint32_t* infol, int ib) {
    constexpr int NW = T / 64;
    int total = 0, before = 0;
    const int w = (int)threadIdx.x;
    for (int i = 0; i < NW; ++i) {
        const int c = __builtin_popcountll(~w4_window<T>(A.fmask, kk, i));
        before += i < w ? c : 0;
        total += c;
    }
    if (w < NW) {
        const uint64_t ub = xub[w];
        int off = ib + before;
        for (uint64_t im = ~w4_window<T>(A.fmask, kk, w); im != 0ull; im &= im - 1ull, ++off)
            if ((ub >> __builtin_ctzll(im)) & 1ull) atomicOr(&infol[off >> 5], 1u << (off & 31));
    }
    return total;
}

// WPB task waves a workgroup, one workgroup a CU: twelve (768 threads) up to 512 trellises, ten at
// 1024 (the codeword's rows take more LDS).  One workgroup a CU asks the register allocator for 170
// VGPRs: the task phases need ~120, and the memoryless subtree (wave 0, ~2 % of the time) spills
// instead of pushing every wave to 256 -- at eight waves a CU the tasks ran 31 % slower than at twelve
// (scripts/dbg/w4_tasks.hip).
template <int TB, int WPB>
__global__ __launch_bounds__(WPB * 64, 1) void k_sc_del_w4(DelArgs A) {
    constexpr int BLK = WPB * 64;
    constexpr int T = 1 << TB;
    constexpr int LV = T / 16, NW = T / 64;
    constexpr int WPC = T / 2;  // x_hat words a codeword (16 T bits)
    __shared__ W4Buf wb[WPB];
    __shared__ double vm[T], vp0[T], vp1[T];
    __shared__ uint16_t hist[T], sy[T];
    __shared__ uint8_t sm[T];
    __shared__ uint8_t xmb[T];
    __shared__ unsigned long long xb[LV], xub[NW];
    __shared__ uint32_t infol[WPC];
    __shared__ long long s_next;
    __shared__ int s_task[8];  // node k's next task (the waves take the codeword's trellises in turn)
    extern __shared__ uint32_t rxb[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // this workgroup's trellis caches (the launcher's workspace, kW4Cache bytes a trellis), or none
    uint8_t* cache = A.leaf ? reinterpret_cast<uint8_t*>(A.leaf) + (size_t)blockIdx.x * T * kW4Cache : nullptr;
    for (long long it = 0;; ++it) {
        long long cw;
        if (A.wtiles) {
            if (threadIdx.x == 0) s_next = (long long)atomicAdd(A.wtiles, 1ull);
            __syncthreads();
            cw = s_next;
        } else {
            cw = (long long)blockIdx.x + it * (long long)gridDim.x;
        }
        if (cw >= A.B) break;
        // the received word, bit-packed; each trellis's segment (m > 16: no edges)
        pack_rows<1, BLK>(A, cw, rxb, lane);
        for (int i = threadIdx.x; i < WPC; i += BLK) infol[i] = 0u;
        __syncthreads();
        int len = A.rx_len[cw];
        len = len < 0 ? 0 : (len > A.stride ? A.stride : len);
        for (int t = threadIdx.x; t < T; t += BLK) {
            int s, m;
            segment_of_packed(rxb, len, TB, t, s, m);
            uint32_t y = 0;
            if (m > 0 && m <= kW4L) {
                const int w0 = s >> 5;
                const uint64_t lo = rxb[w0], hi = (w0 + 1 < A.rw) ? rxb[w0 + 1] : 0u;
                y = (uint32_t)(((hi << 32) | lo) >> (s & 31)) & (uint32_t)((1u << m) - 1u);
            }
            sm[t] = (uint8_t)(m <= kW4L ? m : kW4L + 1);
            sy[t] = (uint16_t)y;
            hist[t] = 0;
        }
        if (threadIdx.x < 8) s_task[threadIdx.x] = 0;
        __syncthreads();
        int ib = 0;  // information bits so far
        int have1 = -1, have2 = -1;  // the depth-1 (k >> 2) / depth-2 (k >> 1) trellises in the cache
#pragma unroll 1
        for (int k = 0; k < 8; ++k) {
            const int km = 2 * k, kp = 2 * k + 1;
            // (A.gate_id bit 0, diagnostics only: skip the tasks, so a launch times the rest)
            if (!(A.gate_id & 1ull) && !(w4_rate0<T>(A.fmask, km) && w4_rate0<T>(A.fmask, kp))) {
                int mode = 0;
                if (cache) {
                    mode = have2 == (k >> 1) ? kW4Load2 : ((have1 == (k >> 2) ? kW4Load1 : kW4Save1) | kW4Save2);
                    if (mode & kW4Save1) have1 = k >> 2;
                    have2 = k >> 1;
                }
                // up to 256 trellises the tasks come from a counter, not a fixed stride: their costs differ
                // (segment lengths), and the node's subtree waits for the slowest wave (n = 12: 60.3 ->
                // 68.2 k cw/s); at 512 / 1024 the fixed stride measured faster (32.7 / 13.5 k against 31.5 /
                // 10.1 k), so it stays there
                constexpr bool kDyn = TB <= 8;
#pragma unroll 1
                for (int ts = wv;; ts += WPB) {
                    int t = ts;
                    if constexpr (kDyn) {
                        t = 0;
                        if (lane == 0) t = atomicAdd(&s_task[k], 1);
                        t = __builtin_amdgcn_readfirstlane(t);
                    }
                    if (t >= T) break;
                    // the task's segment and history are wave-uniform: scalar registers
                    W4Dims D;
                    D.set(__builtin_amdgcn_readfirstlane((int)sm[t]), (uint32_t)__builtin_amdgcn_readfirstlane((int)sy[t]),
                          A.pd);
                    w4_task(W4WaveRun{lane}, wb[wv], D, k, (uint32_t)__builtin_amdgcn_readfirstlane((int)hist[t]),
                            cache ? cache + (size_t)t * kW4Cache : nullptr, mode);
                    if (lane < 3) {
                        const int p = (int)bitrev((uint32_t)t, TB);
                        double* dst = lane == 0 ? vm : lane == 1 ? vp0 : vp1;
                        dst[p] = wb[wv].out[lane];
                    }
                }
            }
            __syncthreads();
            // the minus node, then every position's plus row by its decision, then the plus node
            w4_subtree<TB>(A, vm, km, xb, xub);
            ib += w4_info<T>(A, km, xub, infol, ib);
            for (int p = threadIdx.x; p < T; p += BLK) {
                const uint32_t x = (uint32_t)(xb[p >> 4] >> (p & 15)) & 1u;
                xmb[p] = (uint8_t)x;
                vm[p] = x ? vp1[p] : vp0[p];
            }
            __syncthreads();
            w4_subtree<TB>(A, vm, kp, xb, xub);
            ib += w4_info<T>(A, kp, xub, infol, ib);
            for (int t = threadIdx.x; t < T; t += BLK) {
                const int p = (int)bitrev((uint32_t)t, TB);
                const uint32_t xp = (uint32_t)(xb[p >> 4] >> (p & 15)) & 1u;
                hist[t] = (uint16_t)(hist[t] | ((uint32_t)xmb[p] << km) | (xp << kp));
            }
            __syncthreads();
        }
        // x_hat: trellis t's slice is natural positions [16 t, 16 t + 16)
        if (A.xhat)
            for (int i = threadIdx.x; i < WPC; i += BLK)
                A.xhat[(long long)i * A.B + cw] = w4_enc16(hist[2 * i]) | (w4_enc16(hist[2 * i + 1]) << 16);
        if (A.info)
            for (int i = threadIdx.x; i < (ib + 31) / 32; i += BLK) A.info[(long long)i * A.B + cw] = infol[i];
        __syncthreads();  // rxb / sm / hist / infol are rewritten by the next codeword
    }
}

}  // namespace

DelKern del_kernel_w4(int tb, int alt) {
    (void)alt;
    switch (tb) {
        case 6: return k_sc_del_w4<6, 12>;
        case 7: return k_sc_del_w4<7, 12>;
        case 8: return k_sc_del_w4<8, 12>;
        case 9: return k_sc_del_w4<9, 12>;
        case 10: return k_sc_del_w4<10, 10>;
        default: return nullptr;
    }
}

// threads a workgroup of del_kernel_w4(tb)
int del_w4_block(int tb) { return (tb == 10 ? 10 : 12) * 64; }

}  // namespace pcub
