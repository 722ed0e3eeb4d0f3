// sc_del.hip -- C-ABI launcher of the deletion-channel SC decoder (kernel template:
// sc_del_kern.h, instantiated per trellis length in sc_del_n*.hip).
//
// pcub_sc_decode_deletion replaces BinaryPolarEncoderDecoder.decode
// (BinaryPolarEncoderDecoder.py:71-99, recursion :223-325) when the xy vector
// distribution is the CollectionOfBinaryTrellises built by
// buildCollectionOfBinaryTrellises_uniformInput_deletion
// (VectorDistributions/CollectionOfBinaryTrellises.py:106-129) from a received word.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "polarcub_sc.h"
#include "sc_del_dense.h"
#include "sc_del_kern.h"
#include "trellis_wave.h"

using namespace pcub;

extern "C" int pcub_sc_dynamic_tiles(void);  // sc_bin.hip: work tiles from a counter

namespace pcub {
int del_w4_block(int tb);  // sc_del_w4.hip: threads a workgroup of del_kernel_w4(tb)
}

namespace {

constexpr int kMaxOnes = 3;
// received row stride: a segment's positions are relative to its start (16-bit vertex positions
// in trellis_body.h), the row index itself is an int
constexpr int kMaxStride = 1 << 24;

std::atomic<int> g_dense{1};  // the table-driven layout allowed (pcub_sc_set_deletion_dense)
std::atomic<int> g_dense_rate1{1};  // the 8-lane layout's rate-1 shortcut (pcub_sc_set_deletion_rate1)
std::atomic<int> g_dense_lanes{8};  // lanes a codeword of the table-driven layout (8, 16; 4 up to 64 trellises)
std::atomic<int> g_wave4{1};        // n0 = 4: the wave-per-task kernel allowed (pcub_sc_set_deletion_wave)
// the wave-per-task kernel keeps its codeword's received word bit-packed in LDS next to ~80 KB of its own
constexpr long long kW4MaxRxLds = 32768;

// Status words of table-checked launches (one ring per device; sc_del_kern.h, DelArgs::gate): a
// table-driven launch that rejects its table writes its launch id into its word, and the gated
// fallback launch behind it on the same stream decodes the batch without the table only then.
// Ids are unique per process, so a word left by an earlier launch never matches.  Limit: a word is
// reused after kGateRing launches, so at most kGateRing table-checked launches may be in flight on
// one device at once (streams included) -- one whose word was overwritten by a rejecting launch
// 2^16 ids later would skip its fallback.  2^16 words (512 KiB a device) put that far beyond any
// queue depth (round 5; 1,024 before).
constexpr int kGateRing = 1 << 16;
constexpr int kMaxDevices = 64;
std::mutex g_gate_mu;
unsigned long long* g_gate_ring[kMaxDevices] = {};
std::atomic<unsigned long long> g_gate_next{1};

// Per-launch group counters of the table-driven kernel (DelArgs::wtiles): a per-device ring, a slot a
// launch, zeroed on the launch's stream before it (kGateRing launches in flight before a slot is reused).
std::mutex g_ctr_mu;
unsigned long long* g_ctr_ring[kMaxDevices] = {};
std::atomic<unsigned long long> g_ctr_next{0};

int counter_slot(unsigned long long** slot, hipStream_t st) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    if (dev < 0 || dev >= kMaxDevices) return (int)hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> lk(g_ctr_mu);
        if (!g_ctr_ring[dev]) {
            void* p = nullptr;
            if ((e = hipMalloc(&p, kGateRing * sizeof(unsigned long long))) != hipSuccess) return (int)e;
            g_ctr_ring[dev] = (unsigned long long*)p;
        }
    }
    *slot = g_ctr_ring[dev] + (g_ctr_next.fetch_add(1) % kGateRing);
    return (int)hipMemsetAsync(*slot, 0, sizeof(unsigned long long), st);
}

int gate_slot(unsigned long long** slot, unsigned long long* id) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    if (dev < 0 || dev >= kMaxDevices) return (int)hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_gate_mu);
    if (!g_gate_ring[dev]) {
        void* p = nullptr;
        if ((e = hipMalloc(&p, kGateRing * sizeof(unsigned long long))) != hipSuccess) return (int)e;
        if ((e = hipMemset(p, 0, kGateRing * sizeof(unsigned long long))) != hipSuccess) return (int)e;
        g_gate_ring[dev] = (unsigned long long*)p;
    }
    *id = g_gate_next.fetch_add(1);
    *slot = g_gate_ring[dev] + (*id % kGateRing);
    return 0;
}

// the table header (sc_del_kern.h, tab_ok): magic, n0, pd, zeros
__device__ void tab_header(double* tab, int n0, double pd) {
    tab[0] = from_bits((long long)kTabMagic);
    tab[1] = (double)n0;
    tab[2] = pd;
    for (int i = 3; i < kTabHdr; ++i) tab[i] = 0.0;
}

// the n0 = 3 segment-state table: one thread per entry, the header then 512 x 256 doubles (entry j
// of a row: value k = floor(log2(j + 1)) after history j + 1 - 2^k; entry 255: padding)
__global__ __launch_bounds__(256) void k_del_n03_table(double pd, double* tab) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) tab_header(tab, 3, pd);
    if (i >= kN03States * kN03Row) return;
    const int st = i / kN03Row, j = i % kN03Row;
    if (j == kN03Row - 1) {
        tab[kTabHdr + i] = 0.0;
        return;
    }
    int k = 0;
    while ((2 << k) <= j + 1) ++k;
    tab[kTabHdr + i] = n03_table_entry(st, k, (uint32_t)(j + 1 - (1 << k)), pd);
}

// the n0 = 2 table (trellis_n02.h): the header, then one thread per (state, child) row part (entry 15
// of every row padding)
__global__ __launch_bounds__(256) void k_del_n02_table(double pd, double* tab) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) tab_header(tab, 2, pd);
    if (i < kN02States * 5) n02_table_entry(i / 5, i % 5, pd, tab + kTabHdr + (i / 5) * kN02Row);
    if (i < kN02States) tab[kTabHdr + i * kN02Row + kN02Row - 1] = 0.0;
}

DelKern del_kernel(int n0, int tb, bool exp, int ones) {
    if (ones < 0 || ones > kMaxOnes) return nullptr;
    const int oc = ones > 0 ? kMaxOnes : 0;
    if (tb > 8) return n0 == 4 && !exp && oc == 0 ? del_kernel_n4_wide(tb) : nullptr;
#define PCUB_DEL_PICK(k) \
    case k: return exp ? del_kernel_n##k##_x(tb, oc) : oc == 0 ? del_kernel_n##k##_d0(tb) : del_kernel_n##k##_d3(tb);
    switch (n0) {
        PCUB_DEL_PICK(1)
        PCUB_DEL_PICK(2)
        PCUB_DEL_PICK(3)
        PCUB_DEL_PICK(4)
        default: return nullptr;
    }
#undef PCUB_DEL_PICK
}

// comb(ones, i) * (1 - pd)^i * pd^(ones - i), left to right as the reference evaluates it
// (BinaryTrellis.py:343-345), with libm pow like CPython's float ** int.
OnesProbs ones_probs(int ones, double pd) {
    OnesProbs op;
    op.ones = ones;
    for (int i = 0; i < 4; ++i) op.pr[i] = 1.0;
    if (ones <= 0) return op;
    double comb = 1.0;
    for (int i = 0; i <= ones; ++i) {
        if (i > 0) comb = comb * (double)(ones - i + 1) / (double)i;  // small exact integers
        op.pr[i] = comb * std::pow(1.0 - pd, (double)i) * std::pow(pd, (double)(ones - i));
    }
    return op;
}

// the table-driven layout (sc_del_dense.h) when the stage has a table: n0 = 2 (the caller's, or
// built per workgroup) or n0 = 3 with a table given (checked on the device: tab_ok), no ones,
// 16 .. 256 trellises, and the group's received words fit LDS bit-packed
// lanes a codeword of the table-driven layout for 2^tb trellises (pcub_sc_set_deletion_lanes)
int dense_lanes(int tb) {
    const int g = g_dense_lanes.load(std::memory_order_relaxed);
    return (tb <= 6 || g != 4) ? g : 8;  // 4 lanes only up to 64 trellises
}

bool use_dense(int n, int n0, int ones, int stride, const double* table) {
    const long long rw = ((long long)stride + 31) / 32;
    const long long cpb = kDelBlock / dense_lanes(n - n0);
    return g_dense.load(std::memory_order_relaxed) && ones == 0 && (n0 == 2 || (n0 == 3 && table)) &&
           n - n0 >= 4 && cpb * rw * 4 <= kDenseMaxRxLds && del_kernel_dense(n0, n - n0, false, dense_lanes(n - n0)) != nullptr;
}

// A persistent grid for kernel k: one resident grid striding over the codeword groups.  The occupancy
// API reports one workgroup a CU too many for 256-thread blocks at 97 .. 112 SGPRs
// (MI355X_MICROARCH.md, occupancy row): 800 / (112 + 16) = 6 waves a SIMD at most, and an over-size
// persistent grid leaves its last workgroups to run after the others.
long long resident_grid(DelKern k, size_t lds, long long grid) {
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kDelBlock, lds) == hipSuccess && cus > 0 && occ > 0) {
        const long long res = (long long)cus * (occ < 6 ? occ : 6);
        if (grid > res) grid = res;
    }
    return grid;
}

int launch_del(bool exp, const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n, int32_t n0,
               int32_t ones, double pd, const uint32_t* frozen_mask, const uint32_t* frozen_val,
               const uint32_t* frozen_val_cw, int32_t K, uint32_t* info_words, uint32_t* xhat_words, double* leaf,
               const double* table, void* stream) {
    const DelKern kern = del_kernel(n0, n - n0, exp, ones);
    if (!kern || B < 0 || stride < 0 || stride > kMaxStride || !frozen_mask || (!frozen_val && !frozen_val_cw))
        return PCUB_EINVAL;
    if (K < 0 || K > (1 << n) || (!exp && K > 0 && !info_words) || (B > 0 && (!rx || !rx_len))) return PCUB_EINVAL;
    if (exp && !leaf) return PCUB_EINVAL;
    if (!(pd >= 0.0 && pd <= 1.0)) return PCUB_EINVAL;
    if (B == 0) return 0;
    DelArgs A;
    A.rx = rx;
    A.rx_len = rx_len;
    A.B = B;
    A.stride = stride;
    A.n = n;
    A.pd = pd;
    A.op = ones_probs(ones, pd);
    A.fmask = frozen_mask;
    A.fval = frozen_val;
    A.fval_cw = frozen_val_cw;
    A.info = info_words;
    A.xhat = xhat_words;
    A.leaf = leaf;
    A.tab = ((n0 == 2 || n0 == 3) && ones == 0) ? table : nullptr;
    A.gate = nullptr;
    A.gate_id = 0;
    const long long rw = ((long long)stride + 31) / 32;
    // n0 = 4 without ones (main_deletion's n = 12 .. 14): one wave a (trellis, depth-3 node) task, the
    // trellises in LDS (sc_del_w4.hip), codewords from a per-launch counter
    const int w4m = g_wave4.load(std::memory_order_relaxed);
    if (!exp && n0 == 4 && ones == 0 && w4m && rw * 4 <= kW4MaxRxLds) {
        const DelKern wk = del_kernel_w4(n - n0, 0);
        // (the kernel's LDS is ~140 KB before the packed row: a row too long for what is left goes to the
        // lane kernel)
        int w4occ = 0;
        if (wk && hipOccupancyMaxActiveBlocksPerMultiprocessor(&w4occ, wk, del_w4_block(n - n0), (size_t)(rw * 4)) != hipSuccess)
            w4occ = 0;
        if (wk && w4occ > 0) {
            A.rw = (int)rw;
            A.gate_id = w4m == 3 ? 1ull : 0ull;  // diagnostics: tasks skipped
            const size_t lds = (size_t)(rw * 4);
            // one resident workgroup a CU (k_sc_del_w4's launch bounds), at most one a codeword
            const int wblk = del_w4_block(n - n0);
            long long grid = B;
            {
                int dev = 0, cus = 0;
                if (hipGetDevice(&dev) == hipSuccess &&
                    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0 &&
                    grid > (long long)cus * w4occ)
                    grid = (long long)cus * w4occ;
            }
            if (pcub_sc_dynamic_tiles()) {
                const int rc = counter_slot(&A.wtiles, (hipStream_t)stream);
                if (rc) return rc;
            }
            // the per-trellis depth-1 / depth-2 caches of the resident workgroups (trellis_wave.h), a
            // stream-ordered workspace in the export-only leaf slot (this kernel never exports)
            void* ws = nullptr;
            hipError_t e = hipMallocAsync(&ws, (size_t)grid * ((size_t)1 << (n - n0)) * kW4Cache, (hipStream_t)stream);
            if (e != hipSuccess) return (int)e;
            A.leaf = (double*)ws;
            hipLaunchKernelGGL(wk, dim3((unsigned)grid), dim3(wblk), lds, (hipStream_t)stream, A);
            const int rc = (int)hipGetLastError();
            e = hipFreeAsync(ws, (hipStream_t)stream);
            return rc ? rc : (int)e;
        }
    }
    const bool dense = !exp && use_dense(n, n0, ones, stride, table);
    // the table-driven kernel checks the caller's table on the device (n0 = 3, and n0 = 2 with a table
    // given); behind it on the stream goes a gated fallback that decodes only if the check failed:
    // for n0 = 2 the table-driven kernel that builds its own table, for n0 = 3 k_sc_del without one
    const bool checked = dense && A.tab;
    if (checked) {
        const int rc = gate_slot(&A.gate, &A.gate_id);
        if (rc) return rc;
    }
    const int dg = dense_lanes(n - n0);
    DelKern k = dense ? del_kernel_dense(n0, n - n0, n0 == 2 && A.tab, dg) : kern;
    if (dense && dg == 8 && !g_dense_rate1.load(std::memory_order_relaxed)) {
        DelKern k0 = del_kernel_dense(n0, n - n0, n0 == 2 && A.tab, dg, false);
        if (k0) k = k0;
    }
    // the general kernel's workgroup: 256 threads, or T for 512 / 1024 trellises (one codeword)
    const int blk = dense ? kDelBlock : ((n - n0) > 8 ? 1 << (n - n0) : kDelBlock);
    long long cpb = dense ? kDelBlock / dg : blk >> (n - n0);
    long long grid = (B + cpb - 1) / cpb;
    // bit-packed received words in LDS when the group's words fit in 32 KiB (always for
    // the 64-trellis shapes; very long padded rows of small codes parse from HBM)
    A.rw = (dense || cpb * rw * 4 <= 32768) ? (int)rw : 0;
    size_t lds = A.rw ? (size_t)(cpb * rw * 4) : 0;
    // the table-driven kernel's staging area for its group's raw rows (sc_del_dense.h)
    if (dense && dense_stage_bytes(stride, rx, (int)cpb))
        lds = (size_t)(dense_stage_off((int)rw, (int)cpb) * 4 + dense_stage_bytes(stride, rx, (int)cpb));
    // n0 = 2 without ones (and the table-driven layout): each workgroup first builds or copies the
    // segment-state table, so the launch is persistent
    if (dense || (n0 == 2 && ones == 0)) grid = resident_grid(k, lds, grid);
    if (grid * blk > 0xffffffffLL) return PCUB_EINVAL;  // 32-bit dispatch grid (work-items)
    if (dense && pcub_sc_dynamic_tiles()) {
        const int rc = counter_slot(&A.wtiles, (hipStream_t)stream);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(blk), lds, (hipStream_t)stream, A);
    int rc = (int)hipGetLastError();
    if (rc || !checked) return rc;
    // the gated fallback: the same batch without the table, on a resident grid (its workgroups read
    // the status word and leave when the table-driven launch succeeded)
    DelArgs F = A;
    F.tab = nullptr;
    F.wtiles = nullptr;  // the gated fallback keeps the static stride
    const bool fb_dense = n0 == 2;
    const DelKern fk = fb_dense ? del_kernel_dense(2, n - n0, false, dg) : kern;
    const long long fcpb = fb_dense ? kDelBlock / dg : kDelBlock >> (n - n0);
    F.rw = (fb_dense || fcpb * rw * 4 <= 32768) ? (int)rw : 0;
    size_t flds = F.rw ? (size_t)(fcpb * rw * 4) : 0;
    if (fb_dense && dense_stage_bytes(stride, rx, (int)fcpb))
        flds = (size_t)(dense_stage_off((int)rw, (int)fcpb) * 4 + dense_stage_bytes(stride, rx, (int)fcpb));
    const long long fgrid = resident_grid(fk, flds, (B + fcpb - 1) / fcpb);
    hipLaunchKernelGGL(fk, dim3((unsigned)fgrid), dim3(kDelBlock), flds, (hipStream_t)stream, F);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" int pcub_sc_deletion_supported(int32_t n, int32_t n0, int32_t ones) {
    return del_kernel(n0, n - n0, false, ones) != nullptr;
}

extern "C" int pcub_sc_leaf_deletion_supported(int32_t n, int32_t n0, int32_t ones) {
    return del_kernel(n0, n - n0, true, ones) != nullptr;
}

extern "C" int pcub_sc_decode_deletion(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n,
                                       int32_t n0, int32_t ones, double pd, const uint32_t* frozen_mask,
                                       const uint32_t* frozen_val, int32_t K, uint32_t* info_words,
                                       uint32_t* xhat_words, void* stream) {
    if (!frozen_val) return PCUB_EINVAL;
    return launch_del(false, rx, rx_len, B, stride, n, n0, ones, pd, frozen_mask, frozen_val, nullptr, K, info_words,
                      xhat_words, nullptr, nullptr, stream);
}

extern "C" int pcub_sc_decode_deletion_tab(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride,
                                           int32_t n, int32_t n0, int32_t ones, double pd, const uint32_t* frozen_mask,
                                           const uint32_t* frozen_val, int32_t K, uint32_t* info_words,
                                           uint32_t* xhat_words, const double* table, void* stream) {
    if (!frozen_val) return PCUB_EINVAL;
    return launch_del(false, rx, rx_len, B, stride, n, n0, ones, pd, frozen_mask, frozen_val, nullptr, K, info_words,
                      xhat_words, nullptr, table, stream);
}

extern "C" int pcub_sc_leaf_deletion(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n,
                                     int32_t n0, int32_t ones, double pd, const uint32_t* frozen_mask,
                                     const uint32_t* frozen_val, const uint32_t* frozen_val_cw, int32_t K,
                                     uint32_t* info_words, uint32_t* xhat_words, double* leaf, void* stream) {
    return launch_del(true, rx, rx_len, B, stride, n, n0, ones, pd, frozen_mask, frozen_val, frozen_val_cw, K,
                      info_words, xhat_words, leaf, nullptr, stream);
}

extern "C" int pcub_sc_leaf_deletion_tab(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride,
                                         int32_t n, int32_t n0, int32_t ones, double pd, const uint32_t* frozen_mask,
                                         const uint32_t* frozen_val, const uint32_t* frozen_val_cw, int32_t K,
                                         uint32_t* info_words, uint32_t* xhat_words, double* leaf, const double* table,
                                         void* stream) {
    return launch_del(true, rx, rx_len, B, stride, n, n0, ones, pd, frozen_mask, frozen_val, frozen_val_cw, K,
                      info_words, xhat_words, leaf, table, stream);
}

// Tuning hook (not part of the stable ABI): lanes a codeword of the table-driven deletion layout,
// 8 (the default), 16, or 4 (up to 64 trellises; 8 beyond); returns the previous value, or -1.
extern "C" int pcub_sc_set_deletion_lanes(int32_t g) {
    if (g != 4 && g != 8 && g != 16) return -1;
    return g_dense_lanes.exchange(g);
}

// Diagnostic (not part of the stable ABI): 0 runs the 8-lane table-driven kernel's subtrees without
// the rate-1 shortcut where such a twin is built (n0 = 2 with a table, 64 / 256 trellises); the A/B
// of DESIGN 3.2.  Decisions are identical either way.  Returns the previous setting.
extern "C" int pcub_sc_set_deletion_rate1(int32_t on) { return g_dense_rate1.exchange(on ? 1 : 0); }

// Diagnostic (not part of the stable ABI; 3: the wave kernel with its tasks skipped, a timing probe): 0 sends
// n0 = 4 decodes back to the lane-per-trellis kernel
// k_sc_del instead of the wave-per-task kernel (sc_del_w4.hip); the A/B of DESIGN 3.2.  Decisions are
// identical either way.  Returns the previous setting.
extern "C" int pcub_sc_set_deletion_wave(int32_t on) { return g_wave4.exchange(on < 0 ? 0 : on > 3 ? 3 : on); }

extern "C" int pcub_sc_set_deletion_dense(int32_t on) {
    return g_dense.exchange(on ? 1 : 0);
}

extern "C" int pcub_sc_deletion_dense_layout(int32_t n, int32_t n0, int32_t ones, int32_t stride, const double* table,
                                             double pd) {
    return del_kernel(n0, n - n0, false, ones) != nullptr && stride >= 0 && stride <= kMaxStride &&
           use_dense(n, n0, ones, stride, table);
}

extern "C" int64_t pcub_sc_deletion_table_bytes(int32_t n0) {
    if (n0 == 2) return (int64_t)(kTabHdr + kN02States * kN02Row) * (int64_t)sizeof(double);
    return n0 == 3 ? (int64_t)(kTabHdr + kN03States * kN03Row) * (int64_t)sizeof(double) : 0;
}

extern "C" int pcub_sc_deletion_build_table(int32_t n0, double pd, double* table, void* stream) {
    if ((n0 != 2 && n0 != 3) || !table || ((uintptr_t)table & 7u) || !(pd >= 0.0 && pd <= 1.0)) return PCUB_EINVAL;
    if (n0 == 2)
        hipLaunchKernelGGL(k_del_n02_table, dim3(1), dim3(256), 0, (hipStream_t)stream, pd, table);
    else
        hipLaunchKernelGGL(k_del_n03_table, dim3(kN03States * kN03Row / 256), dim3(256), 0, (hipStream_t)stream, pd,
                           table);
    return (int)hipGetLastError();
}
