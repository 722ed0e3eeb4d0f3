// sc_del_dense.h -- the table-driven deletion decoder: n0 = 2 or 3, no guard-band ones,
// 16 .. 256 trellises, decode mode.
//
// With a segment-state table (trellis_n02.h for n0 = 2, n03_table_entry for n0 = 3) a trellis
// costs one table load per subtree input, so the trellis stages no longer need a lane each:
// k_sc_del's layout (one lane per trellis, the memoryless subtree decoded by 16 lanes of wave 0
// after an LDS exchange and two barriers) leaves three waves of four idle in every subtree call.
// Here a codeword owns G lanes of one wave for the whole decode (G = 8 by default: eight codewords a
// wave, thirty-two a workgroup; 16 and, up to 64 trellises, 4 through pcub_sc_set_deletion_lanes):
// lane j holds the LV = T / G trellises at memoryless positions p = j + G t, looks their values
// up, and decodes the subtree in registers with the binary kernel's WinTree (DelWin at G = 16).
// No LDS exchange and no barrier inside the walk.
//
// Same decisions as k_sc_del (and the reference): the values are the table's, which are the
// per-lane values bit for bit (tests/emu/del_emu.cpp checks every one), the subtree is the same
// WinTree over the same 16-lane layout k_sc_del's wave 0 uses, and the segment parse is
// segment_of's descent (Guardbands.py:47-93) shared between the lane's trellises.
#pragma once

#include "sc_del_kern.h"

namespace pcub {

constexpr int kDenseG = 16;                     // lanes per codeword of the 16-lane form (DelWin's windows)
constexpr int kDenseCPB = kDelBlock / kDenseG;  // its codewords per workgroup (the staging helpers' default)
constexpr int kDenseMaxRxLds = 48 * 1024;       // bit-packed received words per workgroup, at most

// slot of subtree input k (history hist: bit i = the i-th returned bit) in a state's row
template <int N0>
PCUB_HD int dense_slot(int k, uint32_t hist) {
    if constexpr (N0 == 3) {
        return (1 << k) - 1 + (int)hist;
    } else {  // trellis_n02.h's order: [0] v1, [1 + xm] v2, [3 + ym] v3, [7 + 2 ym + xm'] v4
        const uint32_t h0 = hist & 1u, h1 = (hist >> 1) & 1u, ym = (h0 ^ h1) | (h1 << 1);
        return k == 0 ? 0 : k == 1 ? 1 + (int)h0 : k == 2 ? 3 + (int)ym : 7 + 2 * (int)ym + (int)((hist >> 2) & 1u);
    }
}

// the re-encoding DelNode / DelBase apply to a trellis's returned bits: x[2h] = ym[h] ^ yp[h],
// x[2h+1] = yp[h] over the two halves, recursively
template <int L>
PCUB_HD uint32_t enc_hist(uint32_t h) {
    if constexpr (L == 1) {
        return h & 1u;
    } else {
        constexpr int H = L / 2;
        const uint32_t ym = enc_hist<H>(h), yp = enc_hist<H>(h >> H);
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < H; ++i) x |= ((((ym ^ yp) >> i) & 1u) << (2 * i)) | (((yp >> i) & 1u) << (2 * i + 1));
        return x;
    }
}

constexpr int cbitrev(int x, int nbits) {
    int r = 0;
    for (int i = 0; i < nbits; ++i) r |= ((x >> i) & 1) << (nbits - 1 - i);
    return r;
}

// bits [s, s + m) of a bit-packed word (m <= 8, rw words)
PCUB_HD uint32_t packed_bits(const uint32_t* w, int s, int m, int rw) {
    if (m <= 0) return 0u;
    const int wi = s >> 5, sh = s & 31;
    uint64_t x = w[wi];
    if (sh + m > 32 && wi + 1 < rw) x |= (uint64_t)w[wi + 1] << 32;
    return (uint32_t)(x >> sh) & ((1u << m) - 1u);
}

// The segments of the 2^(TB-GB) trellises tr = jr * 2^(TB-GB) + i of one lane (removeDeletionGuardBands'
// descent, segment_of_packed): the GB halvings of jr (G = 2^GB lanes a codeword), shared by them, then a split per level, each
// range halved and both halves trimmed; entry i = [sa[i], se[i]).
template <int TB, int GB = 4>
PCUB_HD void dense_segments(const uint32_t* pw, int len, uint32_t jr, int* sa, int* se) {
    constexpr int TL = TB - GB;
    // four-word probes (trellis_body.h) at 128 trellises (n = 10: 85 -> 95 M cw/s); at 256 (n = 11:
    // 30.0 -> 29.1 M) and at 64 (C5: 1.02 -> 0.86 G) the plain scans are faster
    constexpr bool P4 = TB == 7;
    int a = 0, e = len;
    trim_range_packed<P4>(pw, a, e);
#pragma unroll
    for (int k = GB - 1; k >= 0; --k) {
        const int h = (e - a) / 2;
        if ((jr >> k) & 1u) a += h;
        else e = a + h;
        trim_range_packed<P4>(pw, a, e);
    }
    sa[0] = a;
    se[0] = e;
#pragma unroll
    for (int lev = 0; lev < TL; ++lev) {
#pragma unroll
        for (int i = (1 << lev) - 1; i >= 0; --i) {
            const int a0 = sa[i], e0 = se[i], h = (e0 - a0) / 2;
            int la = a0, le = a0 + h, ra = a0 + h, re = e0;
            trim_range_packed<P4>(pw, la, le);
            trim_range_packed<P4>(pw, ra, re);
            sa[2 * i] = la;
            se[2 * i] = le;
            sa[2 * i + 1] = ra;
            se[2 * i + 1] = re;
        }
    }
}

// Staged received words (round 5): a group's CPB rows are one contiguous run of CPB * stride
// bytes, so the workgroup reads them with 16-byte loads, a few a lane, into an LDS staging area,
// and the waves bit-pack their rows from there; pack_rows' byte loads cost a VMEM instruction
// and a ballot per 64 symbols of every row (12 dependent-latency loads per C5 codeword).  Long rows
// go in chunks of R rows (R a power of two, R * stride + 32 <= kDenseStageMax: at 8 lanes a codeword
// n = 8 stages all 32 rows at once, n = 10 four, n = 11 two), each chunk from the 16-byte boundary
// at or below its first byte.  The launcher sizes the LDS (dense_stage_bytes) and the kernel stages whenever that
// size is nonzero.
constexpr int kDenseStageMax = 24 * 1024;  // staging bytes per workgroup, at most

PCUB_HD int dense_stage_rows(int stride, int cpb = kDenseCPB) {
    int r = cpb;
    while (r > 0 && (long long)r * stride + 32 > kDenseStageMax) r >>= 1;
    return r;
}

PCUB_HD long long dense_stage_bytes(int stride, const void* rx, int cpb = kDenseCPB) {
    const int r = dense_stage_rows(stride, cpb);
    return (r > 0 && ((unsigned long long)rx & 15ull) == 0) ? (long long)r * stride + 32 : 0;  // + the chunk's misalignment, + the last 16-byte load's tail
}

// the staging area: after the packed rows, 16-byte aligned
PCUB_HD long long dense_stage_off(int rw, int cpb = kDenseCPB) { return (((long long)cpb * rw + 3) / 4) * 4; }

// bytes [a0, a0 + nb) of the batch's rows into stg (a0 16-byte aligned; bytes past the batch zero)
__device__ __forceinline__ void stage_bytes(const DelArgs& A, long long a0, uint8_t* stg, int nb) {
    const long long total = A.B * (long long)A.stride;  // bytes of the batch's rows
    for (int o = threadIdx.x * 16; o < nb; o += kDelBlock * 16) {
        const long long go = a0 + o;
        if (go + 16 <= total) {
            *(uint4*)(stg + o) = *(const uint4*)(A.rx + go);
        } else {
            for (int b = 0; b < 16; ++b) stg[o + b] = (go + b < total) ? A.rx[go + b] : (uint8_t)0;
        }
    }
}

// pack_rows over staged rows r0 .. r0 + R - 1 of the group (row r0 at stg0; LDS byte reads)
template <int CPB>
__device__ __forceinline__ void pack_staged(const DelArgs& A, long long grp, const uint8_t* stg0, int r0, int R,
                                            uint32_t* rxb, int lane) {
    const int nch = (A.rw * 32 + 63) / 64;
    for (int gg = r0 + (threadIdx.x >> 6); gg < r0 + R; gg += kDelBlock / 64) {
        long long cg = grp * CPB + gg;
        cg = cg < A.B ? cg : A.B - 1;
        const uint8_t* row = stg0 + (gg - r0) * A.stride;  // (a padding row's bytes are zero; it stores nothing)
        int ln = A.rx_len[cg];
        ln = ln < 0 ? 0 : (ln > A.stride ? A.stride : ln);
        for (int c0 = 0; c0 < nch; c0 += kPackU) {
            uint32_t b[kPackU];
#pragma unroll
            for (int u = 0; u < kPackU; ++u) {
                const int i = (c0 + u) * 64 + lane;
                b[u] = i < ln ? (uint32_t)row[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kPackU; ++u) {
                const unsigned long long msk = __ballot(b[u] == 1u);
                const int wi = 2 * (c0 + u) + (lane & 1);
                if (lane < 2 && wi < A.rw) rxb[gg * A.rw + wi] = (uint32_t)(msk >> (32 * lane));
            }
        }
    }
}

// GT (n0 = 2): the table comes built (pcub_sc_deletion_build_table) and is copied into LDS, instead
// of each workgroup building it: the build's registers (n02_table_entry) set the kernel's peak
// (89 -> 79 VGPRs at 64 trellises: 6 waves a SIMD instead of 5)
// waves a SIMD the register allocation must allow (the SGPR count, 97..112, caps it at 6)
// (8 lanes a codeword: at 6 waves the 80-VGPR cap spills 61 VGPRs, 148 B a lane, and still wins --
// C5 1,005 M vs 970 M at 5 waves (96 VGPRs, 26 spilled) and 876 M at 4 (127 VGPRs, none))
constexpr int dense_waves(int tb) { return tb <= 6 ? 6 : tb == 7 ? 5 : 3; }

// G lanes a codeword (round 5: 8, the default -- eight codewords a wave, T / 8 trellises a lane --
// runs the memoryless subtree's last three levels across lanes instead of four, and a wave
// instruction serves twice the codewords: C5 848 -> 1009 M cw/s, K = 64 303 -> 452 M, n = 10 77 -> 85 M;
// 4 lanes measured slower, 943 / 416 M)
// A trellis's state row and decision history share one packed field: (row << HB) | history, HB = 2^n0
// history bits; n0 = 2 (row < 2^10) packs two trellises a 32-bit word, n0 = 3 (row < 2^18) one.  The
// 8-lane layout holds LV = T / 8 trellises a lane, and the unpacked row[] / hist[] pairs (2 LV VGPRs)
// were a large part of what spilled at the 80-VGPR cap of 6 waves a SIMD.
template <int N0, int LV>
struct RowHist {
    static constexpr int HB = 1 << N0;                     // history bits
    static constexpr int PER = N0 == 2 ? 2 : 1;            // trellises a word
    static constexpr int FB = 32 / PER;                    // field bits
    static constexpr uint32_t FM = PER == 1 ? ~0u : ((1u << FB) - 1u);
    uint32_t w[(LV + PER - 1) / PER];
    PCUB_HD uint32_t field(int t) const { return (w[t / PER] >> (FB * (t % PER))) & FM; }
    PCUB_HD int row(int t) const { return (int)(field(t) >> HB); }
    PCUB_HD uint32_t hist(int t) const { return field(t) & ((1u << HB) - 1u); }
    PCUB_HD void set_row(int t, int r) { w[t / PER] |= ((uint32_t)r << HB) << (FB * (t % PER)); }
    PCUB_HD void add_bit(int t, uint32_t b, int k) { w[t / PER] |= (b << k) << (FB * (t % PER)); }
};

template <int N0, int TB, bool GT = false, int G = kDenseG, bool R1 = true>
__global__ __launch_bounds__(kDelBlock, dense_waves(TB)) void k_sc_del_dense(DelArgs A) {
    constexpr int GB = G == 16 ? 4 : G == 8 ? 3 : 2;
    static_assert(G == 16 || G == 8 || (G == 4 && TB <= 6), "16 or 8 lanes a codeword, or 4 up to 64 trellises");
    constexpr int L = 1 << N0, T = 1 << TB, LV = T / G, CPB = kDelBlock / G;
    constexpr int NW = T > 64 ? T / 64 : 1;
    constexpr int WPC = (T * L + 31) / 32;
    constexpr int ROW = N0 == 2 ? kN02Row : kN03Row;
    constexpr int TL = TB - GB;  // descent levels below the lane's shared prefix
    constexpr uint64_t WM = T >= 64 ? ~0ull : ((1ull << T) - 1ull);
    static_assert((N0 == 2 || N0 == 3) && TB >= 4 && TB <= 8, "dense deletion: n0 2, 3 and 16 .. 256 trellises");
    __shared__ double tab2[N0 == 2 ? kN02States * kN02Row : 1];
    __shared__ uint32_t xs[CPB * WPC];
    extern __shared__ uint32_t rxb[];
    if (A.gate && !(N0 == 3 || GT) && *A.gate != A.gate_id) return;  // a gated fallback (sc_del.hip)
    if constexpr (N0 == 3 || GT) {
        // the caller's table, checked on the device (one scalar load a workgroup): a table built for
        // another n0 or pd is never read; the launch marks its status word and the gated fallback
        // launch behind it decodes the batch without the table (sc_del.hip)
        if (!tab_ok(A.tab, N0, A.pd)) {
            if (threadIdx.x == 0 && A.gate) *A.gate = A.gate_id;
            return;
        }
    }
    const double* tab;  // n0 = 3 (and n0 = 2 with GT): the caller's table, past its header
    if constexpr (N0 == 2) {
        // once per workgroup (persistent launch)
        if constexpr (GT) {
            for (int i = threadIdx.x; i < kN02States * kN02Row; i += kDelBlock) tab2[i] = A.tab[kTabHdr + i];
        } else {
            for (int i = threadIdx.x; i < kN02States * 5; i += kDelBlock)
                n02_table_entry(i / 5, i % 5, A.pd, tab2 + (i / 5) * kN02Row);
        }
        tab = tab2;
    } else {
        tab = A.tab + kTabHdr;
    }
    const int lane = threadIdx.x & 63;
    const int j = threadIdx.x & (G - 1);
    const int g = threadIdx.x / G;
    const uint32_t jr = bitrev((uint32_t)j, GB);
    const long long ngrp = (A.B + CPB - 1) / CPB;
    // codeword groups: the static stride, or the next group of the launch's counter (one atomic a group
    // by thread 0, broadcast through LDS), so the workgroups finish together (round 6)
    __shared__ long long next_grp;
    long long grp = blockIdx.x;
    if (A.wtiles) {
        if (threadIdx.x == 0) next_grp = (long long)atomicAdd(A.wtiles, 1ull);
        __syncthreads();
        grp = next_grp;
    }
#pragma unroll 1
    while (grp < ngrp) {
        const long long cw = grp * CPB + g;
        const bool valid = cw < A.B;
        const long long c = valid ? cw : A.B - 1;  // padding codewords decode a duplicate, store nothing
        for (int i = threadIdx.x; i < CPB * WPC; i += kDelBlock) xs[i] = 0;
        if (dense_stage_bytes(A.stride, A.rx, CPB)) {  // received words: staged by 16-byte loads, packed from LDS
            uint8_t* stg = (uint8_t*)(rxb + dense_stage_off(A.rw, CPB));
            const int R = dense_stage_rows(A.stride, CPB);
            for (int r0 = 0; r0 < CPB; r0 += R) {
                const long long b0 = (grp * CPB + r0) * (long long)A.stride;
                const long long a0 = b0 & ~15ll;
                const int mis = (int)(b0 - a0);
                if (r0) __syncthreads();  // the previous chunk's rows are packed
                stage_bytes(A, a0, stg, R * A.stride + mis);
                __syncthreads();
                pack_staged<CPB>(A, grp, stg + mis, r0, R, rxb, lane);
            }
        } else {
            pack_rows<CPB>(A, grp, rxb, lane);  // received words bit-packed into LDS (sc_del_kern.h)
        }
        __syncthreads();

        // segments (removeDeletionGuardBands' descent): trellis tr = jr * 2^TL + i is reached by
        // the 4 halvings of jr (shared by the lane's trellises), then the TL of i
        const uint32_t* pw = rxb + g * A.rw;
        int len = A.rx_len[c];
        len = len < 0 ? 0 : (len > A.stride ? A.stride : len);
        int sa[LV], se[LV];
        dense_segments<TB, GB>(pw, len, jr, sa, se);
        // local value t (position j + G t) is trellis jr * 2^TL + bitrev(t): its state's row; the
        // walk's decision history (empty) beside it
        RowHist<N0, LV> rh;
#pragma unroll
        for (int i = 0; i < (LV + RowHist<N0, LV>::PER - 1) / RowHist<N0, LV>::PER; ++i) rh.w[i] = 0;
#pragma unroll
        for (int t = 0; t < LV; ++t) {
            const int i = cbitrev(t, TL);
            const int s = sa[i], m = se[i] - sa[i];
            const uint32_t y = m <= L ? packed_bits(pw, s, m, A.rw) : 0u;
            rh.set_row(t, (N0 == 2 ? n02_state(m, y) : n03_state(m, y)) * ROW);
        }

        // the walk: 2^n0 memoryless subtrees, input k of each trellis from its row and history
        uint32_t acc = 0;
        int nacc = 0, infow = 0;
#pragma unroll 1
        for (int k = 0; k < L; ++k) {
            uint64_t fm[NW], fv[NW], ub[NW];
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const int us = k * T + 64 * w;
                if constexpr (T >= 64) {
                    fm[w] = (uint64_t)A.fmask[us >> 5] | ((uint64_t)A.fmask[(us >> 5) + 1] << 32);
                    fv[w] = (uint64_t)A.fval[us >> 5] | ((uint64_t)A.fval[(us >> 5) + 1] << 32);
                } else {
                    fm[w] = (uint64_t)((A.fmask[us >> 5] >> (us & 31)) & (uint32_t)WM);
                    fv[w] = (uint64_t)((A.fval[us >> 5] >> (us & 31)) & (uint32_t)WM);
                }
                ub[w] = 0;
            }
            bool rate0 = true;
#pragma unroll
            for (int w = 0; w < NW; ++w) rate0 = rate0 && (fm[w] == WM);
            uint32_t bits;
            if (rate0) {  // decisions = the frozen values (wave-uniform)
                bits = WinTree<LV, G, NW>::frozen(ub, fv, j);
            } else {
                double v[LV];
#pragma unroll
                for (int t = 0; t < LV; ++t) v[t] = tab[rh.row(t) + dense_slot<N0>(k, rh.hist(t))];
                if constexpr (NW == 1 || G != 16) bits = WinTree<LV, G, NW, R1>::run(v, ub, fm, fv, lane);
                else bits = DelWin<LV, NW>::run(v, ub, fm, fv, lane);
            }
#pragma unroll
            for (int t = 0; t < LV; ++t) rh.add_bit(t, (bits >> t) & 1u, k);
            // information bits in u order (lane j = 0 holds the subtree's decisions)
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                for (uint64_t im = ~fm[w] & WM; im != 0ull; im &= im - 1ull) {
                    acc |= (uint32_t)((ub[w] >> __builtin_ctzll(im)) & 1ull) << nacc;
                    if (++nacc == 32) {
                        if (valid && j == 0 && A.info) A.info[(long long)infow * A.B + cw] = acc;
                        acc = 0;
                        nacc = 0;
                        ++infow;
                    }
                }
            }
        }
        if (nacc && valid && j == 0 && A.info) A.info[(long long)infow * A.B + cw] = acc;

        // x_hat: trellis tr's slice is natural positions [tr L, (tr + 1) L) (L <= 8: one word)
#pragma unroll
        for (int t = 0; t < LV; ++t) {
            const int pos = (int)((jr << TL) | (uint32_t)cbitrev(t, TL)) * L;
            atomicOr(&xs[g * WPC + (pos >> 5)], enc_hist<L>(rh.hist(t)) << (pos & 31));
        }
        __syncthreads();
        if (A.xhat && valid)
            for (int i = j; i < WPC; i += G) A.xhat[(long long)i * A.B + cw] = xs[g * WPC + i];
        __syncthreads();  // xs / rxb are reused by the workgroup's next group
        if (A.wtiles) {  // (every thread read next_grp before this group's first barrier)
            if (threadIdx.x == 0) next_grp = (long long)atomicAdd(A.wtiles, 1ull);
            __syncthreads();
            grp = next_grp;
        } else {
            grp += gridDim.x;
        }
    }
}

// sc_del_dense.hip; nullptr outside n0 2, 3 and tb 4 .. 8 (gt: n0 = 2 with a built table; g = 4: tb <= 6);
// r1 = false: the subtrees without the rate-1 shortcut (8 lanes a codeword only)
DelKern del_kernel_dense(int n0, int tb, bool gt = false, int g = kDenseG, bool r1 = true);

}  // namespace pcub
