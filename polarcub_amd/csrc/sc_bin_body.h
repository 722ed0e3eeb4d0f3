// sc_bin_body.h -- one-codeword SC decode schedule (binary, uniform prior).
//
// Replaces BinaryPolarEncoderDecoder.recursiveEncodeDecode (decode branch,
// BinaryPolarEncoderDecoder.py:223-325).  G lanes decode one codeword (G = 1, 2,
// 4, 8); all lanes of a wave run the identical (data-independent) tree schedule.
//
// Storage ("half-split" = bit-reversed order inside every node).  A node of
// length L keeps its values at positions p = 0..L-1 such that its minus/plus
// children are  out[p] = op(in[p], in[p + L/2]).  The reference pairs rows
// (2h, 2h+1); position p holds row bitrev_L(p), which makes both statements
// the same computation.  The node's re-encoded vector in the same order is
//     y = [ y_minus ^ y_plus | y_plus ]
// (BinaryPolarEncoderDecoder.py:319-323 permuted), so partial sums are combined
// IN PLACE by a word-wise XOR of the left half with the right half.
//
// Lanes of a codeword.  Lane j of the G lanes owns the positions p = j (mod G)
// of every node with L >= G (local index t = p / G).  Because p and p + L/2
// have the same residue, every butterfly with L >= 2G is lane-local, and each
// lane runs exactly the G = 1 schedule on a "virtual" tree of length N/G.  A
// virtual leaf is a real node of length G holding one value per lane; it is
// finished by XSub<G> with cross-lane exchanges (lane ^ G/2, ^ G/4, .., ^ 1).
// The re-encoded bits also stay lane-local, and x_hat's natural-order segment
// k (N/G bits) is exactly lane bitrev_g(k)'s local bits, bit-reversed.
//
// Levels (per lane, virtual): depth d holds N_v >> d values.  Depth 0 is the
// input (never normalised, never copied).  Depths 1 .. D-1 live in a per-slot
// scratch buffer (compact f64, two values per 16-byte access, slot-minor so a
// wave's access is one contiguous 1 KiB).  Depth D = log2(N_v / S) goes straight
// to registers and the S-value subtree below it is fully unrolled (SubV).
#pragma once
#include "sc_common.h"

namespace pcub {

struct BinArgs {
    const double2* xy;         // [N][B] raw pairs
    const double* xc;          // [N][B] compact normalised rows (the CR kernels' root instead of xy)
    long long B;
    int n;                     // log2 N
    const uint32_t* fmask;     // ceil(N/32)
    const uint32_t* fval;      // ceil(N/32)
    uint32_t* info;            // [ceil(K/32)][B]
    uint32_t* xhat;            // [ceil(N/32)][B] or null
    uint32_t* uout;            // [ceil(N/32)][B] or null
    double2* scratch;          // [(N_v/2 - S) pairs][nslots]
    uint32_t* ybits;           // [N_v/32][nslots]
    long long nslots;
    const uint8_t* ef;         // [2^D] first rate-0 depth of each subtree's chain (first_frozen_depth)
    int tile;                  // root layout: 0 = [N][B] rows; T > 0 = [ceil(B/T)][N][T] (T codewords a tile)
    const uint32_t* cmask;     // [N/32][8] per frozen-mask word: compress masks mv0..mv4, info count, info mask
    // k_sc_bin's wave tiles (64 / G codewords each) handed out by a counter (zeroed before the launch)
    // instead of a static stride, so the waves finish together (round 6); null: the static stride
    unsigned long long* wtiles = nullptr;
};

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// The next work tile of a launch's counter (the decode kernels' dynamic tiles, round 6): one vector
// atomic from lane 0, its value made wave-uniform
__device__ __forceinline__ long long next_wave_tile(unsigned long long* c, int lane) {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(c, 1ull);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, 0), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), 0);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

#endif

// Information-bit compress masks of one 32-bit frozen-mask word (Hacker's Delight 7-4, "compress"):
// with m = ~fm the information positions, x -> the bits of x at m packed to the right is
//     x &= m;  for i in 0..4: t = x & mv_i;  x = (x ^ t) | (t >> 2^i)
// and mv_i depends on m alone, so the decode kernel gets them from a table built once per launch.
// out[0..4] = mv_i, out[5] = popcount(m), out[6] = m, out[7] = 0.
PCUB_HD void compress_masks(uint32_t fm, uint32_t* out) {
    uint32_t m = ~fm;
    out[5] = (uint32_t)__builtin_popcount(m);
    out[6] = m;
    out[7] = 0u;
    uint32_t mk = ~m << 1;
    for (int i = 0; i < 5; ++i) {
        uint32_t mp = mk ^ (mk << 1);
        mp ^= mp << 2;
        mp ^= mp << 4;
        mp ^= mp << 8;
        mp ^= mp << 16;
        const uint32_t mv = mp & m;
        out[i] = mv;
        m = (m ^ mv) | (mv >> (1 << i));
        mk &= ~mp;
    }
}

// the bits of x at the information positions of word `cm` (compress_masks), packed to the right
PCUB_HD uint32_t compress_info(uint32_t x, const uint32_t* cm) {
    x &= cm[6];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t t = x & cm[i];
        x = (x ^ t) | (t >> (1 << i));
    }
    return x;
}

// Offset (in rows' elements) of codeword cw's root row 0, and the stride between root rows.
PCUB_HD long long root_base(const BinArgs& A, long long cw) {
    if (A.tile <= 0) return cw;
    return (cw / A.tile) * ((long long)A.tile << A.n) + cw % A.tile;
}
PCUB_HD long long root_stride(const BinArgs& A) { return A.tile > 0 ? (long long)A.tile : A.B; }

// Rate-0 table.  Register subtree k (real u range [k*SU, (k+1)*SU)) is reached
// by a chain that starts at depth d0(k) = 1 (k = 0) or D - ctz(k).  Returns the
// smallest depth e in [d0, D] whose node on that chain has every u frozen, or
// D + 1.  Such a node is never evaluated: nothing outside it reads it, and the
// reference's decisions inside it are the frozen values.
PCUB_HD bool range_frozen(const uint32_t* fmask, long long a, long long len) {
    if (len < 32) {
        const uint32_t m = ((1u << len) - 1u) << (a & 31);
        return (fmask[a >> 5] & m) == m;
    }
    for (long long w = a >> 5; w < (a + len) >> 5; ++w)
        if (fmask[w] != 0xffffffffu) return false;
    return true;
}

PCUB_HD int first_frozen_depth(const uint32_t* fmask, int k, int D, int SU) {
    const int d0 = (k == 0) ? 1 : D - __builtin_ctz((unsigned)k);
    for (int e = d0; e <= D; ++e) {
        const long long sub = 1LL << (D - e);  // register subtrees under a depth-e node
        const long long first = ((long long)k >> (D - e)) << (D - e);
        if (range_frozen(fmask, first * SU, sub * SU)) return e;
    }
    return D + 1;
}

#if defined(__HIP_DEVICE_COMPILE__)
// Exchange with lane ^ MASK.  Inside a row of 16 lanes this is DPP (VALU moves, no
// LDS round trip: the cross-lane leaf chains are serial, so the ds_bpermute latency
// is on the critical path): MASK 1, 2 a quad_perm; MASK 8 the row rotation by 8;
// MASK 4 the rotation by 12 (row_ror:k gives lane i the value of lane i - k mod 16),
// then banks 1 and 3 of the row (lanes 4-7, 12-15) overwritten by the rotation by 4
// (checked on the GPU by tests/emu/dpp_check.hip).  Wider masks use __shfl_xor.  Every caller
// exchanges inside an aligned group of >= 2*MASK lanes that share their control
// flow, so the source lane is always active.
template <int CTRL, int BANKS = 0xF>
PCUB_HD unsigned dpp32(unsigned old, unsigned src) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, 0xF, BANKS, false);
}

template <int MASK>
PCUB_HD unsigned xor_lane32(unsigned x) {
    // every lane is written (all rows and banks, no bound_ctrl): no old value to materialise
    if constexpr (MASK == 1) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    else if constexpr (MASK == 2) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    else if constexpr (MASK == 8) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);
    else return dpp32<0x124, 0xA>(dpp32<0x12C>(0u, x), x);      // row_ror:12, banks 1,3: row_ror:4
}

template <int MASK>
PCUB_HD double xor_shfl_c(double v) {
    if constexpr (MASK == 1 || MASK == 2 || MASK == 4 || MASK == 8) {
        const unsigned long long b = (unsigned long long)as_bits(v);
        const unsigned lo = xor_lane32<MASK>((unsigned)b);
        const unsigned hi = xor_lane32<MASK>((unsigned)(b >> 32));
        return from_bits((long long)(((unsigned long long)hi << 32) | lo));
    } else {
        return __shfl_xor(v, MASK);
    }
}
#else
template <int MASK>
PCUB_HD double xor_shfl_c(double v) { return v; }  // host emulation runs G = 1 only
#endif

// A real node of length M (M <= G) with position (lane & (M-1)) held by each lane.
// Returns this lane's bit of the node's (half-split) encoding; ORs the M
// decisions u_UBASE .. u_UBASE+M-1 (identical in all lanes) into ub.
template <int M, int UBASE>
struct XSub {
    static PCUB_HD uint32_t run(double v, uint64_t& ub, uint64_t fm, uint64_t fv, int lane) {
        const double w = xor_shfl_c<M / 2>(v);
        const bool lo = (lane & (M / 2)) == 0;
        if constexpr (M == 2) {
            // both leaves of the pair from one product, u1's decision for either u0 (no branch:
            // leaf_g's if/else compiled to an exec-masked region; 75.0 -> 78.1 M cw/s at C2)
            uint32_t d0, d10, d11;
            leaf_pair_x(v, w, lo, d0, d10, d11);
            const uint32_t u0 = ((fm >> UBASE) & 1u) ? (uint32_t)((fv >> UBASE) & 1u) : d0;
            const uint32_t u1 = ((fm >> (UBASE + 1)) & 1u) ? (uint32_t)((fv >> (UBASE + 1)) & 1u) : (u0 ? d11 : d10);
            ub |= ((uint64_t)u0 << UBASE) | ((uint64_t)u1 << (UBASE + 1));
            return lo ? (u0 ^ u1) : u1;
        } else {
            // a frozen child (wave-uniform test) is not evaluated: its decisions are
            // the frozen values and its encoding their polar transform
            constexpr int H = M / 2;
            constexpr uint64_t HM = (1ull << H) - 1ull;
            const int pos = lane & (H - 1);
            uint32_t ym, yp;
            if (all_frozen<H>(fm, UBASE)) {
                ym = frozen_local<1, H>(fv >> UBASE, pos) & 1u;
                ub |= fv & (HM << UBASE);
            } else {
                ym = XSub<H, UBASE>::run(op_f(v, w), ub, fm, fv, lane);
            }
            if (all_frozen<H>(fm, UBASE + H)) {
                yp = frozen_local<1, H>(fv >> (UBASE + H), pos) & 1u;
                ub |= fv & (HM << (UBASE + H));
            } else {
                yp = XSub<H, UBASE + H>::run(op_g_x(v, w, lo, ym), ub, fm, fv, lane);
            }
            return lo ? (ym ^ yp) : yp;
        }
    }
};

// Rate-1 nodes (round 5).  In a node with no frozen position, SC's decisions are the hard decisions
// of its inputs whenever every minus transform inside it keeps the orientation its inputs give it:
// with t = (1 - r) / (1 + r) per value, a minus output has t = t_a t_b (exactly, before rounding) and
// a plus output under the hard decision of its left sibling t >= max(t_a, t_b), so every value in the
// node has t >= prod t_i over the node's inputs.  When that product is >= 2^-17 every canonical
// minus transform compares p0 = 1 + ra rb against p1 = ra + rb with p0 - p1 = (1 - ra)(1 - rb) >=
// 2^-17, far above the 2^-51 its roundings can move, so p1 > p0 never holds, every output ratio is
// < 1 and carries the XOR of its inputs' orientations, every plus transform takes the same-orientation
// branch, and every leaf decides its value's orientation: the node's re-encoding is the inputs' signs
// and its decisions are their polar transform (an involution) -- the values the recursion would compute
// bit for bit.  A NaN ((0, 0)) or a tie (r = 1) makes the product NaN or 0 and fails the test.  The
// test runs per codeword (its G lanes) and the wave takes the shortcut only when all its codewords
// pass (a uniform branch); otherwise the recursion runs as before.
template <int G>
PCUB_HD uint64_t spread_stride(uint64_t x) {  // bit t -> bit t * G (the inverse of gather_stride)
    if constexpr (G == 1) {
        return x;
    } else if constexpr (G == 2) {
        x &= 0xFFFFFFFFull;
        x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
        x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
        x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
        x = (x | (x << 2)) & 0x3333333333333333ull;
        return (x | (x << 1)) & 0x5555555555555555ull;
    } else if constexpr (G == 4) {
        x &= 0xFFFFull;
        x = (x | (x << 24)) & 0x000000FF000000FFull;
        x = (x | (x << 12)) & 0x000F000F000F000Full;
        x = (x | (x << 6)) & 0x0303030303030303ull;
        return (x | (x << 3)) & 0x1111111111111111ull;
    } else if constexpr (G == 8) {
        x &= 0xFFull;
        x = (x | (x << 28)) & 0x0000000F0000000Full;
        x = (x | (x << 14)) & 0x0003000300030003ull;
        return (x | (x << 7)) & 0x0101010101010101ull;
    } else if constexpr (G == 16) {
        x &= 0xFull;
        x = (x | (x << 30)) & 0x0000000300000003ull;
        return (x | (x << 15)) & 0x0001000100010001ull;
    } else if constexpr (G == 32) {
        return ((x & 1ull) | ((x & 2ull) << 31));
    } else {
        static_assert(G == 64, "lanes per codeword");
        return x & 1ull;
    }
}

// x OR-ed over the aligned group of G lanes
template <int G, int M = 1>
PCUB_HD uint64_t or_group(uint64_t x) {
    if constexpr (M >= G) {
        return x;
    } else {
        return or_group<G, 2 * M>(x | (uint64_t)as_bits(xor_shfl_c<M>(from_bits((long long)x))));
    }
}

template <int G, int M = 1>
PCUB_HD double mul_group(double x) {
    if constexpr (M >= G) {
        return x;
    } else {
        return mul_group<G, 2 * M>(x * xor_shfl_c<M>(x));
    }
}

// every codeword of the wave passes the rate-1 test on its L values per lane (a wave-uniform answer)
template <int L, int G>
PCUB_HD bool rate1_sure(const double* v) {
    double p1 = 1.0, p2 = 1.0;  // prod (1 - r), prod (1 + r) over the codeword's values
#pragma unroll
    for (int t = 0; t < L; ++t) {
        const double r = __builtin_fabs(v[t]);
        p1 *= __builtin_fmax(1.0 - r, 0.0);  // r > 1 (only from negative root rows) or NaN: 0, fails
        p2 *= 1.0 + r;
    }
    p1 = mul_group<G>(p1);
    p2 = mul_group<G>(p2);
    const bool ok = p1 >= 0x1p-17 * p2;  // false on NaN
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(!ok) == 0ull;
#else
    return ok;
#endif
}

// the rate-1 node of L values per lane at virtual leaf BASE_V: local encoding bits = the values'
// orientations; decisions u_{BASE_V*G ..} = the polar transform of the node's natural-order encoding
// (position t*G + j is lane j's local bit t)
template <int L, int BASE_V, int G>
PCUB_HD uint32_t rate1_node(const double* v, uint64_t& ub, int lane) {
    static_assert(L * G <= 64, "one window");
    uint32_t h = 0;
#pragma unroll
    for (int t = 0; t < L; ++t) h |= (hi32(v[t]) >> 31) << t;
    const uint64_t x = or_group<G>(spread_stride<G>(h) << (lane & (G - 1)));
    ub |= polar_bits(x) << (BASE_V * G);
    return h;
}

// Register-resident virtual subtree of L values per lane; virtual leaf BASE_V
// covers real u positions [BASE_V*G, BASE_V*G + G).  Returns L local encoding bits.
// R1: try the rate-1 shortcut (the deletion kernels choose: their rows hold ties and (0, 0) pairs;
// the 16-lane layout never qualifies, G <= 8, and the 8-lane one measured it)
template <int L, int BASE_V, int G, bool R1 = true>
struct SubV {
    static PCUB_HD uint32_t run(const double* v, uint64_t& ub, uint64_t fm, uint64_t fv, int lane) {
        if constexpr (R1 && L >= 2 && L * G >= 16 && G <= 8) {
            // a rate-1 node (no frozen position; wave-uniform) whose codewords all pass the test
            constexpr uint64_t NM = (L * G == 64) ? ~0ull : ((1ull << (L * G)) - 1ull);
            if (((fm >> (BASE_V * G)) & NM) == 0ull && rate1_sure<L, G>(v)) return rate1_node<L, BASE_V, G>(v, ub, lane);
        }
        if constexpr (L == 1) {
            static_assert(G >= 2, "G == 1 stops at L == 2");
            return XSub<G, BASE_V * G>::run(v[0], ub, fm, fv, lane);
        } else if constexpr (L == 2 && G == 1) {
            uint32_t d0, d10, d11;
            leaf_pair(v[0], v[1], d0, d10, d11);
            const uint32_t u0 = ((fm >> BASE_V) & 1u) ? (uint32_t)((fv >> BASE_V) & 1u) : d0;
            const uint32_t u1 = ((fm >> (BASE_V + 1)) & 1u) ? (uint32_t)((fv >> (BASE_V + 1)) & 1u) : (u0 ? d11 : d10);
            ub |= ((uint64_t)u0 << BASE_V) | ((uint64_t)u1 << (BASE_V + 1));
            return (u0 ^ u1) | (u1 << 1);
        } else {
            // Rate-0 children (all u frozen; the test is wave-uniform) are skipped:
            // the reference's decisions there are the frozen values whatever the
            // probabilities, so only their re-encoding is needed.
            constexpr int H = L / 2;
            constexpr int HR = H * G;  // real leaves per child
            constexpr uint64_t HM = (HR == 64) ? ~0ull : ((1ull << HR) - 1ull);
            constexpr uint32_t LMASK = (H == 32) ? 0xffffffffu : ((1u << H) - 1u);
            const int j = lane & (G - 1);
            double c[H];
            uint32_t ym, yp;
            if (all_frozen<HR>(fm, BASE_V * G)) {
                ym = frozen_local<H, G>(fv >> (BASE_V * G), j) & LMASK;
                ub |= fv & (HM << (BASE_V * G));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_f(v[t], v[t + H]);
                ym = SubV<H, BASE_V, G, R1>::run(c, ub, fm, fv, lane);
            }
            if (all_frozen<HR>(fm, (BASE_V + H) * G)) {
                yp = frozen_local<H, G>(fv >> ((BASE_V + H) * G), j) & LMASK;
                ub |= fv & (HM << ((BASE_V + H) * G));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_g(v[t], v[t + H], (ym >> t) & 1u);
                yp = SubV<H, BASE_V + H, G, R1>::run(c, ub, fm, fv, lane);
            }
            return (ym ^ yp) | (yp << H);
        }
    }
};

// One stored level of compact values: pair q (positions 2q, 2q+1) at p[q * s].
struct Lvl {
    double2* p;
    long long s;
};

// Source of a fused chain pass: the raw root (depth 0) or a stored level, plus
// the partial sums of the first op's minus child when that op is a plus transform.
struct Chain {
    const double2* in;  // root: the wave's tile (uniform); this lane's rows at byte offset lin
    const double* inc;  // compact root (R == 3): the same rows, one double each
    uint32_t lin;       // this lane's byte offset from in / inc (pairs: 16 B a row element, compact: 8)
    long long B;
    int nv;             // log2 of the virtual (per-lane) length
    Lvl src;            // compact source level (depth a > 0)
    const uint32_t* Y;  // local re-encoded bits, word w at Y[w * ns]
    long long ns;
    int ystart;         // first local u position of the minus child at depth a+1
};

// Global-memory access helpers.  The per-k pointer laundering (see launder())
// hides the pointers' provenance, so without an explicit address-space cast the
// compiler emits flat instructions (which also tie up the LDS counter).  GL =
// false keeps a generic access (for a level that may live in LDS).  NT = non-
// temporal: the input rows are streamed exactly twice, far apart in time.
#if defined(__HIP_DEVICE_COMPILE__)
typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) d2v gd2v;
typedef __attribute__((address_space(1))) uint32_t gu32;
#endif

#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(1))) double gd1;
#endif

// one double of the compact root (non-temporal: streamed twice, far apart)
PCUB_HD double ld1nt(const double* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_nontemporal_load((const gd1*)p);
#else
    return *p;
#endif
}

template <bool NT = false, bool GL = true>
PCUB_HD double2 ld2(const double2* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (GL) {
        const gd2v* g = (const gd2v*)p;
        const d2v v = NT ? __builtin_nontemporal_load(g) : *g;
        return double2{v.x, v.y};
    }
#endif
    return *p;
}

template <bool NT = false, bool GL = true>
PCUB_HD void st2(double2* p, double2 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (GL) {
        gd2v* g = (gd2v*)p;
        d2v t;
        t.x = v.x;
        t.y = v.y;
        if constexpr (NT) __builtin_nontemporal_store(t, g);
        else *g = t;
        return;
    }
#endif
    *p = v;
}

PCUB_HD uint32_t ldu(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const gu32*)p;
#else
    return *p;
#endif
}

PCUB_HD void stu(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    *(gu32*)p = v;
#else
    *p = v;
#endif
}

// Re-encoded bits (Y): a per-slot global buffer, or (YL) this thread's column of an LDS
// array (word w at Y[w * kBinBlock]): the plus passes read them and every combine rewrites
// them, so in LDS they never travel to L2/HBM.
template <bool YL>
PCUB_HD uint32_t ldy(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (YL) return *(const __attribute__((address_space(3))) uint32_t*)p;
#endif
    return ldu(p);
}

template <bool YL>
PCUB_HD void sty(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (YL) {
        *(__attribute__((address_space(3))) uint32_t*)p = v;
        return;
    }
#endif
    stu(p, v);
}

// Split register level (HL variants): the first half of the chain's last level lives in
// this thread's LDS column (value t at hl[t * kHlStride]), the second half in registers.
constexpr int kHlStride = 256;  // = kBinBlock: one column per thread of the workgroup

PCUB_HD void stl(double* p, double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    *(__attribute__((address_space(3))) double*)p = v;
#else
    *p = v;
#endif
}

PCUB_HD double ldl(const double* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(3))) double*)p;
#else
    return *p;
#endif
}

// Root rows.  Local position t of lane j is real position p = j + G*t < N/2,
// which pairs natural rows (2q, 2q+1) with q = bitrev_{n-1}(p).  The bits of j
// and of G*t are disjoint, so q = bitrev_{n-1}(j) + bitrev_{nv-1}(t): the lane
// part is folded into the lane's root pointer (Chain::in) once, and the row
// offset of a position is wave-uniform.
PCUB_HD long long root_row(int t, int nv) { return (long long)bitrev((uint32_t)t, nv - 1); }

// Makes a per-lane pointer opaque to the optimiser at this point, so addresses
// derived from it are recomputed in the loop (one or two VALU ops) instead of
// being hoisted out of it and held live in registers across the whole schedule.
template <class T>
PCUB_HD T* launder(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(p));
#endif
    return p;
}

// a wave-uniform pointer kept in SGPRs (the same laundering for a base every lane shares)
template <class T>
PCUB_HD T* launder_s(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(p));
#endif
    return p;
}

// a 64-bit value every lane of the wave holds, moved to SGPRs
PCUB_HD long long uniform64(long long v) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
#else
    return v;
#endif
}

// wave-uniform base + 32-bit lane byte offset: global loads with an SGPR base and a VGPR offset
// (no 64-bit address arithmetic in the VALU)
template <bool NT = false>
PCUB_HD double2 ld2o(const double2* base, uint32_t lo) {
    return ld2<NT>((const double2*)((const char*)base + lo));
}
PCUB_HD double ld1nto(const double* base, uint32_t lo) { return ld1nt((const double*)((const char*)base + lo)); }

// Keeps the scheduler from hoisting the next column's loads above this point
// (bounds the live registers of the unrolled final pass).
PCUB_HD void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}

// A register subtree's u decisions and frozen bits live in NW 64-bit windows
// (NW = S*G/64 when the subtree has more than 64 real positions): WinTree splits
// the subtree at its top nodes until each part is one window.
template <int L, int G, int NWIN, bool R1 = true>
struct WinTree {
    static PCUB_HD uint32_t run(const double* v, uint64_t* ub, const uint64_t* fm, const uint64_t* fv, int lane) {
        if constexpr (NWIN == 1) {
            return SubV<L, 0, G, R1>::run(v, ub[0], fm[0], fv[0], lane);
        } else {
            constexpr int H = L / 2;
            constexpr int HW = NWIN / 2;
            double c[H];
            uint32_t ym, yp;
            if (frozen_windows(fm)) {
                ym = WinTree<H, G, HW>::frozen(ub, fv, lane & (G - 1));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_f(v[t], v[t + H]);
                ym = WinTree<H, G, HW, R1>::run(c, ub, fm, fv, lane);
            }
            if (frozen_windows(fm + HW)) {
                yp = WinTree<H, G, HW>::frozen(ub + HW, fv + HW, lane & (G - 1));
            } else {
#pragma unroll
                for (int t = 0; t < H; ++t) c[t] = op_g(v[t], v[t + H], (ym >> t) & 1u);
                yp = WinTree<H, G, HW, R1>::run(c, ub + HW, fm + HW, fv + HW, lane);
            }
            return (ym ^ yp) | (yp << H);
        }
    }

    // NWIN/2 full windows all frozen (the half is rate-0)
    static PCUB_HD bool frozen_windows(const uint64_t* fm) {
        bool all = true;
#pragma unroll
        for (int w = 0; w < NWIN / 2; ++w) all = all && (fm[w] == ~0ull);
        return all;
    }

    // a rate-0 subtree: decisions = frozen values, encoding = their polar transform
    static PCUB_HD uint32_t frozen(uint64_t* ub, const uint64_t* fv, int j) {
        if constexpr (NWIN == 1) {
            constexpr uint64_t WM = (L * G == 64) ? ~0ull : ((1ull << (L * G)) - 1ull);
            ub[0] = fv[0] & WM;
            return frozen_local<L, G>(fv[0], j);
        } else {
            constexpr int H = L / 2;
            const uint32_t ym = WinTree<H, G, NWIN / 2>::frozen(ub, fv, j);
            const uint32_t yp = WinTree<H, G, NWIN / 2>::frozen(ub + NWIN / 2, fv + NWIN / 2, j);
            return (ym ^ yp) | (yp << H);
        }
    }
};

// Small codes (N <= 32): everything in registers, one lane per codeword.
template <int NN>
PCUB_HD void decode_small(const BinArgs& A, long long cw, bool store) {
    constexpr int n = (NN <= 1) ? 0 : (NN <= 2) ? 1 : (NN <= 4) ? 2 : (NN <= 8) ? 3 : (NN <= 16) ? 4 : 5;
    const long long B = root_stride(A);  // root row stride ([N][B] rows or a tile's width)
    const double2* in = A.xy + root_base(A, cw);
    const uint64_t fm = A.fmask[0], fv = A.fval[0];
    uint64_t ub = 0;
    uint32_t y;
    if constexpr (NN == 1) {
        // leaf on the raw root: calcMarginalizedProbabilities (:52-69) on an
        // un-normalised pair, decided exactly as the reference does.
        const double2 a = in[0];
        double s = 0.0;
        s += a.x;
        s += a.y;
        uint32_t d = 0;
        if (s > 0.0) d = (a.x / s >= a.y / s) ? 0u : 1u;
        ub = (fm & 1u) ? (fv & 1u) : d;
        y = (uint32_t)ub;
    } else {
        double c[NN / 2];
#pragma unroll
        for (int t = 0; t < NN / 2; ++t) {
            const int p = (int)bitrev((uint32_t)t, n - 1);
            c[t] = op_f_raw(in[(long long)(2 * p) * B], in[(long long)(2 * p + 1) * B]);
        }
        uint32_t ym, yp;
        if constexpr (NN == 2) {
            ym = ((fm & 1u) ? (uint32_t)(fv & 1u) : leaf_v(c[0]));
            ub |= ym;
        } else {
            ym = SubV<NN / 2, 0, 1>::run(c, ub, fm, fv, 0);
        }
#pragma unroll
        for (int t = 0; t < NN / 2; ++t) {
            const int p = (int)bitrev((uint32_t)t, n - 1);
            c[t] = op_g_raw(in[(long long)(2 * p) * B], in[(long long)(2 * p + 1) * B], (ym >> t) & 1u);
        }
        if constexpr (NN == 2) {
            yp = ((fm & 2u) ? (uint32_t)((fv >> 1) & 1u) : leaf_v(c[0]));
            ub |= (uint64_t)yp << 1;
        } else {
            yp = SubV<NN / 2, NN / 2, 1>::run(c, ub, fm, fv, 0);
        }
        y = (ym ^ yp) | (yp << (NN / 2));
    }
    if (!store) return;
    uint32_t acc = 0;
    int nacc = 0;
    const uint32_t valid = (NN == 32) ? 0xffffffffu : ((1u << NN) - 1u);
    for (uint32_t im = ~(uint32_t)fm & valid; im != 0u; im &= im - 1u) {
        acc |= (uint32_t)((ub >> __builtin_ctz(im)) & 1u) << nacc;
        ++nacc;
    }
    if (nacc) A.info[cw] = acc;
    if (A.uout) A.uout[cw] = (uint32_t)ub;
    if (A.xhat) {
        uint32_t x = 0;  // x_hat[i] = y[bitrev_n(i)]
#pragma unroll
        for (int i = 0; i < NN; ++i) x |= ((y >> bitrev((uint32_t)i, n)) & 1u) << i;
        A.xhat[cw] = x;
    }
}

}  // namespace pcub
