// Host emulation of the HIP decode schedule (TEST ONLY).
// Compiles polarcub_amd/csrc/sc_bin_body.h -- the exact code the kernel runs --
// for the CPU, lane by lane, so schedule/indexing bugs show up in the CPU test
// suite.  Not part of the product library; nothing in polarcub_amd loads it.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "sc_bin_sched.h"

using namespace pcub;

extern "C" int emu_decode_bin(const double* xy, long long B, int n, const uint32_t* fmask, const uint32_t* fval,
                              uint32_t* info, uint32_t* xhat, uint32_t* uout, int S) {
    const int N = 1 << n;
    BinArgs A;
    A.xy = (const double2*)xy;
    A.B = B;
    A.n = n;
    A.fmask = fmask;
    A.fval = fval;
    A.info = info;
    A.xhat = xhat;
    A.uout = uout;
    A.ef = nullptr;
    A.cmask = nullptr;
    A.tile = 0;
    if (n <= 5) {
        for (long long b = 0; b < B; ++b) {
            switch (n) {
                case 0: decode_small<1>(A, b, true); break;
                case 1: decode_small<2>(A, b, true); break;
                case 2: decode_small<4>(A, b, true); break;
                case 3: decode_small<8>(A, b, true); break;
                case 4: decode_small<16>(A, b, true); break;
                case 5: decode_small<32>(A, b, true); break;
            }
        }
        return 0;
    }
    const long long nslots = 4;  // emulate a few slots, reused across codewords
    if (N < 2 * S) return -1;
    std::vector<double2> scr((size_t)(N / 2 - S) * nslots + 1);
    std::vector<uint32_t> yb((size_t)(N / 32) * nslots);
    const int D = n - (S == 8 ? 3 : S == 16 ? 4 : 5);
    std::vector<uint8_t> ef((size_t)1 << D);
    for (int k = 0; k < (1 << D); ++k) ef[k] = (uint8_t)first_frozen_depth(fmask, k, D, S);
    A.ef = ef.data();
    std::vector<uint32_t> cm((size_t)(N / 32) * 8);
    for (int i = 0; i < N / 32; ++i) compress_masks(fmask[i], cm.data() + 8 * i);
    A.cmask = cm.data();
    A.scratch = scr.data();
    A.ybits = yb.data();
    A.nslots = nslots;
    for (long long b = 0; b < B; ++b) {
        if (S == 8) decode_codeword<8, 1>(A, b, 0, 0, b % nslots, true);
        else if (S == 16) decode_codeword<16, 1>(A, b, 0, 0, b % nslots, true);
        else decode_codeword<32, 1>(A, b, 0, 0, b % nslots, true);
    }
    return 0;
}

// The compact-root schedule (CR: root rows as compact normalised doubles [N][B]).
extern "C" int emu_decode_bin_compact(const double* xc, long long B, int n, const uint32_t* fmask,
                                      const uint32_t* fval, uint32_t* info, uint32_t* xhat, int S, int hl) {
    const int N = 1 << n;
    const int SR = S;
    if (n <= 5 || N < 2 * SR) return -1;
    BinArgs A;
    A.xy = nullptr;
    A.xc = xc;
    A.B = B;
    A.n = n;
    A.fmask = fmask;
    A.fval = fval;
    A.info = info;
    A.xhat = xhat;
    A.uout = nullptr;
    A.tile = 0;
    const long long nslots = 4;
    std::vector<double2> scr((size_t)(N / 2 - SR) * nslots + 1);
    std::vector<uint32_t> yb((size_t)(N / 32 + 2) * nslots);
    int s = 0;
    while ((1 << s) < SR) ++s;
    const int D = n - s;
    std::vector<uint8_t> ef((size_t)1 << D);
    for (int k = 0; k < (1 << D); ++k) ef[k] = (uint8_t)first_frozen_depth(fmask, k, D, SR);
    A.ef = ef.data();
    std::vector<uint32_t> cm((size_t)(N / 32) * 8);
    for (int i = 0; i < N / 32; ++i) compress_masks(fmask[i], cm.data() + 8 * i);
    A.cmask = cm.data();
    A.scratch = scr.data();
    A.ybits = yb.data();
    A.nslots = nslots;
    (void)hl;  // the split level needs S*G >= 64 (not emulable at one lane per codeword)
    for (long long b = 0; b < B; ++b) {
        if (S == 8) decode_codeword<8, 1, false, 1, false, false, 0, true>(A, b, 0, 0, b % nslots, true);
        else if (S == 16) decode_codeword<16, 1, false, 1, false, false, 0, true>(A, b, 0, 0, b % nslots, true);
        else decode_codeword<32, 1, false, 1, false, false, 0, true>(A, b, 0, 0, b % nslots, true);
    }
    return 0;
}

// helper self-checks: polar_bits against the half-split recursion, gather_stride against a bit loop
static uint64_t enc_rec(uint64_t u, int L) {
    if (L == 1) return u & 1u;
    const uint64_t m = (L / 2 == 64) ? ~0ull : ((1ull << (L / 2)) - 1ull);
    const uint64_t ym = enc_rec(u & m, L / 2), yp = enc_rec(u >> (L / 2), L / 2);
    return (ym ^ yp) | (yp << (L / 2));
}
template <int G>
static int check_gather(uint64_t x) {
    for (int j = 0; j < G; ++j) {
        uint64_t r = 0;
        for (int t = 0; j + G * t < 64; ++t) r |= ((x >> (j + G * t)) & 1ull) << t;
        if (gather_stride<G>(x >> j) != r) return 1;
    }
    return 0;
}
extern "C" int emu_check_bits(uint64_t seed) {
    int bad = 0;
    uint64_t x = seed;
    for (int it = 0; it < 2000; ++it) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        if (polar_bits(x) != enc_rec(x, 64)) ++bad;
        bad += check_gather<1>(x) + check_gather<2>(x) + check_gather<4>(x) + check_gather<8>(x);
    }
    return bad;
}
