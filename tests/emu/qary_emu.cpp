// Host emulation of the q-ary decode schedule (TEST ONLY): compiles
// polarcub_amd/csrc/sc_qary_body.h -- the code the kernel runs -- for the CPU.
#include <stdint.h>

#include <vector>

#include "sc_qary_body.h"

using namespace pcub;

template <int Q, int S>
static void run_s(const QArgs& A, long long B) {
    for (long long b = 0; b < B; ++b) decode_qary_cw<Q, S>(A, b, b % A.nslots, true);
}

// the split-level schedule (HL): the LDS column is a host array with the kernel's stride
template <int Q, int S>
static void run_h(const QArgs& A, long long B) {
    std::vector<double> hl((size_t)S * Q * kQHlStride);
    for (long long b = 0; b < B; ++b)
        decode_qary_cw<Q, S, 1, 1, false, true>(A, b, b % A.nslots, true, 0, 0, nullptr, 0, hl.data());
}

template <int Q>
static int run(const double* xy, long long B, int n, const uint8_t* frozen, uint8_t* info, uint8_t* xhat, int S0) {
    const bool hl = S0 < 0;  // negative: the split-level schedule with |S0| register positions
    const int S = hl ? -S0 : S0;
    const int SR = hl ? 2 * S : S;
    const int N = 1 << n;
    const long long ns = 3;  // a few slots, reused across codewords
    std::vector<uint32_t> words((N + 31) / 32, 0u);
    for (int i = 0; i < N; ++i) words[i >> 5] |= (uint32_t)(frozen[i] != 0) << (i & 31);
    int s = 0;
    while ((1 << s) < SR) ++s;
    const int D = n - s;
    std::vector<uint8_t> ef((size_t)1 << D);
    for (int k = 0; k < (1 << D); ++k) ef[k] = (uint8_t)first_frozen_depth(words.data(), k, D, SR);
    std::vector<double2> scr((size_t)(N - 2 * SR) * ((Q + 1) / 2) * ns + 1);
    std::vector<uint32_t> ys((size_t)(N + 3) / 4 * ns);  // bytes' worth: enough for every QPack
    QArgs A;
    A.xy = xy;
    A.B = B;
    A.n = n;
    A.fwords = words.data();
    A.ef = ef.data();
    A.info = info;
    A.xhat = xhat;
    A.scratch = scr.data();
    A.ysym = ys.data();
    A.nslots = ns;
    A.ylds_words = 0;
    A.tile = 0;
    if (hl) {
        switch (S) {
            case 1: run_h<Q, 1>(A, B); break;
            case 2: run_h<Q, 2>(A, B); break;
            case 4: run_h<Q, 4>(A, B); break;
            default: run_h<Q, 8>(A, B); break;
        }
        return 0;
    }
    switch (S) {
        case 1: run_s<Q, 1>(A, B); break;
        case 2: run_s<Q, 2>(A, B); break;
        case 4: run_s<Q, 4>(A, B); break;
        case 8: run_s<Q, 8>(A, B); break;
        default: run_s<Q, 16>(A, B); break;
    }
    return 0;
}

// xy: [N][B][q] native layout; info [K][B], xhat [N][B]
extern "C" int emu_decode_qary(const double* xy, long long B, int n, int q, const uint8_t* frozen, uint8_t* info,
                               uint8_t* xhat, int S) {
    if ((1 << n) < (S < 0 ? -4 * S : 2 * S)) return -1;
    switch (q) {
        case 2: return run<2>(xy, B, n, frozen, info, xhat, S);
        case 3: return run<3>(xy, B, n, frozen, info, xhat, S);
        case 4: return run<4>(xy, B, n, frozen, info, xhat, S);
        case 5: return run<5>(xy, B, n, frozen, info, xhat, S);
        case 8: return run<8>(xy, B, n, frozen, info, xhat, S);
        default: return -1;
    }
}

// q_div (shared reciprocal + Markstein correction, guarded) against plain IEEE
// division: `count` quadruples (p0..p3, t) from the caller, returns the mismatches.
extern "C" long long emu_qdiv_check(const double* p, const double* t, long long count) {
    long long bad = 0;
    for (long long i = 0; i < count; ++i) {
        QV<4> v;
        for (int x = 0; x < 4; ++x) v.p[x] = p[4 * i + x];
        q_div<4>(v, t[i]);
        for (int x = 0; x < 4; ++x) {
            const double want = p[4 * i + x] / t[i];
            if (__builtin_memcmp(&want, &v.p[x], sizeof(double)) != 0) ++bad;
        }
    }
    return bad;
}
