// Host emulation of the q-ary decode schedule (TEST ONLY): compiles
// polarcub_amd/csrc/sc_qary_body.h -- the code the kernel runs -- for the CPU.
#include <stdint.h>

#include <vector>

#include "sc_qary_body.h"

using namespace pcub;

template <int Q>
static int run(const double* xy, long long B, int n, const uint8_t* frozen, uint8_t* info, uint8_t* xhat, int S) {
    const int N = 1 << n;
    const long long ns = 3;  // a few slots, reused across codewords
    std::vector<uint32_t> words((N + 31) / 32, 0u);
    for (int i = 0; i < N; ++i) words[i >> 5] |= (uint32_t)(frozen[i] != 0) << (i & 31);
    int s = 0;
    while ((1 << s) < S) ++s;
    const int D = n - s;
    std::vector<uint8_t> ef((size_t)1 << D);
    for (int k = 0; k < (1 << D); ++k) ef[k] = (uint8_t)first_frozen_depth(words.data(), k, D, S);
    std::vector<double2> scr((size_t)(N - 2 * S) * ((Q + 1) / 2) * ns + 1);
    std::vector<uint32_t> ys((size_t)(N + 3) / 4 * ns);
    QArgs A;
    A.xy = xy;
    A.B = B;
    A.n = n;
    A.frozen = frozen;
    A.ef = ef.data();
    A.info = info;
    A.xhat = xhat;
    A.scratch = scr.data();
    A.ysym = ys.data();
    A.nslots = ns;
    for (long long b = 0; b < B; ++b) {
        switch (S) {
            case 1: decode_qary_cw<Q, 1>(A, b, b % ns, true); break;
            case 2: decode_qary_cw<Q, 2>(A, b, b % ns, true); break;
            case 4: decode_qary_cw<Q, 4>(A, b, b % ns, true); break;
            default: decode_qary_cw<Q, 8>(A, b, b % ns, true); break;
        }
    }
    return 0;
}

// xy: [N][B][q] native layout; info [K][B], xhat [N][B]
extern "C" int emu_decode_qary(const double* xy, long long B, int n, int q, const uint8_t* frozen, uint8_t* info,
                               uint8_t* xhat, int S) {
    if ((1 << n) < 2 * S) return -1;
    switch (q) {
        case 2: return run<2>(xy, B, n, frozen, info, xhat, S);
        case 3: return run<3>(xy, B, n, frozen, info, xhat, S);
        case 4: return run<4>(xy, B, n, frozen, info, xhat, S);
        case 5: return run<5>(xy, B, n, frozen, info, xhat, S);
        case 8: return run<8>(xy, B, n, frozen, info, xhat, S);
        default: return -1;
    }
}
