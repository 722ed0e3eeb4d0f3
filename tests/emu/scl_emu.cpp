// Test-only host build of the list decoder (scl_body.h), ns = 1 slabs, one codeword at a time.
// The same code runs on the GPU in k_scl (scl.hip); tests/test_scl.py checks this build against
// the oracle's restatement (oracle/scl_oracle.py).
#include <stdint.h>

#include <vector>

// slab traffic and frame-loop iterations of the last emu_scl call (emu_scl_counts)
static long long g_touch_bytes = 0, g_frames = 0;
#define PCUB_SCL_TOUCH(b) (g_touch_bytes += (b))
#define PCUB_SCL_FRAME() (++g_frames)
#include "scl_body.h"

extern "C" void emu_scl_counts(long long* bytes, long long* frames) {
    *bytes = g_touch_bytes;
    *frames = g_frames;
}

extern "C" int emu_scl(const double* xy, long long B, int q, int n, int L, const uint8_t* frozen,
                       const uint8_t* fvals, int nF, const uint8_t* actual, int K, uint8_t* out_info,
                       double* out_prob, int* out_size, double* out_actual, int use_log) {
    g_touch_bytes = 0;
    g_frames = 0;
    pcub::SclLayout Y;
    Y.init(n, q, L, K);
    std::vector<double> cells((size_t)Y.ncells);
    std::vector<uint8_t> bytes((size_t)Y.nbytes);
    pcub::SclArgs A;
    A.xy = xy;
    A.B = B;
    A.n = n;
    A.q = q;
    A.L = L;
    A.K = K;
    A.frozen = frozen;
    A.fvals = fvals;
    A.nF = nF;
    A.actual = actual;
    A.out_info = out_info;
    A.out_prob = out_prob;
    A.out_size = out_size;
    A.out_actual = out_actual;
    A.log = use_log;
    A.cells = cells.data();
    A.bytes = bytes.data();
    A.ns = 1;
    for (long long cw = 0; cw < B; ++cw) pcub::scl_decode_cw(A, cw, 0, true);
    return 0;
}
