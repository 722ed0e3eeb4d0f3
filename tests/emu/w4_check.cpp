// Host check of trellis_wave.h (the n0 = 4 wave-per-task trellises) against trellis_body.h's Trel
// walk (test-only): on random segments (length, received bits, deletion probability) and random
// decision histories, the three rows of every depth-3 node -- minus, plus after 0, plus after 1 --
// must be bit-identical to DelBase / DelNode's (the collapse values the memoryless subtree reads),
// and the re-encoding of the 16 decisions must equal the recursion's.
//   w4_check <cases> <seed>    (exit status 0: all equal)
#include <cstdio>
#include <cstdlib>
#include <random>

#include "trellis_wave.h"

using namespace pcub;

struct HostRun {
    template <class F>
    void operator()(F&& f) const {
        for (int l = 0; l < 64; ++l) f(l);
    }
};

static long long g_fail = 0, g_cmp = 0;

// DelBase<16> / DelNode walk on Trel, rows[k][0..2] per depth-3 node k; returns the root encoding
static uint32_t ref_rows(const BaseT<16>& b, uint32_t hist, double rows[8][3]) {
    using Cap = DelCap<16, 0>;
    auto* c1 = new Trel<8, Cap::V, Cap::E(1)>;
    auto* c2 = new Trel<4, Cap::V, Cap::E(2)>;
    auto* c3 = new Trel<2, Cap::V, Cap::E(3)>;
    uint32_t y1[2];
    for (int h1 = 0; h1 < 2; ++h1) {
        trellis_transform_base<16>(b, *c1, h1 ? &y1[0] : nullptr);
        trellis_normalize<8>(*c1);
        uint32_t y2[2];
        for (int h2 = 0; h2 < 2; ++h2) {
            trellis_transform<8>(*c1, *c2, h2 ? &y2[0] : nullptr);
            trellis_normalize<4>(*c2);
            uint32_t y3[2];
            for (int h3 = 0; h3 < 2; ++h3) {
                trellis_transform<4>(*c2, *c3, h3 ? &y3[0] : nullptr);
                trellis_normalize<2>(*c3);
                const int k = 4 * h1 + 2 * h2 + h3;
                double m0, m1;
                trellis_collapse(*c3, nullptr, m0, m1);
                rows[k][0] = norm_pack(m0, m1);
                for (uint32_t xm = 0; xm < 2; ++xm) {
                    trellis_collapse(*c3, &xm, m0, m1);
                    rows[k][1 + xm] = norm_pack(m0, m1);
                }
                const uint32_t xm = (hist >> (2 * k)) & 1u, xp = (hist >> (2 * k + 1)) & 1u;
                y3[h3] = (xm ^ xp) | (xp << 1);
            }
            y2[h2] = w4_combine(y3[0], y3[1], 2);
        }
        y1[h1] = w4_combine(y2[0], y2[1], 4);
    }
    delete c1;
    delete c2;
    delete c3;
    return w4_combine(y1[0], y1[1], 8);
}

static bool same_bits(double a, double b) { return as_bits(a) == as_bits(b) || (a != a && b != b); }

int main(int argc, char** argv) {
    const long long n = argc > 1 ? std::atoll(argv[1]) : 2000;
    std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1);
    const double pds[] = {0.0, 0.01, 0.1, 0.1, 0.2, 0.37, 0.5, 0.9, 1.0};
    auto* wb = new W4Buf;
    auto* cache = new uint8_t[kW4Cache];
    long long hist_m[18] = {};
    for (long long i = 0; i < n; ++i) {
        const int r = (int)(rng() % 16);
        const int m = r < 10 ? (int)(16 - (rng() % 6)) : r < 15 ? (int)(rng() % 17) : (int)(17 + rng() % 3);
        ++hist_m[m < 17 ? m : 17];
        const uint32_t y = (m <= 16) ? (uint32_t)(rng() & ((1ull << m) - 1ull)) : 0u;
        const double pd = pds[rng() % 9];
        const uint32_t hist = (uint32_t)(rng() & 0xffffu);
        BaseT<16> b;
        b.m = m;
        b.d = 16 - m;
        b.y = y;
        b.pins = 0.5 * (1.0 - pd);
        b.pdel = 0.5 * pd;
        double rows[8][3];
        const uint32_t xr = ref_rows(b, hist, rows);
        W4Dims D;
        D.set(m, y, pd);
        // half the cases run through the depth-1 / depth-2 cache as sc_del_w4.hip drives it, with random
        // nodes skipped (rate-0 nodes run no tasks, so a later node may find its trellis not cached)
        const bool use_cache = (i & 1) != 0;
        const uint32_t skip = use_cache ? (uint32_t)(rng() & rng() & 0xffu) : 0u;
        int have1 = -1, have2 = -1;
        for (int k = 0; k < 8; ++k) {
            if ((skip >> k) & 1u) continue;
            int mode = 0;
            if (use_cache) {
                mode = (have2 == (k >> 1)) ? kW4Load2 : ((have1 == (k >> 2)) ? kW4Load1 : kW4Save1) | kW4Save2;
                if (mode & kW4Save1) have1 = k >> 2;
                have2 = k >> 1;
            }
            w4_task(HostRun{}, *wb, D, k, hist, use_cache ? cache : nullptr, mode);
            for (int o = 0; o < 3; ++o) {
                ++g_cmp;
                if (!same_bits(wb->out[o], rows[k][o])) {
                    if (g_fail++ < 12)
                        std::printf("case %lld (m=%d y=%#x pd=%g hist=%#x) node %d row %d: %.17g vs ref %.17g\n", i, m, y, pd,
                                    hist, k, o, wb->out[o], rows[k][o]);
                }
            }
        }
        ++g_cmp;
        if (w4_enc16(hist) != xr && g_fail++ < 12) std::printf("case %lld: encoding %#x vs %#x\n", i, w4_enc16(hist), xr);
    }
    delete wb;
    delete[] cache;
    std::printf("w4_check: %lld cases, %lld comparisons, %lld mismatches; m histogram:", n, g_cmp, g_fail);
    for (int m = 0; m < 18; ++m) std::printf(" %lld", hist_m[m]);
    std::printf("\n");
    return g_fail ? 1 : 0;
}
