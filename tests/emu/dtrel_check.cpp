// Host check of trellis_dense.h against trellis_body.h (test-only): on random segments (length,
// received bits, deletion probability) and random decision histories, every stage of the dense
// representation -- transform from the implicit base, normalise, transform, collapse -- must hold
// the same edges in the same creation order, the same vertices in the same insertion order and
// bit-identical probabilities as Trel's, and the same collapsed values.
//   dtrel_check <cases> <seed>    (exit status 0: all equal)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "trellis_dense.h"

using namespace pcub;

static long long g_fail = 0, g_cmp = 0;

static bool same_bits(double a, double b) { return as_bits(a) == as_bits(b); }

template <class TR, int L, int D>
static void compare(const TR& t, const DTrel<L, D>& d, const char* what) {
    constexpr int LEN = DTrel<L, D>::LEN;
    ++g_cmp;
    if (d.m > L) {  // no edges either way
        for (int l = 0; l < LEN; ++l)
            if (t.ne[l] != 0) {
                if (g_fail++ < 10) std::printf("%s: m > L but Trel layer %d has %d edges\n", what, l, (int)t.ne[l]);
                return;
            }
        return;
    }
    for (int l = 0; l <= LEN; ++l) {
        if (t.nv[l] != d.nv[l]) {
            if (g_fail++ < 10) std::printf("%s: layer %d vertices %d vs %d\n", what, l, (int)t.nv[l], (int)d.nv[l]);
            return;
        }
        for (int i = 0; i < t.nv[l]; ++i)
            if (t.vp[l][i] != d.lo(l) + d.vord[l][i]) {
                if (g_fail++ < 10) std::printf("%s: layer %d vertex %d: %d vs %d\n", what, l, i, (int)t.vp[l][i], d.lo(l) + d.vord[l][i]);
                return;
            }
    }
    for (int l = 0; l < LEN; ++l) {
        if (t.ne[l] != d.ne[l]) {
            if (g_fail++ < 10) std::printf("%s: edge layer %d: %d vs %d edges\n", what, l, (int)t.ne[l], (int)d.ne[l]);
            return;
        }
        for (int r = 0; r < t.ne[l]; ++r) {
            const uint32_t k = t.key[l][r];
            const int s = d.eord[l][r];
            if (ek_from(k) != d.s_from(l, s) || ek_to(k) != d.s_to(l, s) || ek_lbl(k) != DTrel<L, D>::s_lbl(s) ||
                !same_bits(t.p[l][r], d.p[l][s])) {
                if (g_fail++ < 10)
                    std::printf("%s: layer %d edge %d: (%d->%d,%d) %.17g vs (%d->%d,%d) %.17g\n", what, l, r, ek_from(k), ek_to(k),
                                ek_lbl(k), t.p[l][r], d.s_from(l, s), d.s_to(l, s), DTrel<L, D>::s_lbl(s), d.p[l][s]);
                return;
            }
        }
    }
}

static void cmp_val(double a, double b, const char* what) {
    ++g_cmp;
    if (!same_bits(a, b) && !(a != a && b != b)) {
        if (g_fail++ < 10) std::printf("%s: %.17g vs %.17g\n", what, a, b);
    }
}

// the DelNode walk below a depth-D node, both representations side by side, random decisions
template <int L, int D>
struct Walk {
    using Cap = DelCap<L, 0>;
    static constexpr int LEN = L >> D;
    template <class TR>
    static uint32_t run(const TR& t, const DTrel<L, D>& d, std::mt19937_64& rng) {
        if constexpr (LEN == 2) {
            double a0, a1, b0, b1;
            trellis_collapse(t, nullptr, a0, a1);
            dtrellis_collapse(d, nullptr, b0, b1);
            cmp_val(a0, b0, "collapse minus m0");
            cmp_val(a1, b1, "collapse minus m1");
            const uint32_t xm = (uint32_t)(rng() & 1u);
            trellis_collapse(t, &xm, a0, a1);
            dtrellis_collapse(d, &xm, b0, b1);
            cmp_val(a0, b0, "collapse plus m0");
            cmp_val(a1, b1, "collapse plus m1");
            const uint32_t xp = (uint32_t)(rng() & 1u);
            return (xm ^ xp) | (xp << 1);
        } else {
            constexpr int H = LEN / 2;
            Trel<H, Cap::V, Cap::E(D + 1)>* c = new Trel<H, Cap::V, Cap::E(D + 1)>;
            DTrel<L, D + 1>* e = new DTrel<L, D + 1>();
            uint32_t y[2];
            for (int half = 0; half < 2; ++half) {
                trellis_transform<LEN>(t, *c, half ? &y[0] : nullptr);
                trellis_normalize<H>(*c);
                dtrellis_transform(d, *e, half ? &y[0] : nullptr);
                dtrellis_normalize(*e);
                compare(*c, *e, half ? "transform plus" : "transform minus");
                y[half] = Walk<L, D + 1>::run(*c, *e, rng);
            }
            delete c;
            delete e;
            uint32_t x = 0;
            for (int h = 0; h < H; ++h) x |= ((((y[0] ^ y[1]) >> h) & 1u) << (2 * h)) | (((y[1] >> h) & 1u) << (2 * h + 1));
            return x;
        }
    }
};

template <int L>
static void one_case(std::mt19937_64& rng) {
    using Cap = DelCap<L, 0>;
    const double pds[] = {0.0, 0.01, 0.1, 0.2, 0.37, 0.5, 0.9, 1.0};
    BaseT<L> b;
    // lengths around L (most segments), a few far from it, a few with no edges (m > L)
    const int r = (int)(rng() % 16);
    b.m = r < 10 ? (int)(L - (rng() % 5)) : r < 14 ? (int)(rng() % (L + 1)) : (int)(L + 1 + rng() % 3);
    b.d = L - b.m;
    b.y = (uint32_t)rng() & ((b.m >= 32) ? 0xffffffffu : ((1u << (b.m < 0 ? 0 : (b.m > L ? 0 : b.m))) - 1u));
    const double pd = pds[rng() % 8];
    b.pins = 0.5 * (1.0 - pd);
    b.pdel = 0.5 * pd;
    auto* t = new Trel<L / 2, Cap::V, Cap::E(1)>;
    auto* d = new DTrel<L, 1>();
    uint32_t y[2];
    for (int half = 0; half < 2; ++half) {
        trellis_transform_base<L>(b, *t, half ? &y[0] : nullptr);
        trellis_normalize<L / 2>(*t);
        dtrellis_transform_base(b, *d, half ? &y[0] : nullptr);
        dtrellis_normalize(*d);
        compare(*t, *d, half ? "base plus" : "base minus");
        y[half] = Walk<L, 1>::run(*t, *d, rng);
    }
    delete t;
    delete d;
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? std::atoll(argv[1]) : 20000;
    std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1);
    for (long long i = 0; i < n; ++i) {
        if (i & 1) one_case<16>(rng);
        else one_case<8>(rng);
    }
    std::printf("dtrel_check: %lld cases, %lld comparisons, %lld mismatches\n", n, g_cmp, g_fail);
    return g_fail ? 1 : 0;
}
