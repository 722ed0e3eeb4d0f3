// Host emulation of the deletion-channel decode (TEST ONLY).
// Compiles polarcub_amd/csrc/trellis_body.h -- the trellis code the kernel runs --
// for the CPU and drives it level-synchronously over the T trellises of a
// codeword, with a scalar SC over the collapsed memoryless rows in natural order
// (the kernel does that part with cross-lane XSub).  Not part of the product
// library; nothing in polarcub_amd loads it.
#include <stdint.h>
#include <string.h>

#include <cmath>
#include <vector>

#include "trellis_body.h"
#include "trellis_n02.h"
#include "sc_del_dense.h"
#include "sc_del_kern.h"

using namespace pcub;

namespace {

struct Ctx {
    const uint32_t* fmask;
    const uint32_t* fval;
    int u;  // next u index
    std::vector<int> info;
};

int fbit(const uint32_t* w, int i) { return (int)((w[i >> 5] >> (i & 31)) & 1u); }

// SC over compact normalised values in natural order; returns the re-encoded vector.
std::vector<int> mem_sc(const std::vector<double>& v, Ctx& cx) {
    const size_t M = v.size();
    if (M == 1) {
        const int i = cx.u++;
        if (fbit(cx.fmask, i)) return {fbit(cx.fval, i)};
        const int d = (int)leaf_v(v[0]);
        cx.info.push_back(d);
        return {d};
    }
    std::vector<double> c(M / 2);
    for (size_t h = 0; h < M / 2; ++h) c[h] = op_f(v[2 * h], v[2 * h + 1]);
    const std::vector<int> xm = mem_sc(c, cx);
    for (size_t h = 0; h < M / 2; ++h) c[h] = op_g(v[2 * h], v[2 * h + 1], (uint32_t)xm[h]);
    const std::vector<int> xp = mem_sc(c, cx);
    std::vector<int> x(M);
    for (size_t h = 0; h < M / 2; ++h) {
        x[2 * h] = xm[h] ^ xp[h];
        x[2 * h + 1] = xp[h];
    }
    return x;
}

// the kernel's capacities: up to 3 guard-band ones when there are any (sc_del.hip)
template <int L, int OC>
using Cap = DelCap<L, OC>;

template <int L>
constexpr int depth_of(int len) {
    return (L / len == 1) ? 0 : (L / len == 2) ? 1 : (L / len == 4) ? 2 : (L / len == 8) ? 3 : 4;
}

// n0 = 3 without ones: every value handed to the memoryless subtree must equal its entry of the
// kernel's segment-state table (sc_del_kern.h, n03_table_entry), indexed by the trellis's
// segment and the bits the subtree returned to it before
std::vector<int> g_k3;
std::vector<uint32_t> g_h3;
long long g_n03_checks = 0;

// the kernel's top level for n0 >= 3 without ones: children of the implicit base trellis
// (BaseT), which must equal the children of the stored one field by field
std::vector<BaseT<16>> g_base;  // per trellis, the segment (m, bits) as BaseT<L> sees it
bool g_use_base = false;
long long g_base_checks = 0;

template <class A, class B>
void same_trellis(const A& x, const B& y, int len) {
    for (int l = 0; l <= len; ++l) {
        if (x.nv[l] != y.nv[l]) throw 4;
        for (int i = 0; i < x.nv[l]; ++i)
            if (x.vp[l][i] != y.vp[l][i]) throw 4;
    }
    for (int i = 0; i < x.nv[0]; ++i)
        if (as_bits(x.pr0[i]) != as_bits(y.pr0[i])) throw 4;
    for (int i = 0; i < x.nv[len]; ++i)
        if (as_bits(x.prL[i]) != as_bits(y.prL[i])) throw 4;
    for (int l = 0; l < len; ++l) {
        if (x.ne[l] != y.ne[l]) throw 4;
        for (int e = 0; e < x.ne[l]; ++e)
            if (x.key[l][e] != y.key[l][e] || as_bits(x.p[l][e]) != as_bits(y.p[l][e])) throw 4;
    }
}

template <int L>
BaseT<L> base_of(int t) {
    BaseT<L> b;
    b.m = g_base[t].m;
    b.d = L - b.m;
    b.y = g_base[t].y;
    b.pins = g_base[t].pins;
    b.pdel = g_base[t].pdel;
    return b;
}

template <int L, int LEN, int OC>
struct Node {
    template <class PT, class CT>
    static void child(const std::vector<PT>& ts, size_t t, CT& c, const uint32_t* dec) {
        trellis_transform<LEN>(ts[t], c, dec);
        if constexpr (LEN == L && OC == 0 && L >= 8) {
            if (g_use_base) {
                Trel<LEN / 2, Cap<L, OC>::V, Cap<L, OC>::E(depth_of<L>(LEN / 2))> cb;
                trellis_transform_base<L>(base_of<L>((int)t), cb, dec);
                same_trellis(cb, c, LEN / 2);
                ++g_base_checks;
                trellis_transform_base<L>(base_of<L>((int)t), c, dec);  // the kernel's child
            }
        }
    }

    template <class PT>
    static std::vector<uint32_t> run(const std::vector<PT>& ts, Ctx& cx, int ones) {
        const size_t T = ts.size();
        std::vector<uint32_t> out(T);
        if constexpr (LEN == 2) {
            Trel<1, Cap<L, OC>::V, Cap<L, OC>::E(depth_of<L>(1))> c;
            std::vector<double> vals(T);
            std::vector<int> xm;
            auto check3 = [&](const std::vector<double>& v) {
                if constexpr (L == 8 && OC == 0) {
                    if (ones != 0 || g_k3.size() != T) return;
                    for (size_t t = 0; t < T; ++t) {
                        const int st = n03_state(g_base[t].m, g_base[t].y);
                        const double e = n03_table_entry(st, g_k3[t], g_h3[t], g_base[t].pdel * 2.0);
                        if (as_bits(e) != as_bits(v[t])) throw 7;
                        ++g_n03_checks;
                    }
                }
            };
            auto record3 = [&](const std::vector<int>& bits) {
                if (g_k3.size() != T) return;
                for (size_t t = 0; t < T; ++t) g_h3[t] |= (uint32_t)(bits[t] & 1) << g_k3[t]++;
            };
            for (int half = 0; half < 2; ++half) {
                if (half) {
                    check3(vals);
                    xm = mem_sc(vals, cx);
                    record3(xm);
                }
                for (size_t t = 0; t < T; ++t) {
                    const uint32_t d = half ? (uint32_t)xm[t] : 0u;
                    double c0, c1;
                    trellis_transform<2>(ts[t], c, half ? &d : nullptr);
                    trellis_marginal(c, c0, c1);
                    if (ones == 0) {  // the kernel's shortcut (no child built) must agree
                        double m0, m1;
                        trellis_collapse(ts[t], half ? &d : nullptr, m0, m1);
                        if (as_bits(c0) != as_bits(m0) || as_bits(c1) != as_bits(m1)) throw 1;
                    }
                    vals[t] = norm_pack(c0, c1);
                }
                if (half) {
                    check3(vals);
                    const std::vector<int> xp = mem_sc(vals, cx);
                    record3(xp);
                    for (size_t t = 0; t < T; ++t) out[t] = (uint32_t)((xm[t] ^ xp[t]) | (xp[t] << 1));
                }
            }
        } else {
            constexpr int H = LEN / 2;
            using CT = Trel<H, Cap<L, OC>::V, Cap<L, OC>::E(depth_of<L>(H))>;
            std::vector<CT> cs(T);
            for (size_t t = 0; t < T; ++t) {
                child(ts, t, cs[t], nullptr);
                trellis_normalize<H>(cs[t]);
            }
            const std::vector<uint32_t> ym = Node<L, H, OC>::run(cs, cx, ones);
            for (size_t t = 0; t < T; ++t) {
                child(ts, t, cs[t], &ym[t]);
                trellis_normalize<H>(cs[t]);
            }
            const std::vector<uint32_t> yp = Node<L, H, OC>::run(cs, cx, ones);
            for (size_t t = 0; t < T; ++t) {
                uint32_t x = 0;
                for (int h = 0; h < H; ++h)
                    x |= ((((ym[t] ^ yp[t]) >> h) & 1u) << (2 * h)) | (((yp[t] >> h) & 1u) << (2 * h + 1));
                out[t] = x;
            }
        }
        return out;
    }
};

// n0 = 2 through the register-resident representation (trellis_n02.h), level-synchronous
// over the T trellises: the kernel's del_n02 with XSub replaced by mem_sc.
bool use_n02 = false;

template <class BitF>
std::vector<uint32_t> decode_n02(const BitF& bit, int len, int tb, double pd, Ctx& cx) {
    const int T = 1 << tb;
    std::vector<Base02> b(T);
    for (int t = 0; t < T; ++t) {
        int s, m;
        segment_of(bit, len, tb, t, s, m);
        b[t].m = m;
        b[t].d = kN02L - m;
        b[t].y = 0;
        if (m <= kN02L)
            for (int i = 0; i < m; ++i) b[t].y |= (uint32_t)(bit(s + i) & 1) << i;
        b[t].pins = 0.5 * (1.0 - pd);
        b[t].pdel = 0.5 * pd;
    }
    // the kernel's per-workgroup segment-state table (n02_table_entry): every value below must
    // equal its table entry bit for bit
    std::vector<double> tab(kN02States * kN02Row, 0.0);
    for (int st = 0; st < kN02States; ++st)
        for (int cv = 0; cv < 5; ++cv) n02_table_entry(st, cv, pd, tab.data() + st * kN02Row);
    auto check_tab = [&](int t, int k, double v) {
        if (as_bits(tab[n02_state(b[t].m, b[t].y) * kN02Row + k]) != as_bits(v)) throw 6;
    };
    std::vector<Child02> c(T);
    std::vector<uint32_t> y[2];
    std::vector<double> vals(T);
    for (int half = 0; half < 2; ++half) {
        // the kernel's collapse (gathered paths), checked against the full scan bit for bit
        auto collapse = [](const Child02& ch, const uint32_t* dec, double& m0, double& m1) {
            Paths02 q;
            n02_paths(ch, q);
            n02_collapse_paths(q, dec, m0, m1);
            double r0, r1;
            n02_collapse(ch, dec, r0, r1);
            if (as_bits(r0) != as_bits(m0) || as_bits(r1) != as_bits(m1)) throw 5;
        };
        for (int t = 0; t < T; ++t) {
            n02_transform(b[t], half ? &y[0][t] : nullptr, c[t]);
            n02_normalize(c[t]);
            double m0, m1;
            collapse(c[t], nullptr, m0, m1);
            vals[t] = norm_pack(m0, m1);
            check_tab(t, half ? 3 + (int)y[0][t] : 0, vals[t]);
        }
        const std::vector<int> xm = mem_sc(vals, cx);
        for (int t = 0; t < T; ++t) {
            double m0, m1;
            const uint32_t d = (uint32_t)xm[t];
            collapse(c[t], &d, m0, m1);
            vals[t] = norm_pack(m0, m1);
            check_tab(t, half ? 7 + 2 * (int)y[0][t] + xm[t] : 1 + xm[t], vals[t]);
        }
        const std::vector<int> xp = mem_sc(vals, cx);
        y[half].resize(T);
        for (int t = 0; t < T; ++t) y[half][t] = (uint32_t)((xm[t] ^ xp[t]) | (xp[t] << 1));
    }
    std::vector<uint32_t> x(T);
    for (int t = 0; t < T; ++t) {
        const uint32_t ym = y[0][t], yp = y[1][t];
        uint32_t o = 0;
        for (int h = 0; h < 2; ++h) o |= ((((ym ^ yp) >> h) & 1u) << (2 * h)) | (((yp >> h) & 1u) << (2 * h + 1));
        x[t] = o;
    }
    return x;
}

OnesProbs ones_probs(int ones, double pd) {  // as sc_del.hip's launcher
    OnesProbs op;
    op.ones = ones;
    for (int i = 0; i < 4; ++i) op.pr[i] = 1.0;
    double comb = 1.0;
    for (int i = 0; ones > 0 && i <= ones; ++i) {
        if (i > 0) comb = comb * (double)(ones - i + 1) / (double)i;
        op.pr[i] = comb * std::pow(1.0 - pd, (double)i) * std::pow(pd, (double)(ones - i));
    }
    return op;
}

template <int N0, int OC>
void decode_one_oc(const uint8_t* w, int len, int n, double pd, int ones, Ctx& cx, std::vector<int>& xhat) {
    constexpr int L = 1 << N0;
    const int tb = n - N0;
    const int T = 1 << tb;
    auto bit = [w](int i) { return (int)w[i]; };
    const OnesProbs op = ones_probs(ones, pd);
    std::vector<Trel<L, Cap<L, OC>::V, Cap<L, OC>::E0>> base(T);
    g_base.assign(T, BaseT<16>{});
    g_k3.assign(L == 8 ? T : 0, 0);
    g_h3.assign(L == 8 ? T : 0, 0u);
    for (int t = 0; t < T; ++t) {
        int s, m;
        segment_of(bit, len, tb, t, s, m);
        trellis_build<L>(base[t], bit, s, m, pd, op);
        const BaseT<L> b = base_segment<L>(bit, s, m, pd);
        g_base[t].m = b.m;
        g_base[t].y = b.y;
        g_base[t].pins = b.pins;
        g_base[t].pdel = b.pdel;
    }
    std::vector<uint32_t> x;
    if constexpr (N0 == 2 && OC == 0) {
        if (use_n02) {
            x = decode_n02(bit, len, tb, pd, cx);
        } else {
            x = Node<L, L, OC>::run(base, cx, ones);
        }
    } else {
        x = Node<L, L, OC>::run(base, cx, ones);
    }
    xhat.assign((size_t)T * L, 0);
    for (int t = 0; t < T; ++t)
        for (int i = 0; i < L; ++i) xhat[(size_t)t * L + i] = (int)((x[t] >> i) & 1u);
}

template <int N0>
void decode_one(const uint8_t* w, int len, int n, double pd, int ones, Ctx& cx, std::vector<int>& xhat) {
    if (ones > 0) decode_one_oc<N0, 3>(w, len, n, pd, ones, cx, xhat);
    else decode_one_oc<N0, 0>(w, len, n, pd, ones, cx, xhat);
}

}  // namespace

extern "C" int emu_decode_deletion(const uint8_t* rx, const int32_t* rx_len, long long B, int stride, int n, int n0,
                                   int ones, double pd, const uint32_t* fmask, const uint32_t* fval, uint32_t* info,
                                   uint32_t* xhat) {
    if (ones < 0 || ones > 3) return -1;
    const int N = 1 << n;
    int K = 0;
    for (int i = 0; i < N; ++i) K += 1 - fbit(fmask, i);
    for (long long b = 0; b < B; ++b) {
        Ctx cx{fmask, fval, 0, {}};
        std::vector<int> xh;
        const uint8_t* w = rx + b * (long long)stride;
        const int len = rx_len[b];
        try {
            switch (n0) {
                case 1: decode_one<1>(w, len, n, pd, ones, cx, xh); break;
                case 2: decode_one<2>(w, len, n, pd, ones, cx, xh); break;
                case 3: decode_one<3>(w, len, n, pd, ones, cx, xh); break;
                case 4: decode_one<4>(w, len, n, pd, ones, cx, xh); break;
                default: return -1;
            }
        } catch (int e) {
            return e == 4 ? -4    // the implicit base's child differs from the stored base's
                 : e == 5 ? -5    // the n0 = 2 path-list collapse differs from the full scan
                          : -3;   // trellis_collapse disagrees with the materialised child's marginal
        }
        if ((int)cx.info.size() != K) return -2;
        for (int i = 0; i < K; ++i)
            if (cx.info[i]) info[(long long)(i >> 5) * B + b] |= 1u << (i & 31);
        for (int i = 0; i < N; ++i)
            if (xh[i]) xhat[(long long)(i >> 5) * B + b] |= 1u << (i & 31);
    }
    return 0;
}

extern "C" void emu_set_n02(int on) { use_n02 = on != 0; }
extern "C" long long emu_n03_checks() { return g_n03_checks; }

// n0 >= 3 without ones: the top level from the implicit base trellis (checked against the stored one)
extern "C" void emu_set_base(int on) { g_use_base = on != 0; }
extern "C" long long emu_base_checks() { return g_base_checks; }

// segment_of on bytes vs segment_of_packed on the packed word (the kernel's parse), for
// random words with long zero runs (guard bands) and every trellis of 1..6 levels.
// Returns the number of disagreeing (word, levels, t) cases.
extern "C" long long emu_check_segments(uint64_t seed, int words) {
    uint64_t st = seed * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&st]() {
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        return st;
    };
    long long bad = 0;
    for (int it = 0; it < words; ++it) {
        const int len = (int)(rnd() % 700);
        std::vector<uint8_t> w(len + 1, 0);
        int i = 0;
        while (i < len) {
            const int run = (int)(rnd() % (rnd() % 4 == 0 ? 90 : 4)) + 1;
            const uint8_t v = (uint8_t)(rnd() % 3 == 0 ? 0 : (rnd() & 1));
            for (int j = 0; j < run && i < len; ++j, ++i) w[i] = (rnd() % 5 == 0) ? (uint8_t)(rnd() & 1) : v;
        }
        std::vector<uint32_t> pk((len + 31) / 32 + 1, 0);
        for (int j = 0; j < len; ++j)
            if (w[j] == 1) pk[j >> 5] |= 1u << (j & 31);
        auto bit = [&w](int j) { return (int)w[j]; };
        for (int lv = 1; lv <= 6; ++lv)
            for (int t = 0; t < (1 << lv); ++t) {
                int s0, m0, s1, m1;
                pcub::segment_of(bit, len, lv, t, s0, m0);
                pcub::segment_of_packed(pk.data(), len, lv, t, s1, m1);
                bad += (s0 != s1 || m0 != m1) ? 1 : 0;
            }
    }
    return bad;
}

// The table-driven layout's own host-visible pieces (sc_del_dense.h), against their definitions:
// dense_segments (a lane's shared descent + per-level splits) = segment_of_packed for every trellis
// of the lane, for 16..256 trellises; enc_hist<L> = DelNode's recursive re-encoding; dense_slot<2>
// = the n02 table's layout for every history.  Returns the number of disagreements.
namespace {
uint32_t enc_ref(uint32_t h, int L) {  // DelNode: x[2i] = ym[i] ^ yp[i], x[2i+1] = yp[i]
    if (L == 1) return h & 1u;
    const int H = L / 2;
    const uint32_t ym = enc_ref(h & ((1u << H) - 1u), H), yp = enc_ref(h >> H, H);
    uint32_t x = 0;
    for (int i = 0; i < H; ++i) x |= ((((ym ^ yp) >> i) & 1u) << (2 * i)) | (((yp >> i) & 1u) << (2 * i + 1));
    return x;
}

template <int TB>
long long dense_seg_check(const std::vector<uint32_t>& pk, int len) {
    constexpr int LV = 1 << (TB - 4);
    long long bad = 0;
    for (int j = 0; j < 16; ++j) {
        const uint32_t jr = pcub::bitrev((uint32_t)j, 4);
        int sa[LV], se[LV];
        pcub::dense_segments<TB>(pk.data(), len, jr, sa, se);
        for (int i = 0; i < LV; ++i) {
            int s, m;
            pcub::segment_of_packed(pk.data(), len, TB, (int)(jr << (TB - 4)) + i, s, m);
            bad += (s != sa[i] || m != se[i] - sa[i]) ? 1 : 0;
        }
    }
    return bad;
}
}  // namespace

extern "C" long long emu_check_dense(uint64_t seed, int words) {
    uint64_t st = seed * 0x9E3779B97F4A7C15ull + 7;
    auto rnd = [&st]() {
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        return st;
    };
    long long bad = 0;
    for (int it = 0; it < words; ++it) {
        const int len = (int)(rnd() % 4000);
        std::vector<uint8_t> w(len + 1, 0);
        int i = 0;
        while (i < len) {
            const int run = (int)(rnd() % (rnd() % 4 == 0 ? 120 : 4)) + 1;
            const uint8_t v = (uint8_t)(rnd() % 3 == 0 ? 0 : (rnd() & 1));
            for (int j = 0; j < run && i < len; ++j, ++i) w[i] = (rnd() % 5 == 0) ? (uint8_t)(rnd() & 1) : v;
        }
        std::vector<uint32_t> pk((len + 31) / 32 + 1, 0);
        for (int j = 0; j < len; ++j)
            if (w[j] == 1) pk[j >> 5] |= 1u << (j & 31);
        bad += dense_seg_check<4>(pk, len) + dense_seg_check<5>(pk, len) + dense_seg_check<6>(pk, len) +
               dense_seg_check<7>(pk, len) + dense_seg_check<8>(pk, len);
    }
    for (uint32_t h = 0; h < 256; ++h) {
        bad += (pcub::enc_hist<8>(h) != enc_ref(h, 8)) ? 1 : 0;
        if (h < 16) bad += (pcub::enc_hist<4>(h) != enc_ref(h, 4)) ? 1 : 0;
    }
    // dense_slot<2>: [0] v1, [1 + xm] v2, [3 + ym] v3, [7 + 2 ym + xm'] v4 (ym = (xm ^ xp) | xp << 1)
    for (uint32_t h = 0; h < 8; ++h) {
        const uint32_t xm = h & 1u, xp = (h >> 1) & 1u, ym = (xm ^ xp) | (xp << 1), xm2 = (h >> 2) & 1u;
        bad += (pcub::dense_slot<2>(0, 0) != 0) ? 1 : 0;
        bad += (pcub::dense_slot<2>(1, h & 1u) != 1 + (int)xm) ? 1 : 0;
        bad += (pcub::dense_slot<2>(2, h & 3u) != 3 + (int)ym) ? 1 : 0;
        bad += (pcub::dense_slot<2>(3, h) != 7 + 2 * (int)ym + (int)xm2) ? 1 : 0;
    }
    for (int k = 0; k < 8; ++k)
        for (uint32_t h = 0; h < (1u << k); ++h) bad += (pcub::dense_slot<3>(k, h) != (1 << k) - 1 + (int)h) ? 1 : 0;
    return bad;
}
