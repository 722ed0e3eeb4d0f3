// qary_construct.cpp -- degrading / upgrading construction of q-ary polar codes (host C++,
// no GPU).  SURVEY.md section 8(f) rank 3, the q-ary half.
//
// Restates, with the reference's floating-point operations in the reference's order
// (ScalarDistributions/QaryMemorylessDistribution.py):
//   oneHotBinaryMemorylessDistributions  :98-153   (q-1 binary channels, x_j = [x == j] given x >= j)
//   calcXMarginals                       :155-165
//   minusTransform / plusTransform       :182-212
//   degrade_dynamic                      :218-260   (each one-hot channel degraded to M letters,
//                                                   letters re-indexed by the product of the M's)
//   upgrade_dynamic                      :329-475   (each one-hot channel upgraded; every old letter
//                                                   split over its left/centre/right images)
//   calcConversionToYNewMultipliers / yoldToNew_*  :477-483, 717-734
//   removeZeroProbOutput / normalize     :708-715, 736-751  (normalize sums the SORTED flattened list)
//   calcMFromL                           :753-755
//   errorProb / totalVariation           :53-61, 87-96
//   calcTVAndPe_degradingUpgrading       :934-991   (the whole tree; the .npy cache is host Python)
// The binary one-hot degrade/upgrade is the shared core of tv_construct.cpp (tv_core.h).
// Python's sum() over a list is a left-to-right double sum starting from int 0 (exact for
// the first term); list.sort is a stable ascending sort.
#include <float.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "polarcub_construct.h"
#include "tv_core.h"

namespace {

using pcub::tv::Err;
using pcub::tv::Letter;
using pcub::tv::UpAux;

struct QDist {
    int q = 0;
    std::vector<double> p;  // rows x q, probs[y][x]
    int64_t rows() const { return q ? (int64_t)p.size() / q : 0; }
    const double* row(int64_t y) const { return p.data() + y * q; }
    double* row(int64_t y) { return p.data() + y * q; }
};

double row_sum(const double* r, int q) {  // sum(probTuple)
    double s = 0.0;
    for (int x = 0; x < q; ++x) s += r[x];
    return s;
}

QDist minus_t(const QDist& d) {
    QDist o;
    o.q = d.q;
    const int q = d.q;
    const int64_t n = d.rows();
    o.p.assign((size_t)(n * n * q), 0.0);
    int64_t k = 0;
    for (int64_t a = 0; a < n; ++a)
        for (int64_t b = 0; b < n; ++b, ++k) {
            const double* y1 = d.row(a);
            const double* y2 = d.row(b);
            double* t = o.row(k);
            for (int x1 = 0; x1 < q; ++x1)
                for (int x2 = 0; x2 < q; ++x2) t[(x1 + x2) % q] += y1[x1] * y2[x2];
        }
    return o;
}

QDist plus_t(const QDist& d) {
    QDist o;
    o.q = d.q;
    const int q = d.q;
    const int64_t n = d.rows();
    o.p.assign((size_t)(n * n * q * q), 0.0);
    int64_t k = 0;
    for (int64_t a = 0; a < n; ++a)
        for (int64_t b = 0; b < n; ++b)
            for (int u1 = 0; u1 < q; ++u1, ++k) {
                const double* y1 = d.row(a);
                const double* y2 = d.row(b);
                double* t = o.row(k);
                for (int u2 = 0; u2 < q; ++u2) t[u2] += y1[(u1 - u2 + q) % q] * y2[u2];
            }
    return o;
}

int64_t calc_m(int64_t L, int q) { return (int64_t)floor(pow((double)L, 1.0 / (q - 1)) + DBL_EPSILON); }

// oneHotBinaryMemorylessDistributions: channel j has one letter per old letter y (same index)
std::vector<std::vector<Letter>> one_hot(const QDist& d, Err& err) {
    const int q = d.q;
    const int64_t n = d.rows();
    std::vector<double> marg(q, 0.0), pgt(q, 0.0);
    for (int x = 0; x < q; ++x) {
        double s = 0.0;
        for (int64_t y = 0; y < n; ++y) s += d.row(y)[x];
        marg[x] = s;
    }
    for (int x = q - 2; x >= 0; --x) pgt[x] = pgt[x + 1] + marg[x + 1];
    std::vector<std::vector<Letter>> ch(q - 1, std::vector<Letter>((size_t)n));
    for (int64_t y = 0; y < n; ++y) {
        const double* r = d.row(y);
        double prev0 = 0.0, prev1 = 0.0;
        for (int j = q - 2; j >= 0; --j) {
            const double pbone = r[j];
            const double pbzero = (j == q - 2) ? r[j + 1] : prev1 + prev0;
            prev0 = pbzero;
            prev1 = pbone;
            if (j == 0) {
                ch[j][y] = Letter{pbzero, pbone};
            } else {
                if (pgt[j - 1] == 0.0) {
                    err.set(PCUB_EZERODIV);
                    return ch;
                }
                ch[j][y] = Letter{pbzero / pgt[j - 1], pbone / pgt[j - 1]};
            }
        }
    }
    return ch;
}

void remove_zero(QDist& d) {
    std::vector<double> o;
    o.reserve(d.p.size());
    for (int64_t y = 0; y < d.rows(); ++y)
        if (row_sum(d.row(y), d.q) > 0.0) o.insert(o.end(), d.row(y), d.row(y) + d.q);
    d.p.swap(o);
}

void normalize(QDist& d) {
    std::vector<double> t = d.p;
    std::stable_sort(t.begin(), t.end(), [](double a, double b) { return a < b; });
    double s = 0.0;
    for (double v : t) s += v;
    for (double& v : d.p) v /= s;
}

std::vector<int64_t> multipliers(const std::vector<int64_t>& sizes) {
    std::vector<int64_t> m(sizes.size(), 1);
    for (size_t x = 1; x < sizes.size(); ++x) m[x] = m[x - 1] * sizes[x - 1];
    return m;
}

QDist degrade_dynamic(const QDist& d, int64_t L, Err& err) {
    const int q = d.q;
    const int64_t n = d.rows();
    QDist o;
    o.q = q;
    std::vector<std::vector<Letter>> oh = one_hot(d, err);
    if (err.code) return o;
    const int64_t M = calc_m(L, q);
    std::vector<int64_t> sizes(q - 1);
    std::vector<std::vector<int64_t>> map(q - 1, std::vector<int64_t>((size_t)n, 0));  // default: letter 0
    for (int x = 0; x < q - 1; ++x) {
        std::vector<int64_t> g1, g2;
        pcub::tv::merge_equivalent(oh[x], &g1, err);
        if (err.code) return o;
        const std::vector<Letter> dg = pcub::tv::degrade_merged(oh[x], M, &g2, err);
        if (err.code) return o;
        sizes[x] = (int64_t)dg.size();
        for (int64_t y = 0; y < n; ++y)
            if (g1[y] >= 0) map[x][y] = g2[g1[y]];
    }
    const std::vector<int64_t> mult = multipliers(sizes);
    int64_t total = 1;
    for (int64_t s : sizes) total *= s;
    o.p.assign((size_t)(total * q), 0.0);
    for (int64_t y = 0; y < n; ++y) {
        int64_t yn = 0;
        for (int x = 0; x < q - 1; ++x) yn += map[x][y] * mult[x];
        double* t = o.row(yn);
        for (int x = 0; x < q; ++x) t[x] += d.row(y)[x];
    }
    remove_zero(o);
    normalize(o);
    return o;
}

constexpr int kLeft = 0, kCenter = 1, kRight = 2;

double pxy(const std::vector<Letter>& ch, int x, int64_t y) {  // probXGivenY
    const Letter& l = ch[y];
    return (x ? l.p1 : l.p0) / (l.p0 + l.p1);
}

QDist upgrade_dynamic(const QDist& d, int64_t L, Err& err) {
    const int q = d.q;
    const int64_t n = d.rows();
    QDist o;
    o.q = q;
    const std::vector<std::vector<Letter>> orig = one_hot(d, err);
    if (err.code) return o;
    const int64_t M = calc_m(L, q);
    std::vector<std::vector<Letter>> up(q - 1);
    std::vector<int64_t> sizes(q - 1);
    // mapped[(y * (q-1) + i) * 3 + lcr]: upgraded letter of old letter y in channel i, or -1 (None)
    std::vector<int64_t> mapped((size_t)(n * (q - 1) * 3), -1);
    for (int i = 0; i < q - 1; ++i) {
        std::vector<Letter> ch = orig[i];
        std::vector<int64_t> g1;
        pcub::tv::merge_equivalent(ch, &g1, err);
        if (err.code) return o;
        std::vector<UpAux> aux;
        up[i] = pcub::tv::upgrade_merged(ch, M, err, &aux);
        if (err.code) return o;
        sizes[i] = (int64_t)up[i].size();
        std::vector<std::vector<int64_t>> members(ch.size());  // merged letter -> old letters
        for (int64_t y = 0; y < n; ++y)
            if (g1[y] >= 0) members[g1[y]].push_back(y);
        for (size_t z = 0; z < aux.size(); ++z) {
            const std::vector<int64_t>* sets[3] = {&aux[z].l, &aux[z].c, &aux[z].r};
            for (int lcr = 0; lcr < 3; ++lcr)
                for (int64_t k : *sets[lcr])
                    for (int64_t y : members[k]) {
                        int64_t& m = mapped[(size_t)((y * (q - 1) + i) * 3 + lcr)];
                        if (m != -1) {
                            err.set(PCUB_EASSERT);
                            return o;
                        }
                        m = (int64_t)z;
                    }
        }
    }
    const std::vector<int64_t> mult = multipliers(sizes);
    int64_t total = 1;
    for (int64_t s : sizes) total *= s;
    o.p.assign((size_t)(total * q), 0.0);
    std::vector<int> lcr(q - 1);
    std::vector<double> pr0(q - 1), pr1(q - 1), mfn(q + 1);
    for (int64_t y = 0; y < n; ++y) {
        auto M3 = [&](int i, int c) { return mapped[(size_t)((y * (q - 1) + i) * 3 + c)]; };
        const double ymarg = row_sum(d.row(y), q);
        for (int i = 0; i < q - 1; ++i) {  // initializeLCRVector
            if (M3(i, kLeft) == -1) {
                if (M3(i, kRight) != -1) {
                    err.set(PCUB_EASSERT);
                    return o;
                }
                lcr[i] = kCenter;
            } else {
                if (M3(i, kCenter) != -1 || M3(i, kRight) == -1) {
                    err.set(PCUB_EASSERT);
                    return o;
                }
                lcr[i] = kLeft;
            }
        }
        for (;;) {
            int64_t yn = 0;
            for (int i = 0; i < q - 1; ++i) {
                const int64_t m = M3(i, lcr[i]);
                yn += (m != -1 ? m : 0) * mult[i];
            }
            // calc_probs_of_x_ynew_given_yold
            for (int i = 0; i < q - 1; ++i) {
                const std::vector<Letter>& U = up[i];
                const std::vector<Letter>& O = orig[i];
                if (O[y].p0 + O[y].p1 == 0.0) {
                    pr0[i] = pr1[i] = -1000.0;
                } else if (lcr[i] == kCenter) {
                    pr0[i] = pxy(O, 0, y);
                    pr1[i] = pxy(O, 1, y);
                } else {
                    const int64_t zn = M3(i, lcr[i]);
                    const int64_t zo = M3(i, lcr[i] == kRight ? kLeft : kRight);
                    double t[2];
                    for (int x = 0; x < 2; ++x) {
                        const double fm = pxy(U, x, zn);
                        double num, den;
                        if (pxy(U, x, zo) < 0.5) {
                            den = pxy(U, x, zn) - pxy(U, x, zo);
                            num = pxy(O, x, y) - pxy(U, x, zo);
                        } else {
                            den = pxy(U, 1 - x, zo) - pxy(U, 1 - x, zn);
                            num = pxy(U, 1 - x, zo) - pxy(O, 1 - x, y);
                        }
                        if (den == 0.0) {
                            err.set(PCUB_EZERODIV);
                            return o;
                        }
                        t[x] = fm * num / den;
                    }
                    pr0[i] = t[0];
                    pr1[i] = t[1];
                }
            }
            mfn[q - 1] = 1.0;
            for (int i = q - 2; i >= 0; --i) mfn[i] = mfn[i + 1] * (pr0[i] + pr1[i]);
            double ztn = 1.0;
            double* row = o.row(yn);
            for (int x = 0; x < q; ++x) {
                double prob;
                if (x < q - 1) {
                    prob = ztn * pr1[x] * mfn[x + 1];
                    ztn *= pr0[x];
                } else {
                    prob = ztn;
                }
                prob *= ymarg;
                row[x] += prob;
            }
            // iterateLCRVector
            bool more = false;
            for (int i = 0; i < q - 1; ++i) {
                if (lcr[i] == kLeft) {
                    lcr[i] = kRight;
                    more = true;
                    break;
                } else if (lcr[i] == kRight) {
                    lcr[i] = kLeft;
                }
            }
            if (!more) break;
        }
    }
    remove_zero(o);
    normalize(o);
    return o;
}

double error_prob(const QDist& d) {
    double total = 0.0;
    std::vector<double> t(d.q);
    for (int64_t y = 0; y < d.rows(); ++y) {
        t.assign(d.row(y), d.row(y) + d.q);
        std::stable_sort(t.begin(), t.end(), [](double a, double b) { return a < b; });
        double s = 0.0;
        for (int x = 0; x + 1 < d.q; ++x) s += t[x];
        total += s;
    }
    return total;
}

double total_variation(const QDist& d) {
    double s = 0.0;
    for (int64_t y = 0; y < d.rows(); ++y) {
        const double* r = d.row(y);
        for (int a = 0; a < d.q; ++a)
            for (int b = 0; b < d.q; ++b) s += fabs(r[a] - r[b]);
    }
    return s / (double)(2 * (d.q - 1));
}

QDist load(int q, const double* probs, int64_t n) {
    QDist d;
    d.q = q;
    d.p.assign(probs, probs + n * q);
    return d;
}

int store(const QDist& d, double* out, int64_t cap, int64_t* out_n) {
    *out_n = d.rows();
    if (d.rows() > cap) return PCUB_EINVAL;
    std::copy(d.p.begin(), d.p.end(), out);
    return 0;
}

// one polarisation tree, leaves in u order (minus child first), each level's 2^m children
// on `threads` workers
int tree(QDist root, int n, int64_t L, bool up, int threads, double* vec) {
    std::vector<QDist> lvl{std::move(root)};
    for (int m = 1; m <= n; ++m) {
        const size_t cnt = lvl.size() * 2;
        std::vector<QDist> nxt(cnt);
        std::vector<Err> errs(cnt);
        std::atomic<size_t> next_task{0};
        auto work = [&]() {
            for (size_t t; (t = next_task.fetch_add(1)) < cnt;) {
                const QDist c = (t & 1) ? plus_t(lvl[t / 2]) : minus_t(lvl[t / 2]);
                nxt[t] = up ? upgrade_dynamic(c, L, errs[t]) : degrade_dynamic(c, L, errs[t]);
            }
        };
        const int nt = std::max(1, std::min<int>(threads, (int)cnt));
        std::vector<std::thread> pool;
        for (int i = 1; i < nt; ++i) pool.emplace_back(work);
        work();
        for (std::thread& th : pool) th.join();
        for (const Err& e : errs)
            if (e.code) return e.code;
        lvl.swap(nxt);
    }
    for (size_t i = 0; i < lvl.size(); ++i) vec[i] = up ? total_variation(lvl[i]) : error_prob(lvl[i]);
    return 0;
}

bool q_ok(int32_t q) { return q >= 2 && q <= 64; }

}  // namespace

extern "C" int pcub_qmd_degrade(int32_t q, const double* probs, int64_t n, int64_t L, double* out, int64_t out_cap,
                                int64_t* out_n) {
    if (!q_ok(q) || n < 1 || L < 1 || !probs || !out || !out_n) return PCUB_EINVAL;
    Err err;
    const QDist o = degrade_dynamic(load(q, probs, n), L, err);
    if (err.code) return err.code;
    return store(o, out, out_cap, out_n);
}

extern "C" int pcub_qmd_upgrade(int32_t q, const double* probs, int64_t n, int64_t L, double* out, int64_t out_cap,
                                int64_t* out_n) {
    if (!q_ok(q) || n < 1 || L < 1 || !probs || !out || !out_n) return PCUB_EINVAL;
    Err err;
    const QDist o = upgrade_dynamic(load(q, probs, n), L, err);
    if (err.code) return err.code;
    return store(o, out, out_cap, out_n);
}

extern "C" int pcub_qmd_error_prob(int32_t q, const double* probs, int64_t n, double* pe, double* tv) {
    if (!q_ok(q) || n < 0 || (n > 0 && !probs) || !pe || !tv) return PCUB_EINVAL;
    const QDist d = load(q, probs, n);
    *pe = error_prob(d);
    *tv = total_variation(d);
    return 0;
}

extern "C" int pcub_qary_construct(int32_t q, int32_t n, int64_t L, const double* xprobs, int64_t nx,
                                   const double* xyprobs, int64_t nxy, double* TV, double* Pe, int32_t threads) {
    if (!q_ok(q) || n < 0 || n > 24 || L < 1 || !xyprobs || nxy < 1 || !Pe || !TV || (xprobs && nx < 1))
        return PCUB_EINVAL;
    if (threads < 1) threads = (int32_t)std::max(1u, std::thread::hardware_concurrency());
    const size_t N = (size_t)1 << n;
    if (xprobs) {
        const int rc = tree(load(q, xprobs, nx), n, L, true, threads, TV);
        if (rc) return rc;
    } else {
        std::fill(TV, TV + N, 0.0);
    }
    return tree(load(q, xyprobs, nxy), n, L, false, threads, Pe);
}
