// tv_construct.cpp -- Tal-Vardy degrading / upgrading construction of binary polar
// codes (host C++, no GPU).  SURVEY.md section 8(f) rank 3: the frozen-set design
// that runs once per code on either side of the decode path.
//
// Restates, with the reference's floating-point operations in the reference's
// order (Python floats are IEEE binary64; this file is built with
// -ffp-contract=off and libm's log2, which CPython's math.log2 calls):
//   BinaryMemorylessDistribution.removeZeroProbOutput   ScalarDistributions/BinaryMemorylessDistribution.py:92-108
//   .sortProbs                                          :110-165
//   .mergeEquivalentSymbols (math.isclose, rel 1e-9)    :167-208
//   .normalize                                          :88-90
//   .minusTransform / .plusTransform                    :261-285
//   .degrade(L)  (greedy merge of LLR-adjacent letters)  :287-346
//   .upgrade(L)  (greedy split of a letter onto its neighbours) :348-427
//   eta / hxgiveny                                      :450-477
//   _calcKey_degrade / _calcKey_upgrade / upgradedLeftRightProbs  :510-621
//   calcFrozenSet_degradingUpgrading (TV / Pe vectors)  :624-680
//   LinkedListHeap (array min-heap over a doubly linked list, the reference's
//   tie behaviour: an element rises past an equal key)  ScalarDistributions/UpgradingDegrading/LinkedListHeap.py:4-191
// The construction runs the 2^m independent channels of each level on a thread pool.
// The binary core (tv_core.h) is shared with the q-ary construction (qary_construct.cpp).
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "polarcub_construct.h"
#include "tv_core.h"

namespace pcub {
namespace tv {

const double kInf = INFINITY;

double py_sum(const Letter& l) { return l.p0 + l.p1; }  // sum([p0, p1]) = (0 + p0) + p1

double eta(double p, Err& err) {
    if (!(0.0 <= p && p <= 1.0 + 10 * 2.220446049250313e-16)) err.set(PCUB_EASSERT);
    if (!(p < 1.0)) p = 1.0;  // min(1.0, p)
    return p == 0.0 ? 0.0 : -p * log2(p);
}

double hxgiveny(const Letter& d, Err& err) {
    const double py = d.p0 + d.p1;
    if (py == 0.0) {
        err.set(PCUB_EZERODIV);
        return 0.0;
    }
    return py * (eta(d.p0 / py, err) + eta(d.p1 / py, err));
}

// math.isclose(a, b) with rel_tol = 1e-9, abs_tol = 0
bool py_isclose(double a, double b) {
    if (a == b) return true;
    if (isinf(a) || isinf(b)) return false;
    const double diff = fabs(b - a);
    return diff <= fabs(1e-09 * b) || diff <= fabs(1e-09 * a) || diff <= 0.0;
}

// group[i]: index of the letter original letter i now belongs to (-1: dropped)
struct Dist {
    std::vector<Letter> p;
    std::vector<int64_t> members;  // per current letter: the original letters, as a contiguous run
    std::vector<int64_t> start;    // run start per letter (start.size() == p.size() + 1)
};

void remove_zero(std::vector<Letter>& p, std::vector<int64_t>& id) {
    size_t w = 0;
    for (size_t i = 0; i < p.size(); ++i)
        if (py_sum(p[i]) > 0.0) {
            p[w] = p[i];
            id[w] = id[i];
            ++w;
        }
    p.resize(w);
    id.resize(w);
}

// sortProbs: letters with p(x=0|y) > 1/2 first, by ascending p(x=1|y); then the rest by
// descending p(x=0|y); Python's sort is stable and compares keys with '<' only.
void sort_probs(std::vector<Letter>& p, std::vector<int64_t>& id) {
    struct K {
        double key;
        size_t i;
    };
    std::vector<K> zero, one;
    for (size_t i = 0; i < p.size(); ++i) {
        const double s = py_sum(p[i]);
        if (p[i].p0 / s > 0.5) zero.push_back({p[i].p1 / s, i});
        else one.push_back({-p[i].p0 / s, i});
    }
    auto lt = [](const K& a, const K& b) { return a.key < b.key; };
    std::stable_sort(zero.begin(), zero.end(), lt);
    std::stable_sort(one.begin(), one.end(), lt);
    std::vector<Letter> np;
    std::vector<int64_t> nid;
    np.reserve(p.size());
    nid.reserve(p.size());
    for (const K& k : zero) {
        np.push_back(p[k.i]);
        nid.push_back(id[k.i]);
    }
    for (const K& k : one) {
        np.push_back(p[k.i]);
        nid.push_back(id[k.i]);
    }
    p.swap(np);
    id.swap(nid);
}

void normalize(std::vector<Letter>& p) {
    double s = 0.0;  // sum(sum(probs, [])): flattened, left to right
    for (const Letter& l : p) {
        s = s + l.p0;
        s = s + l.p1;
    }
    for (Letter& l : p) {
        l.p0 = l.p0 / s;
        l.p1 = l.p1 / s;
    }
}

// mergeEquivalentSymbols; grp[k] = merged letter of input letter k (or -1)
void merge_equivalent(std::vector<Letter>& p, std::vector<int64_t>* grp, Err& err) {
    const size_t n0 = p.size();
    std::vector<int64_t> id(n0);
    for (size_t i = 0; i < n0; ++i) id[i] = (int64_t)i;
    remove_zero(p, id);
    if (grp) grp->assign(n0, -1);
    if (p.empty()) {
        err.set(PCUB_EINDEX);  // self.probs[0] on an empty list
        return;
    }
    sort_probs(p, id);
    std::vector<Letter> out;
    out.reserve(p.size());
    out.push_back(p[0]);
    if (grp) (*grp)[id[0]] = 0;
    for (size_t i = 1; i < p.size(); ++i) {
        const Letter& a = p[i];
        const Letter& prev = out.back();
        const double sa = py_sum(a), sp = py_sum(prev);
        const bool close = py_isclose(a.p0 / sa, prev.p0 / sp) && py_isclose(a.p1 / sa, prev.p1 / sp);
        if (!close) out.push_back(a);
        else {
            out.back().p0 += a.p0;
            out.back().p1 += a.p1;
        }
        if (grp) (*grp)[id[i]] = (int64_t)out.size() - 1;
    }
    normalize(out);
    p.swap(out);
}

// LinkedListHeap: elements in list order 0..n-1 (initial), a binary min-heap over them.
class ListHeap {
  public:
    std::vector<double> key;
    std::vector<int64_t> prev, next, heap, pos;

    explicit ListHeap(const std::vector<double>& keys) {
        const int64_t n = (int64_t)keys.size();
        key = keys;
        prev.resize(n);
        next.resize(n);
        pos.resize(n);
        heap.reserve(n);
        for (int64_t i = 0; i < n; ++i) {  // insertAtTail, one at a time
            prev[i] = i - 1;
            next[i] = i + 1 < n ? i + 1 : -1;
            pos[i] = (int64_t)heap.size();
            heap.push_back(i);
            up(i);
        }
    }
    int64_t size() const { return (int64_t)heap.size(); }
    int64_t extract_min() {
        const int64_t e = heap[0];
        if (prev[e] >= 0) next[prev[e]] = next[e];
        if (next[e] >= 0) prev[next[e]] = prev[e];
        const int64_t last = heap.back();
        heap.pop_back();
        if (!heap.empty()) {
            heap[0] = last;
            pos[last] = 0;
            down(last);
        }
        return e;
    }
    void update(int64_t e, double k) {
        const double old = key[e];
        key[e] = k;
        if (old < k) down(e);
        else if (old > k) up(e);
    }
    int64_t head() const {
        // the first element still in the list: follow prev from any live element
        int64_t e = heap.empty() ? -1 : heap[0];
        while (e >= 0 && prev[e] >= 0) e = prev[e];
        return e;
    }

  private:
    void swap_(int64_t a, int64_t b) {
        std::swap(pos[a], pos[b]);
        heap[pos[a]] = a;
        heap[pos[b]] = b;
    }
    void up(int64_t e) {
        for (;;) {
            const int64_t i = pos[e];
            const int64_t par = (i + 1) / 2 - 1;
            if (par < 0) break;
            const int64_t pe = heap[par];
            if (key[pe] < key[e]) break;  // equal keys rise
            swap_(e, pe);
        }
    }
    void down(int64_t e) {
        for (;;) {
            const int64_t i = pos[e];
            const int64_t l = 2 * i + 1, r = 2 * i + 2;
            double mk = key[e];
            int64_t mc = -1;
            if (l < size() && key[heap[l]] < mk) {
                mk = key[heap[l]];
                mc = heap[l];
            }
            if (r < size() && key[heap[r]] < mk) {
                mk = key[heap[r]];
                mc = heap[r];
            }
            if (mc < 0) break;
            swap_(e, mc);
        }
    }
};

double key_degrade(const Letter& l, const Letter& c, Err& err) {
    const Letter m{l.p0 + c.p0, l.p1 + c.p1};
    return hxgiveny(m, err) - hxgiveny(l, err) - hxgiveny(c, err);
}

// degrade(L) on merged letters; grp[k] = output letter of merged letter k
std::vector<Letter> degrade_merged(const std::vector<Letter>& in, int64_t L, std::vector<int64_t>* grp, Err& err) {
    const int64_t n = (int64_t)in.size();
    std::vector<Letter> d = in;
    std::vector<double> keys(n);
    for (int64_t i = 0; i < n; ++i) keys[i] = i == 0 ? kInf : key_degrade(d[i - 1], d[i], err);
    ListHeap h(keys);
    std::vector<int64_t> into(n, -1);  // element merged into (its left neighbour at the time)
    while (h.size() > L) {
        const int64_t t = h.extract_min();
        const int64_t l = h.prev[t], r = h.next[t];
        if (l < 0) {
            err.set(PCUB_EATTR);  // None.data in the reference
            break;
        }
        d[l].p0 += d[t].p0;
        d[l].p1 += d[t].p1;
        into[t] = l;
        if (h.prev[l] >= 0) h.update(l, key_degrade(d[h.prev[l]], d[l], err));
        if (r >= 0) h.update(r, key_degrade(d[l], d[r], err));
    }
    std::vector<Letter> out;
    std::vector<int64_t> idx(n, -1);
    for (int64_t e = h.head(); e >= 0; e = h.next[e]) {
        idx[e] = (int64_t)out.size();
        out.push_back(d[e]);
    }
    if (grp) {
        grp->assign(n, -1);
        for (int64_t i = 0; i < n; ++i) {
            int64_t e = i;
            while (idx[e] < 0 && into[e] >= 0) e = into[e];
            (*grp)[i] = idx[e];
        }
    }
    return out;
}

// upgradedLeftRightProbs: the split of the centre letter onto its neighbours
bool upgraded_lr(const Letter& L_, const Letter& C, const Letter& R, Letter& ml, Letter& mr, Err& err) {
    const double piL = py_sum(L_), piC = py_sum(C), piR = py_sum(R);
    const double nL0 = L_.p0 / piL, nL1 = L_.p1 / piL;
    const double nC0 = C.p0 / piC, nC1 = C.p1 / piC;
    const double nR0 = R.p0 / piR, nR1 = R.p1 / piR;
    const bool zeroSide = nL0 < 0.5 && nR0 < 0.5;
    const bool oneSide = !zeroSide && nL1 < 0.5 && nR1 < 0.5;
    double dLR;
    if (zeroSide) dLR = 2.0 * (nL0 - nR0);
    else if (oneSide) dLR = 2.0 * (nR1 - nL1);
    else dLR = (nL0 - nL1) - (nR0 - nR1);
    if (!(dLR > 0.0)) {
        err.set(PCUB_EASSERT);
        return false;
    }
    double thL, thR;
    if (zeroSide) {
        if (nL0 - nC0 < nC0 - nR0) {
            thR = 2.0 * (nL0 - nC0) / dLR;
            thL = 1.0 - thR;
        } else {
            thL = 2.0 * (nC0 - nR0) / dLR;
            thR = 1.0 - thL;
        }
    } else if (oneSide) {
        if (nC1 - nL1 < nR1 - nC1) {
            thR = 2.0 * (nC1 - nL1) / dLR;
            thL = 1.0 - thR;
        } else {
            thL = 2.0 * (nR1 - nC1) / dLR;
            thR = 1.0 - thL;
        }
    } else {
        thR = ((nL0 - nL1) - (nC0 - nC1)) / dLR;
        thL = 1.0 - thR;
    }
    if (!(0.0 <= thL && thL <= 1.0 && 0.0 <= thR && thR <= 1.0)) {
        err.set(PCUB_EASSERT);
        return false;
    }
    ml = Letter{thL * piC * nL0, thL * piC * nL1};
    mr = Letter{thR * piC * nR0, thR * piC * nR1};
    return true;
}

double key_upgrade(const Letter& l, const Letter& c, const Letter& r, Err& err) {
    Letter ml, mr;
    if (!upgraded_lr(l, c, r, ml, mr, err)) return 0.0;
    return hxgiveny(c, err) - hxgiveny(ml, err) - hxgiveny(mr, err);
}

std::vector<Letter> upgrade_merged(const std::vector<Letter>& in, int64_t L, Err& err, std::vector<UpAux>* aux) {
    const int64_t n = (int64_t)in.size();
    std::vector<Letter> d = in;
    // auxiliary [left, centre, right] member lists per element (:368-401): a removed centre's
    // centre and right members join its left neighbour's right set, its centre and left
    // members its right neighbour's left set
    std::vector<UpAux> ax;
    if (aux) {
        ax.resize(n);
        for (int64_t i = 0; i < n; ++i) ax[i].c.push_back(i);
    }
    std::vector<double> keys(n);
    for (int64_t i = 0; i < n; ++i)
        keys[i] = (i == 0 || i == n - 1) ? kInf : key_upgrade(d[i - 1], d[i], d[i + 1], err);
    ListHeap h(keys);
    while (h.size() > L && !err.code) {
        const int64_t t = h.extract_min();
        const int64_t l = h.prev[t], r = h.next[t];
        if (l < 0 || r < 0) {
            err.set(PCUB_EATTR);
            break;
        }
        Letter ml, mr;
        if (!upgraded_lr(d[l], d[t], d[r], ml, mr, err)) break;
        d[l].p0 += ml.p0;
        d[r].p0 += mr.p0;
        d[l].p1 += ml.p1;
        d[r].p1 += mr.p1;
        if (aux) {
            UpAux& A = ax[t];
            std::vector<int64_t>& lr = ax[l].r;
            lr.insert(lr.end(), A.c.begin(), A.c.end());
            lr.insert(lr.end(), A.r.begin(), A.r.end());
            std::vector<int64_t>& rl = ax[r].l;
            rl.insert(rl.end(), A.c.begin(), A.c.end());
            rl.insert(rl.end(), A.l.begin(), A.l.end());
            A = UpAux();
        }
        if (h.prev[l] >= 0) h.update(l, key_upgrade(d[h.prev[l]], d[l], d[r], err));
        if (h.next[r] >= 0) h.update(r, key_upgrade(d[l], d[r], d[h.next[r]], err));
    }
    std::vector<Letter> out;
    if (aux) aux->clear();
    for (int64_t e = h.head(); e >= 0; e = h.next[e]) {
        out.push_back(d[e]);
        if (aux) aux->push_back(std::move(ax[e]));
    }
    return out;
}

std::vector<Letter> minus_t(const std::vector<Letter>& p) {
    std::vector<Letter> o;
    o.reserve(p.size() * p.size());
    for (const Letter& a : p)
        for (const Letter& b : p) o.push_back({a.p0 * b.p0 + a.p1 * b.p1, a.p0 * b.p1 + a.p1 * b.p0});
    return o;
}

std::vector<Letter> plus_t(const std::vector<Letter>& p) {
    std::vector<Letter> o;
    o.reserve(2 * p.size() * p.size());
    for (const Letter& a : p)
        for (const Letter& b : p) {
            o.push_back({a.p0 * b.p0, a.p1 * b.p1});
            o.push_back({a.p1 * b.p0, a.p0 * b.p1});
        }
    return o;
}

// dist.minusTransform().degrade(L) / .upgrade(L) (the transformed channel is merged first)
std::vector<Letter> child(const std::vector<Letter>& p, bool plus, bool up, int64_t L, Err& err) {
    std::vector<Letter> t = plus ? plus_t(p) : minus_t(p);
    merge_equivalent(t, nullptr, err);
    if (err.code) return {};
    return up ? upgrade_merged(t, L, err, nullptr) : degrade_merged(t, L, nullptr, err);
}

double error_prob(const std::vector<Letter>& p) {
    double s = 0.0;
    for (const Letter& l : p) s += (l.p1 < l.p0) ? l.p1 : l.p0;  // min([p0, p1])
    return s;
}

double total_variation(const std::vector<Letter>& p) {
    double s = 0.0;
    for (const Letter& l : p) s += fabs(l.p0 - l.p1);
    return s;
}

std::vector<Letter> load(const double* probs, int64_t n) {
    std::vector<Letter> p((size_t)n);
    for (int64_t i = 0; i < n; ++i) p[i] = Letter{probs[2 * i], probs[2 * i + 1]};
    return p;
}

void store(const std::vector<Letter>& p, double* out, int64_t* out_n) {
    for (size_t i = 0; i < p.size(); ++i) {
        out[2 * i] = p[i].p0;
        out[2 * i + 1] = p[i].p1;
    }
    *out_n = (int64_t)p.size();
}

// The polarisation tree of one channel: leaves in the reference's order (minus child
// first at every node), each level's 2^m children on `threads` workers.
int tree(std::vector<Letter> root, int n, int64_t L, bool up, int threads, double* vec, bool tv) {
    std::vector<std::vector<Letter>> lvl{std::move(root)};
    for (int m = 1; m <= n; ++m) {
        const size_t cnt = lvl.size() * 2;
        std::vector<std::vector<Letter>> nxt(cnt);
        std::vector<Err> errs(cnt);
        std::atomic<size_t> next_task{0};
        auto work = [&]() {
            for (size_t t; (t = next_task.fetch_add(1)) < cnt;) nxt[t] = child(lvl[t / 2], t & 1, up, L, errs[t]);
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
    for (size_t i = 0; i < lvl.size(); ++i) vec[i] = tv ? total_variation(lvl[i]) : error_prob(lvl[i]);
    return 0;
}

}  // namespace tv
}  // namespace pcub

using namespace pcub::tv;

extern "C" int pcub_bmd_merge_equivalent(const double* probs, int64_t n, double* out, int64_t* out_n,
                                         int64_t* group) {
    if (n < 0 || (n > 0 && (!probs || !out)) || !out_n) return PCUB_EINVAL;
    std::vector<Letter> p = load(probs, n);
    std::vector<int64_t> grp;
    Err err;
    merge_equivalent(p, group ? &grp : nullptr, err);
    if (err.code) return err.code;
    store(p, out, out_n);
    if (group) std::copy(grp.begin(), grp.end(), group);
    return 0;
}

extern "C" int pcub_bmd_degrade(const double* merged, int64_t n, int64_t L, double* out, int64_t* out_n,
                                int64_t* group) {
    if (n < 1 || L < 1 || !merged || !out || !out_n) return PCUB_EINVAL;
    std::vector<int64_t> grp;
    Err err;
    std::vector<Letter> o = degrade_merged(load(merged, n), L, group ? &grp : nullptr, err);
    if (err.code) return err.code;
    store(o, out, out_n);
    if (group) std::copy(grp.begin(), grp.end(), group);
    return 0;
}

extern "C" int pcub_bmd_upgrade(const double* merged, int64_t n, int64_t L, double* out, int64_t* out_n) {
    if (n < 1 || L < 1 || !merged || !out || !out_n) return PCUB_EINVAL;
    Err err;
    std::vector<Letter> o = upgrade_merged(load(merged, n), L, err, nullptr);
    if (err.code) return err.code;
    store(o, out, out_n);
    return 0;
}

extern "C" int pcub_bin_construct(int32_t n, int64_t L, const double* xprobs, int64_t nx, const double* xyprobs,
                                  int64_t nxy, double* TV, double* Pe, int32_t threads) {
    if (n < 0 || n > 24 || L < 1 || !xyprobs || nxy < 1 || !Pe || !TV || (xprobs && nx < 1)) return PCUB_EINVAL;
    if (threads < 1) threads = (int32_t)std::max(1u, std::thread::hardware_concurrency());
    const size_t N = (size_t)1 << n;
    if (xprobs) {
        const int rc = tree(load(xprobs, nx), n, L, true, threads, TV, true);
        if (rc) return rc;
    } else {
        std::fill(TV, TV + N, 0.0);
    }
    return tree(load(xyprobs, nxy), n, L, false, threads, Pe, false);
}
