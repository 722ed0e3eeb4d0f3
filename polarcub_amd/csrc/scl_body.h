// scl_body.h -- q-ary SCL / Fast-SSC list decoding of one codeword (host + device).
//
// Restates QaryPolarEncoderDecoder.listDecode / recursiveListDecode
// (QaryPolarEncoderDecoder.py:118-227, 403-757) with its helpers (:759-820), linear domain:
//   * general node: minus transform + sum-normalise of every path, recurse; plus transform of
//     each surviving path from its parent's vector (the minus recursion's index map), recurse;
//     combine x[2h] = (xm + xp) % q, x[2h+1] = (q - xp) % q                        (:684-757)
//   * information leaf: every path forks q ways, prob * m[s] with m the leaf marginal (p / sum,
//     or 1/q); candidates c = s * Lin + i                                            (:424-470)
//   * frozen leaf: prob * m[frozen value]                                            (:471-487)
//   * rate-0 node: encoding T(frozen values); prob * prod_j xy[j][enc_j]               (:494-518)
//   * repetition node (one information index k): q forks, encoding T(frozen values with s at
//     k); prob * prod_j xy[j][enc_j]                                                  (:520-578)
//   * rate-1 node: q^2 forks on the two least reliable positions (reliability = second largest
//     / largest of the row), every other position at its argmax; c = f + q^2 i;
//     prob = (p_a * p_b) * (cur * prod of the row maxima)                             (:580-628, 759-791)
//   * single-parity-check node (its first index taken as the frozen one): q^3 forks on three of
//     the four least reliable positions, the least reliable set by the parity (frozen value minus
//     the argmax symbols); prob = prod over the four * (cur * prod of the maxima)     (:630-682, 793-820)
//   * after every fork: when more than L candidates, keep the min(count_nonzero, L) largest;
//     then divide every metric by the largest (normalize, :867-872)
// with T = polarTransformOfQudits (:1136-1154), as the reference applies it.  Products run left
// to right in position order; sums of a row as Python's sum (0 + p0 + p1 + ...).
//
// Tie-breaking, the one deliberate difference.  The reference prunes with np.argpartition and
// picks the least reliable positions with np.argpartition; numpy 2.2 dispatches float64
// argpartition to x86-simd-sort where AVX-512 exists, so which of TIED candidates survive and in
// what order the kept paths are listed depend on the host CPU.  Here the
// kept paths are the largest metrics, ties to the lower candidate index, listed in ascending
// candidate order; the least reliable positions are the largest ratios, ties to the lower
// position, in ascending (ratio, -position) order (the last is the least reliable, as the
// reference's [-k:] slice of order statistics).  Without ties the surviving path SET and its
// metrics are the reference's.
//
// Log domain (use_log=True, SclArgs::log): rows are log-probabilities; the transforms use numpy's
// logaddexp and scipy's logsumexp normalisation (as sc_qary_log.hip), path metrics add, a prune
// keeps min(count of non -inf, L), normalize subtracts the largest, reliability is (second largest
// - largest), and each product becomes the sum the reference forms: np.sum over a node's positions
// (numpy's pairwise summation, np_sum_pow2), Python's sum over the row maxima and np.sum(axis=1)
// over a fork's selected entries (both left to right).  exp / log1p / log are the platform's, so
// log-domain values agree with the reference to a few ulps (the tests state the tolerance).
//
// One lane per codeword; all per-codeword state in a slab of 8-byte cells and a slab of bytes,
// element e at [e * ns] (slot-minor: a wave's lanes touch consecutive words).  The recursion's
// shape depends only on the frozen mask.  The actual information's path (listDecode's
// actualInformation) is tracked in path slot L: its distributions, encodings and actual_prob.
#pragma once
#include <math.h>
#include <stdint.h>

#include "sc_common.h"

// test instrumentation hooks (tests/emu/scl_emu.cpp counts slab traffic and frame-loop iterations)
#ifndef PCUB_SCL_TOUCH
#define PCUB_SCL_TOUCH(bytes)
#endif
#ifndef PCUB_SCL_FRAME
#define PCUB_SCL_FRAME()
#endif

namespace pcub {

struct SclArgs {
    const double* xy;        // [N][B][q] linear-domain rows
    long long B;
    int n, q, L, K;          // log2 N, alphabet, max list size, information symbols
    const uint8_t* frozen;   // [N] 1 = frozen
    const uint8_t* fvals;    // [nF][B] frozen values in frozen-index order
    int nF;
    const uint8_t* actual;   // [K][B] actual information, or null (no actual path)
    uint8_t* out_info;       // [L][K][B]
    double* out_prob;        // [L][B] final normalised path metrics
    int* out_size;           // [B] final list size
    double* out_actual;      // [B] actual_prob (when actual is given)
    int log;                 // 1: log-domain rows and metrics (use_log=True)
    double* cells;           // slab of 8-byte cells  [ncells][ns]
    uint8_t* bytes;          // slab of bytes         [nbytes][ns]
    long long ns;
};

// Slab layout.  Depth d >= 1 nodes have S = N >> d positions; P = L + 1 path slots.
struct SclLayout {
    int N, q, L, P, K, n;
    long long c_dist, c_prob, c_cand, c_flag, c_map, c_save, c_row, ncells;
    long long b_enc, b_info, b_tmp, nbytes;
    PCUB_HD void init(int n_, int q_, int L_, int K_) {
        n = n_;
        N = 1 << n;
        q = q_;
        L = L_;
        P = L + 1;
        K = K_ > 0 ? K_ : 1;
        const long long fork = (long long)L * q * q * q;
        c_dist = 0;                                 // depth d: P * S * q cells at P*q*(N - 2S)
        c_prob = c_dist + (long long)P * q * N;     // L metrics
        c_cand = c_prob + L;                        // candidate metrics (<= L q^3)
        c_flag = c_cand + fork;                     // candidate kept flags
        c_map = c_flag + fork;                      // per depth: L map entries (a node's output)
        c_save = c_map + (long long)(n + 1) * L;    // per depth: L saved minus maps
        c_row = c_save + (long long)(n + 1) * L;    // 4 rows of q cells (marginals) + N ratios + N maxima
        ncells = c_row + 4LL * q + 2LL * N;
        b_enc = 0;                                  // depth d >= 0: 2 sides x P x S bytes at 2P(2N - 2S)
        b_info = b_enc + 2LL * P * 2 * N;           // 2 buffers x L x K
        b_tmp = b_info + 2LL * L * K;               // q x N (splits) + 2 N (transform)
        nbytes = b_tmp + (long long)q * N + 2LL * N + 8;
    }
    PCUB_HD long long dist(int d, int slot, int pos, int x) const {
        const int S = N >> d;
        return c_dist + (long long)P * q * (N - 2 * S) + ((long long)slot * S + pos) * q + x;
    }
    PCUB_HD long long enc(int d, int side, int slot, int pos) const {
        const int S = N >> d;
        return b_enc + 2LL * P * (2 * N - 2 * S) + ((long long)side * P + slot) * S + pos;
    }
    PCUB_HD long long info(int buf, int l, int k) const { return b_info + ((long long)buf * L + l) * K + k; }
};

struct SclCtx {
    const SclArgs* A;
    SclLayout Y;
    long long cw;
    double* cells;   // this lane's slab base (element e at cells[e * ns])
    uint8_t* bytes;
    long long ns;
    int fi;          // next frozen value
    int buf;         // current information buffer
    bool track;      // actual path present
    bool lg;         // log domain
    double actual_prob;

    PCUB_HD double& C(long long e) {
        PCUB_SCL_TOUCH(8);
        return cells[e * ns];
    }
    PCUB_HD uint8_t& Bt(long long e) {
        PCUB_SCL_TOUCH(1);
        return bytes[e * ns];
    }
    // row element of path slot `slot` at depth d (depth 0: the channel input, shared)
    PCUB_HD double row(int d, int slot, int pos, int x) {
        if (d == 0) return A->xy[((long long)pos * A->B + cw) * Y.q + x];
        return C(Y.dist(d, slot, pos, x));
    }
    PCUB_HD int frozen_value() { return (int)A->fvals[(long long)(fi++) * A->B + cw]; }
    PCUB_HD int actual_sym(int ii) { return (int)A->actual[(long long)ii * A->B + cw]; }
};

constexpr double kSclLn2 = 0.693147180559945309417232121458176568;

// numpy's npy_logaddexp
PCUB_HD double scl_logaddexp(double x, double y) {
    if (x == y) return x + kSclLn2;
    const double t = x - y;
    if (t > 0) return x + log1p(exp(-t));
    if (t <= 0) return y + log1p(exp(t));
    return t;  // NaN
}

// scipy 1.15's logsumexp of q <= 8 values (every maximal element taken out of the sum), as
// sc_qary_log.hip
PCUB_HD double scl_logsumexp(const double* p, int q) {
    double mx = p[0];
    for (int x = 1; x < q; ++x) mx = p[x] > mx ? p[x] : mx;
    double m = 0.0;
    for (int x = 0; x < q; ++x) m += (p[x] == mx) ? 1.0 : 0.0;
    const double shift = isfinite(mx) ? mx : 0.0;
    double rest = 0.0;
    for (int x = 1; x < q; ++x) rest += (p[x] == mx) ? 0.0 : exp(p[x] - shift);
    double s = ((p[0] == mx) ? 0.0 : exp(p[0] - shift)) + rest;
    if (s != 0.0) s = s / m;
    return log1p(s) + log(m) + mx;
}

// metric (x) factor: product, or sum in the log domain
PCUB_HD double scl_mul(const SclCtx& c, double p, double f) { return c.lg ? p + f : p * f; }

// actual_prob update by a factor v and a normalisation weight w (:467-470)
PCUB_HD void scl_scale_actual(SclCtx& c, double v, double w) {
    if (c.lg) c.actual_prob += v - w;
    else c.actual_prob *= v / w;
}

// leaf marginal of a length-1 row into C(c_row + off .. + q)
PCUB_HD void scl_marginal(SclCtx& c, int d, int slot, long long off) {
    const int q = c.Y.q;
    if (c.lg) {
        double r[8];
        for (int x = 0; x < q; ++x) r[x] = c.row(d, slot, 0, x);
        const double s = scl_logsumexp(r, q);
        for (int x = 0; x < q; ++x) c.C(off + x) = s > -INFINITY ? r[x] - s : -log((double)q);
        return;
    }
    double s = 0.0;
    for (int x = 0; x < q; ++x) s = s + c.row(d, slot, 0, x);
    for (int x = 0; x < q; ++x) c.C(off + x) = s > 0.0 ? c.row(d, slot, 0, x) / s : 1.0 / q;
}

// polarTransformOfQudits of v[0..S) (bytes at b) into out[0..S) (bytes at o); tmp at t (S bytes)
PCUB_HD void scl_polar(SclCtx& c, long long b, long long o, long long t, int S) {
    const int q = c.Y.q;
    for (int i = 0; i < S; ++i) c.Bt(o + i) = c.Bt(b + i);
    // each stage splits every block of m into [pair sums | negated odd], then recurses per half
    for (int m = S; m > 1; m >>= 1) {
        for (int blk = 0; blk < S; blk += m) {
            for (int i = 0; i < m / 2; ++i) {
                const int a = c.Bt(o + blk + 2 * i), bb = c.Bt(o + blk + 2 * i + 1);
                c.Bt(t + i) = (uint8_t)((a + bb) % q);
                c.Bt(t + m / 2 + i) = (uint8_t)((q - bb) % q);
            }
            for (int i = 0; i < m; ++i) c.Bt(o + blk + i) = c.Bt(t + i);
        }
    }
}

// keep the largest metrics among n candidates (ties: lower index), at most L; flags in c_flag;
// returns the kept count
PCUB_HD int scl_prune(SclCtx& c, int ncand) {
    const int L = c.Y.L;
    for (int i = 0; i < ncand; ++i) c.C(c.Y.c_flag + i) = 0.0;
    if (ncand <= L) {
        for (int i = 0; i < ncand; ++i) c.C(c.Y.c_flag + i) = 1.0;
        return ncand;
    }
    int nz = 0;  // count_nonzero, or the count of entries that are not -inf (log domain)
    const double zero = c.lg ? -INFINITY : 0.0;
    for (int i = 0; i < ncand; ++i) nz += c.C(c.Y.c_cand + i) != zero;
    // (all candidates zero: the reference fails on the empty list; keep the first one)
    const int keep = nz < L ? (nz > 0 ? nz : 1) : L;
    for (int r = 0; r < keep; ++r) {
        int best = -1;
        double bv = 0.0;
        for (int i = 0; i < ncand; ++i) {
            if (c.C(c.Y.c_flag + i) != 0.0) continue;
            const double v = c.C(c.Y.c_cand + i);
            if (best < 0 || v > bv) {
                best = i;
                bv = v;
            }
        }
        c.C(c.Y.c_flag + best) = 1.0;
    }
    return keep;
}

// divide the kept metrics (compacted into c_prob[0..k)) by their maximum; returns it
PCUB_HD double scl_normalize(SclCtx& c, int k) {
    double mx = c.C(c.Y.c_prob);
    for (int i = 1; i < k; ++i) mx = c.C(c.Y.c_prob + i) > mx ? c.C(c.Y.c_prob + i) : mx;
    for (int i = 0; i < k; ++i) c.C(c.Y.c_prob + i) = c.lg ? c.C(c.Y.c_prob + i) - mx : c.C(c.Y.c_prob + i) / mx;
    return mx;
}

// second largest / largest of a row (np.partition(probs, -2)[-2:])
PCUB_HD double scl_ratio(SclCtx& c, int d, int slot, int pos) {
    const int q = c.Y.q;
    double a = c.row(d, slot, pos, 0), b = c.row(d, slot, pos, 1);
    double hi = a > b ? a : b, lo = a > b ? b : a;
    for (int x = 2; x < q; ++x) {
        const double v = c.row(d, slot, pos, x);
        if (v > hi) {
            lo = hi;
            hi = v;
        } else if (v > lo) {
            lo = v;
        }
    }
    return c.lg ? lo - hi : lo / hi;
}

PCUB_HD int scl_argmax(SclCtx& c, int d, int slot, int pos, double* mx) {
    int arg = 0;
    double best = c.row(d, slot, pos, 0);
    for (int x = 1; x < c.Y.q; ++x) {
        const double v = c.row(d, slot, pos, x);
        if (v > best) {
            best = v;
            arg = x;
        }
    }
    *mx = best;
    return arg;
}

// the k least reliable positions of a node row set (largest ratios; ties to the lower position),
// ascending (ratio, -position) into idx[0..k)
PCUB_HD void scl_least_reliable(SclCtx& c, int d, int slot, int S, int k, int* idx) {
    for (int p = 0; p < S; ++p) c.C(c.Y.c_row + 4 * c.Y.q + p) = scl_ratio(c, d, slot, p);
    int taken = 0;
    for (int r = k - 1; r >= 0; --r) {  // pick the least reliable first: it goes last
        int best = -1;
        double bv = 0.0;
        for (int p = 0; p < S; ++p) {
            bool used = false;
            for (int t = 0; t < taken; ++t) used = used || idx[k - 1 - t] == p;
            if (used) continue;
            const double v = c.C(c.Y.c_row + 4 * c.Y.q + p);
            if (best < 0 || v > bv) {
                best = p;
                bv = v;
            }
        }
        idx[r] = best;
        ++taken;
    }
}

// copy the kept candidates' metrics into c_prob (ascending candidate order), fill the
// information rows of the next buffer from their origin paths (candidate / div when div > 0,
// else candidate % lin), return the kept count
PCUB_HD int scl_commit(SclCtx& c, int ncand, int ii, int div, int lin, int* origin) {
    int k = 0;
    for (int i = 0; i < ncand; ++i)
        if (c.C(c.Y.c_flag + i) != 0.0) {
            origin[k] = i;
            ++k;
        }
    for (int r = 0; r < k; ++r) c.C(c.Y.c_prob + r) = c.C(c.Y.c_cand + origin[r]);
    const int nb = c.buf ^ 1;
    for (int r = 0; r < k; ++r) {
        const int from = div > 0 ? origin[r] / div : origin[r] % lin;
        for (int j = 0; j < ii; ++j) c.Bt(c.Y.info(nb, r, j)) = c.Bt(c.Y.info(c.buf, from, j));
    }
    c.buf = nb;
    return k;
}

// numpy's pairwise sum (the add reduction's inner loop) of positions [off, off + n), n <= 128,
// of row_j[enc_j]
PCUB_HD double scl_np_block(SclCtx& c, int d, int slot, long long e, int off, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += c.row(d, slot, off + i, c.Bt(e + off + i));
        return r;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = c.row(d, slot, off + j, c.Bt(e + off + j));
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += c.row(d, slot, off + i + j, c.Bt(e + off + i + j));
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += c.row(d, slot, off + i, c.Bt(e + off + i));
    return res;
}

// np.sum of row_j[enc_j] over the S (a power of two) positions of a node: numpy halves blocks
// longer than 128 (n2 = n/2 - (n/2) % 8 = n/2 here) and sums the halves, so the 128-blocks combine
// in a balanced binary tree, left + right (a carry chain over the block index)
PCUB_HD double scl_np_sum_pow2(SclCtx& c, int d, int slot, int S, long long e) {
    if (S <= 128) return scl_np_block(c, d, slot, e, 0, S);
    double acc[6];
    const int nb = S / 128;
    for (int b = 0; b < nb; ++b) {
        double v = scl_np_block(c, d, slot, e, b * 128, 128);
        int lvl = 0;
        for (; (b >> lvl) & 1; ++lvl) v = acc[lvl] + v;
        acc[lvl] = v;
    }
    int top = 0;
    while ((1 << top) < nb) ++top;
    return acc[top];
}

// product over the S positions of a node of row_j[enc_j] (enc bytes at e), left to right
// (np.product); the log domain's np.sum
PCUB_HD double scl_prod_enc(SclCtx& c, int d, int slot, int S, long long e) {
    if (c.lg) return scl_np_sum_pow2(c, d, slot, S, e);
    double p = c.row(d, slot, 0, c.Bt(e));
    for (int j = 1; j < S; ++j) p = p * c.row(d, slot, j, c.Bt(e + j));
    return p;
}

// Number of information indices among u0 .. u0 + S - 1.
PCUB_HD int scl_nin(const SclCtx& c, int u0, int S) {
    int nin = 0;
    for (int j = 0; j < S; ++j) nin += c.A->frozen[u0 + j] == 0;
    return nin;
}

// A node the reference decodes without recursing (:424-682): information / frozen leaf, rate-0,
// repetition, rate-1, single parity check.  Decodes the node at depth d covering u indices
// [u0, u0 + N >> d), information index ii, from the Lin input paths (their vectors at depth d,
// slots 0..Lin-1); writes the output encodings at enc(d, side, r, .) and the map (output path
// -> input path) at c_map + d*L; returns the output list size.
PCUB_HD int scl_special(SclCtx& c, int d, int u0, int ii, int side, int Lin, int nin, int* origin) {
    const SclLayout& Y = c.Y;
    const int q = Y.q, L = Y.L, S = Y.N >> d;
    const long long mapo = Y.c_map + (long long)d * L;
        if (S == 1) {
            if (nin == 1) {  // information leaf: q forks per path
                for (int i = 0; i < Lin; ++i) {
                    scl_marginal(c, d, i, Y.c_row);
                    for (int s = 0; s < q; ++s)
                        c.C(Y.c_cand + s * Lin + i) = scl_mul(c, c.C(Y.c_prob + i), c.C(Y.c_row + s));
                }
                const int nc = Lin * q;
                scl_prune(c, nc);
                const int k = scl_commit(c, nc, ii, 0, Lin, origin);
                for (int r = 0; r < k; ++r) {
                    const int i = origin[r] % Lin, s = origin[r] / Lin;
                    c.Bt(Y.info(c.buf, r, ii)) = (uint8_t)s;
                    c.Bt(Y.enc(d, side, r, 0)) = (uint8_t)s;
                    c.C(mapo + r) = (double)i;
                }
                const double w = scl_normalize(c, k);
                if (c.track) {
                    const int a = c.actual_sym(ii);
                    scl_marginal(c, d, L, Y.c_row);
                    scl_scale_actual(c, c.C(Y.c_row + a), w);
                    c.Bt(Y.enc(d, side, L, 0)) = (uint8_t)a;
                }
                return k;
            }
            const int fv = c.frozen_value();  // frozen leaf
            for (int i = 0; i < Lin; ++i) {
                scl_marginal(c, d, i, Y.c_row);
                c.C(Y.c_prob + i) = scl_mul(c, c.C(Y.c_prob + i), c.C(Y.c_row + fv));
                c.Bt(Y.enc(d, side, i, 0)) = (uint8_t)fv;
                c.C(mapo + i) = (double)i;
            }
            const double w = scl_normalize(c, Lin);
            if (c.track) {
                scl_marginal(c, d, L, Y.c_row);
                scl_scale_actual(c, c.C(Y.c_row + fv), w);
                c.Bt(Y.enc(d, side, L, 0)) = (uint8_t)fv;
            }
            return Lin;
        }

        const long long tv = Y.b_tmp;                       // S bytes: a vector
        const long long tt = Y.b_tmp + (long long)q * Y.N;  // S bytes: transform temp
        const long long to = tt + Y.N;                      // S bytes: transform out
        if (nin == 0) {  // rate-0
            for (int j = 0; j < S; ++j) c.Bt(tv + j) = (uint8_t)c.frozen_value();
            scl_polar(c, tv, to, tt, S);
            for (int i = 0; i < Lin; ++i) {
                c.C(Y.c_prob + i) = scl_mul(c, c.C(Y.c_prob + i), scl_prod_enc(c, d, i, S, to));
                for (int j = 0; j < S; ++j) c.Bt(Y.enc(d, side, i, j)) = c.Bt(to + j);
                c.C(mapo + i) = (double)i;
            }
            const double w = scl_normalize(c, Lin);
            if (c.track) {
                scl_scale_actual(c, scl_prod_enc(c, d, L, S, to), w);
                for (int j = 0; j < S; ++j) c.Bt(Y.enc(d, side, L, j)) = c.Bt(to + j);
            }
            return Lin;
        }
        if (nin == 1) {  // repetition: encodings of the q splits at b_tmp + s*N
            int kpos = 0;
            for (int j = 0; j < S; ++j)
                if (c.A->frozen[u0 + j] == 0) kpos = j;
            for (int j = 0; j < S; ++j) c.Bt(tv + j) = (uint8_t)(j == kpos ? 0 : c.frozen_value());
            for (int s = q - 1; s >= 0; --s) {  // split s at b_tmp + s*N (s = 0 last: tv is its input)
                c.Bt(tv + kpos) = (uint8_t)s;
                scl_polar(c, tv, to, tt, S);
                for (int j = 0; j < S; ++j) c.Bt(Y.b_tmp + (long long)s * Y.N + j) = c.Bt(to + j);
            }
            for (int i = 0; i < Lin; ++i)
                for (int s = 0; s < q; ++s)
                    c.C(Y.c_cand + s * Lin + i) =
                        scl_mul(c, c.C(Y.c_prob + i), scl_prod_enc(c, d, i, S, Y.b_tmp + (long long)s * Y.N));
            const int nc = Lin * q;
            scl_prune(c, nc);
            const int k = scl_commit(c, nc, ii, 0, Lin, origin);
            for (int r = 0; r < k; ++r) {
                const int i = origin[r] % Lin, s = origin[r] / Lin;
                c.Bt(Y.info(c.buf, r, ii)) = (uint8_t)s;
                for (int j = 0; j < S; ++j) c.Bt(Y.enc(d, side, r, j)) = c.Bt(Y.b_tmp + (long long)s * Y.N + j);
                c.C(mapo + r) = (double)i;
            }
            const double w = scl_normalize(c, k);
            if (c.track) {
                const int a = c.actual_sym(ii);
                scl_scale_actual(c, scl_prod_enc(c, d, L, S, Y.b_tmp + (long long)a * Y.N), w);
                for (int j = 0; j < S; ++j) c.Bt(Y.enc(d, side, L, j)) = c.Bt(Y.b_tmp + (long long)a * Y.N + j);
            }
            return k;
        }
        if (nin == S || nin == S - 1) {  // rate-1 (q^2 forks) / single parity check (q^3 forks)
            const bool spc = nin == S - 1;
            const int nfork_idx = spc ? 3 : 2;
            const int nsel = spc ? 4 : 2;
            int fork = q * q;
            if (spc) fork *= q;
            const int fv = spc ? c.frozen_value() : 0;
            for (int i = 0; i < Lin; ++i) {
                int idx[4];
                scl_least_reliable(c, d, i, S, nsel, idx);
                // constant positions: argmax symbol and product of maxima, in position order
                double base = c.C(Y.c_prob + i), pm = 1.0;
                bool first = true;
                int csum = 0;
                for (int j = 0; j < S; ++j) {
                    bool sel = false;
                    for (int t = 0; t < nsel; ++t) sel = sel || idx[t] == j;
                    if (sel) continue;
                    double mx;
                    csum += scl_argmax(c, d, i, j, &mx);
                    pm = first ? mx : (c.lg ? pm + mx : pm * mx);  // Python's sum from 0 / np.product
                    first = false;
                }
                base = c.lg ? base + (first ? 0.0 : pm) : (first ? base * 1.0 : base * pm);
                const int delta = ((fv - csum) % q + q) % q;
                for (int f = 0; f < fork; ++f) {
                    int sym[4];
                    int rem = f, ssum = 0;
                    for (int t = nfork_idx - 1; t >= 0; --t) {
                        sym[t] = rem % q;
                        rem /= q;
                        ssum += sym[t];
                    }
                    if (spc) sym[3] = ((delta - ssum) % q + q) % q;
                    double p = c.row(d, i, idx[0], sym[0]);
                    for (int t = 1; t < nsel; ++t) p = scl_mul(c, p, c.row(d, i, idx[t], sym[t]));
                    c.C(Y.c_cand + (long long)fork * i + f) = c.lg ? p + base : p * base;
                }
            }
            const int nc = Lin * fork;
            scl_prune(c, nc);
            const int k = scl_commit(c, nc, ii, fork, Lin, origin);
            const long long xv = Y.b_tmp;  // the fork's codeword part, then its transform
            for (int r = 0; r < k; ++r) {
                const int i = origin[r] / fork, f = origin[r] % fork;
                int idx[4];
                scl_least_reliable(c, d, i, S, nsel, idx);
                int csum = 0;
                for (int j = 0; j < S; ++j) {
                    double mx;
                    const int a = scl_argmax(c, d, i, j, &mx);
                    c.Bt(xv + j) = (uint8_t)a;
                    bool sel = false;
                    for (int t = 0; t < nsel; ++t) sel = sel || idx[t] == j;
                    if (!sel) csum += a;
                }
                const int delta = ((fv - csum) % q + q) % q;
                int rem = f, ssum = 0;
                for (int t = nfork_idx - 1; t >= 0; --t) {
                    const int sv = rem % q;
                    rem /= q;
                    ssum += sv;
                    c.Bt(xv + idx[t]) = (uint8_t)sv;
                }
                if (spc) c.Bt(xv + idx[3]) = (uint8_t)(((delta - ssum) % q + q) % q);
                for (int j = 0; j < S; ++j) c.Bt(Y.enc(d, side, r, j)) = c.Bt(xv + j);
                scl_polar(c, xv, to, tt, S);
                const int off = spc ? 1 : 0;
                for (int j = 0; j + off < S; ++j) c.Bt(Y.info(c.buf, r, ii + j)) = c.Bt(to + off + j);
                c.C(mapo + r) = (double)i;
            }
            const double w = scl_normalize(c, k);
            if (c.track) {
                // T(actual information of the node) (T([frozen value] + information) for SPC)
                for (int j = 0; j < S; ++j) {
                    const int src = spc ? j - 1 : j;
                    c.Bt(tv + j) = (uint8_t)(src < 0 ? fv : c.actual_sym(ii + src));
                }
                scl_polar(c, tv, to, tt, S);
                scl_scale_actual(c, scl_prod_enc(c, d, L, S, to), w);
                for (int j = 0; j < S; ++j) c.Bt(Y.enc(d, side, L, j)) = c.Bt(to + j);
            }
            return k;
        }

    return -1;  // not reached: the caller sends only special nodes here
}

PCUB_HD bool scl_is_special(int S, int nin) { return S == 1 || nin <= 1 || nin >= S - 1; }

// log-domain normalise (t = logsumexp; if t != -inf: p - t) and store a row at depth d
PCUB_HD void scl_store_log(SclCtx& c, int d, int slot, int h, const double* o) {
    const int q = c.Y.q;
    const double t = scl_logsumexp(o, q);
    for (int u = 0; u < q; ++u) c.C(c.Y.dist(d, slot, h, u)) = t != -INFINITY ? o[u] - t : o[u];
}

// General node, before its minus child (:684-700): the minus transform + sum-normalise of every
// path's vector (and the actual path's) into depth d + 1.
PCUB_HD void scl_minus(SclCtx& c, int d, int slot_in, int slot_out) {
    const SclLayout& Y = c.Y;
    const int q = Y.q, H = (Y.N >> d) / 2;
    for (int h = 0; h < H; ++h) {
        double o[8];
        if (c.lg) {
            for (int u = 0; u < q; ++u) o[u] = -INFINITY;
            for (int x1 = 0; x1 < q; ++x1)
                for (int x2 = 0; x2 < q; ++x2) {
                    const int u = (x1 + x2) % q;
                    o[u] = scl_logaddexp(o[u], c.row(d, slot_in, 2 * h, x1) + c.row(d, slot_in, 2 * h + 1, x2));
                }
            scl_store_log(c, d + 1, slot_out, h, o);
            continue;
        }
        for (int u = 0; u < q; ++u) o[u] = 0.0;
        for (int x1 = 0; x1 < q; ++x1)
            for (int x2 = 0; x2 < q; ++x2) {
                const int u = (x1 + x2) % q;
                o[u] = o[u] + c.row(d, slot_in, 2 * h, x1) * c.row(d, slot_in, 2 * h + 1, x2);
            }
        double t = 0.0;
        for (int u = 0; u < q; ++u) t = t + o[u];
        for (int u = 0; u < q; ++u) c.C(Y.dist(d + 1, slot_out, h, u)) = t != 0.0 ? o[u] / t : o[u];
    }
}

// General node, between its children (:701-730): the plus transform of a surviving path from
// its parent's vector given the minus child's encoding at encm.
PCUB_HD void scl_plus(SclCtx& c, int d, int slot_in, int slot_out, long long encm) {
    const SclLayout& Y = c.Y;
    const int q = Y.q, H = (Y.N >> d) / 2;
    for (int h = 0; h < H; ++h) {
        const int u1 = c.Bt(encm + h);
        double o[8];
        if (c.lg) {
            for (int u2 = 0; u2 < q; ++u2)
                o[u2] = scl_logaddexp(-INFINITY, c.row(d, slot_in, 2 * h, (u1 + u2) % q) +
                                                     c.row(d, slot_in, 2 * h + 1, (q - u2) % q));
            scl_store_log(c, d + 1, slot_out, h, o);
            continue;
        }
        for (int u2 = 0; u2 < q; ++u2)
            o[u2] = 0.0 + c.row(d, slot_in, 2 * h, (u1 + u2) % q) * c.row(d, slot_in, 2 * h + 1, (q - u2) % q);
        double t = 0.0;
        for (int u = 0; u < q; ++u) t = t + o[u];
        for (int u = 0; u < q; ++u) c.C(Y.dist(d + 1, slot_out, h, u)) = t != 0.0 ? o[u] / t : o[u];
    }
}

// General node, after its plus child returned Lp paths (:731-757): combine x[2h] = xm + xp,
// x[2h+1] = -xp (mod q) from each output path's minus-side ancestor, and compose the maps.
PCUB_HD void scl_combine(SclCtx& c, int d, int side, int Lp, int* origin) {
    const SclLayout& Y = c.Y;
    const int q = Y.q, L = Y.L, H = (Y.N >> d) / 2;
    const long long mapo = Y.c_map + (long long)d * L;
    const long long save = Y.c_save + (long long)d * L;
    const long long mapm = Y.c_map + (long long)(d + 1) * L;
    for (int r = 0; r < Lp; ++r) {
        const int mi = (int)c.C(mapm + r);
        for (int h = 0; h < H; ++h) {
            const int xm = c.Bt(Y.enc(d + 1, 0, mi, h)), xp = c.Bt(Y.enc(d + 1, 1, r, h));
            c.Bt(Y.enc(d, side, r, 2 * h)) = (uint8_t)((xm + xp) % q);
            c.Bt(Y.enc(d, side, r, 2 * h + 1)) = (uint8_t)((q - xp) % q);
        }
        origin[r] = (int)c.C(save + mi);
    }
    for (int r = 0; r < Lp; ++r) c.C(mapo + r) = (double)origin[r];
    if (c.track)
        for (int h = 0; h < H; ++h) {
            const int xm = c.Bt(Y.enc(d + 1, 0, L, h)), xp = c.Bt(Y.enc(d + 1, 1, L, h));
            c.Bt(Y.enc(d, side, L, 2 * h)) = (uint8_t)((xm + xp) % q);
            c.Bt(Y.enc(d, side, L, 2 * h + 1)) = (uint8_t)((q - xp) % q);
        }
}

// The recursion of recursiveListDecode (:403-757) as a loop over an explicit frame stack (one
// frame per depth, at most log2 N + 1 live): no device function calls itself, so the kernel has
// a fixed private segment and no dynamic stack (scripts/check_isa.py rejects one).  A frame's
// phase says which child it waits for.  Returns the final list size.
constexpr int kSclMaxDepth = 13;  // log2 N <= 12

struct SclFrame {
    int d, u0, ii, side, Lin, phase;
};

PCUB_HD int scl_run(SclCtx& c) {
    const SclLayout& Y = c.Y;
    const int L = Y.L;
    SclFrame st[kSclMaxDepth];
    int origin[64];
    int sp = 0, ret = 0;
    st[0] = SclFrame{0, 0, 0, 0, 1, 0};
    while (sp >= 0) {
        PCUB_SCL_FRAME();
        SclFrame& f = st[sp];
        const int S = Y.N >> f.d, H = S / 2;
        if (f.phase == 0) {
            const int nin = scl_nin(c, f.u0, S);
            if (scl_is_special(S, nin)) {
                ret = scl_special(c, f.d, f.u0, f.ii, f.side, f.Lin, nin, origin);
                --sp;
                continue;
            }
            for (int i = 0; i < f.Lin; ++i) scl_minus(c, f.d, f.d == 0 ? 0 : i, i);
            if (c.track) scl_minus(c, f.d, f.d == 0 ? 0 : L, L);
            f.phase = 1;
            st[sp + 1] = SclFrame{f.d + 1, f.u0, f.ii, 0, f.Lin, 0};
            ++sp;
        } else if (f.phase == 1) {
            const int Lm = ret;
            const long long save = Y.c_save + (long long)f.d * L;
            const long long mapm = Y.c_map + (long long)(f.d + 1) * L;
            for (int r = 0; r < Lm; ++r) c.C(save + r) = c.C(mapm + r);
            const int iim = f.ii + scl_nin(c, f.u0, H);
            for (int r = 0; r < Lm; ++r) scl_plus(c, f.d, f.d == 0 ? 0 : (int)c.C(save + r), r, Y.enc(f.d + 1, 0, r, 0));
            if (c.track) scl_plus(c, f.d, f.d == 0 ? 0 : L, L, Y.enc(f.d + 1, 0, L, 0));
            f.phase = 2;
            st[sp + 1] = SclFrame{f.d + 1, f.u0 + H, iim, 1, Lm, 0};
            ++sp;
        } else {
            scl_combine(c, f.d, f.side, ret, origin);  // ret = the plus child's list size = this node's
            --sp;
        }
    }
    return ret;
}

// decode codeword cw with slab slot `slot`; store = false for padding lanes.  The slab is
// slot-minor (element e of slot s at [e * ns + s]).
PCUB_HD void scl_decode_cw(const SclArgs& A, long long cw, long long slot, bool store) {
    SclCtx c;
    c.A = &A;
    c.Y.init(A.n, A.q, A.L, A.K);
    c.cw = cw;
    c.cells = A.cells + slot;
    c.bytes = A.bytes + slot;
    c.ns = A.ns;
    c.fi = 0;
    c.buf = 0;
    c.track = A.actual != nullptr;
    c.lg = A.log != 0;
    c.actual_prob = c.lg ? 0.0 : 1.0;
    c.C(c.Y.c_prob) = c.lg ? 0.0 : 1.0;
    const int k = scl_run(c);
    if (!store) return;
    const long long B = A.B;
    A.out_size[cw] = k;
    for (int r = 0; r < A.L; ++r) {
        A.out_prob[(long long)r * B + cw] = r < k ? c.C(c.Y.c_prob + r) : 0.0;
        for (int j = 0; j < A.K; ++j)
            A.out_info[((long long)r * A.K + j) * B + cw] = r < k ? c.Bt(c.Y.info(c.buf, r, j)) : (uint8_t)0xff;
    }
    if (c.track && A.out_actual) A.out_actual[cw] = c.actual_prob;
}

}  // namespace pcub
