"""CPU restatement of the reference's q-ary list decoder -- TEST INFRASTRUCTURE ONLY.

Follows QaryPolarEncoderDecoder.recursiveListDecode (QaryPolarEncoderDecoder.py:403-757) node by
node -- leaves :423-490, rate-0 :494-518, repetition :520-578, rate-1 :580-628, single parity
check :630-682, general node :684-757, helpers :759-820, normalize :867-872,
polarTransformOfQudits :1136-1154 -- in plain Python floats (products left to right, row sums
as Python's sum), with the tie rules of polarcub_amd/csrc/scl_body.h in place of np.argpartition:
kept paths = the largest metrics, ties to the lower candidate index, listed in ascending candidate
order; least reliable positions = the largest (second largest / largest) ratios, ties to the
lower position, in ascending (ratio, -position) order.  numpy's float64 argpartition dispatches
to x86-simd-sort where AVX-512 exists, so the reference's own choice among ties and its list order
depend on the CPU; on inputs without ties this restatement keeps the reference's path SET and
metrics, which tests/test_scl.py pins against runs of the reference itself (tests/golden/scl.npz).

use_log=True (the reference's log domain, recursiveListDecode's use_log branches): rows are
log-probabilities; transforms by numpy's logaddexp and scipy's logsumexp normalisation
(VectorDistributions/QaryMemorylessVectorDistribution.py:31-118), path metrics add, a prune keeps
min(count of finite-or-NaN, L), normalize subtracts the largest, reliability is (second largest -
largest), and the products become numpy / Python sums in the reference's orders: np.sum over a
node's positions (numpy's pairwise summation), Python's sum over the row maxima, and the fork
combinations' np.sum(axis=1) (left to right).

Only tests/ use this module.
"""
import math

import numpy as np
from scipy.special import logsumexp


def polar_qudits(q, x):
    """polarTransformOfQudits (QaryPolarEncoderDecoder.py:1136-1154)."""
    x = [int(v) for v in x]
    if len(x) == 1:
        return x
    first = [(x[2 * i] + x[2 * i + 1]) % q for i in range(len(x) // 2)]
    second = [(q - x[2 * i + 1]) % q for i in range(len(x) // 2)]
    return polar_qudits(q, first) + polar_qudits(q, second)


def _psum(row):
    s = 0
    for v in row:
        s = s + v
    return s


def _prod(vals):
    p = vals[0]
    for v in vals[1:]:
        p = p * v
    return p


def _normalize_rows(rows):
    out = []
    for r in rows:
        t = _psum(r)
        out.append([v / t for v in r] if t != 0 else list(r))
    return out


def _minus(rows, q):
    out = []
    for h in range(len(rows) // 2):
        a, b = rows[2 * h], rows[2 * h + 1]
        o = [0.0] * q
        for x1 in range(q):
            for x2 in range(q):
                o[(x1 + x2) % q] = o[(x1 + x2) % q] + a[x1] * b[x2]
        out.append(o)
    return _normalize_rows(out)


def _plus(rows, enc, q):
    out = []
    for h in range(len(rows) // 2):
        a, b, u1 = rows[2 * h], rows[2 * h + 1], int(enc[h])
        out.append([0.0 + a[(u1 + u2) % q] * b[(q - u2) % q] for u2 in range(q)])
    return _normalize_rows(out)


def _marginal(row, q):
    s = _psum(row)
    return [v / s for v in row] if s > 0.0 else [1 / q] * q


def _lae(x, y):
    return float(np.logaddexp(np.float64(x), np.float64(y)))


def _lse(row):
    return float(logsumexp(np.array(row, np.float64)))


def _normalize_rows_log(rows):
    out = []
    for r in rows:
        t = _lse(r)
        out.append([v - t for v in r] if t != -math.inf else list(r))
    return out


def _minus_log(rows, q):
    out = []
    for h in range(len(rows) // 2):
        a, b = rows[2 * h], rows[2 * h + 1]
        o = [-math.inf] * q
        for x1 in range(q):
            for x2 in range(q):
                o[(x1 + x2) % q] = _lae(o[(x1 + x2) % q], a[x1] + b[x2])
        out.append(o)
    return _normalize_rows_log(out)


def _plus_log(rows, enc, q):
    out = []
    for h in range(len(rows) // 2):
        a, b, u1 = rows[2 * h], rows[2 * h + 1], int(enc[h])
        out.append([_lae(-math.inf, a[(u1 + u2) % q] + b[(q - u2) % q]) for u2 in range(q)])
    return _normalize_rows_log(out)


def _marginal_log(row, q):
    s = _lse(row)
    return [v - s for v in row] if s > -math.inf else [-math.log(q)] * q


def _npsum(vals):
    """np.sum of a list of floats (numpy's pairwise summation)"""
    return float(np.sum(np.array(vals, np.float64)))


def _rowsum(vals):
    """np.sum(..., axis=1) of one row of a [forks, k] array: left to right"""
    p = vals[0]
    for v in vals[1:]:
        p = p + v
    return p


def _keep(cand, L, use_log=False):
    """indices of the kept candidates, ascending"""
    if len(cand) <= L:
        return list(range(len(cand)))
    zero = -math.inf if use_log else 0.0
    nz = sum(1 for v in cand if v != zero)
    k = max(1, min(nz, L))  # all zero: the reference fails on the empty list; keep the first
    taken = set()
    for _ in range(k):
        best = None
        for i, v in enumerate(cand):
            if i in taken:
                continue
            if best is None or v > cand[best]:
                best = i
        taken.add(best)
    return sorted(taken)


def _ratio(row, use_log=False):
    s = sorted(row)
    if use_log:
        return float(np.float64(s[-2]) - np.float64(s[-1]))
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.float64(s[-2]) / np.float64(s[-1]))


def _least_reliable(rows, k, use_log=False):
    r = [_ratio(row, use_log) for row in rows]
    order = []
    for _ in range(k):  # the least reliable first; it goes last
        best = None
        for p in range(len(rows)):
            if p in order:
                continue
            if best is None or r[p] > r[best]:
                best = p
        order.append(best)
    return order[::-1]


class ListDecoder:
    """listDecode for one codeword: rows [N][q], frozen mask, frozen values (frozen-index order),
    list size L, optional actual information.  decode() -> (list size, info rows, metrics,
    actual_prob)."""

    def __init__(self, q, frozen_mask, L, use_log=False):
        self.q = int(q)
        self.frozen = [int(v) for v in frozen_mask]
        self.N = len(self.frozen)
        self.L = int(L)
        self.log = bool(use_log)

    def decode(self, xy, frozen_values, actual=None):
        self.fv = [int(v) for v in frozen_values]
        self.fi = 0
        self.actual = None if actual is None else [int(v) for v in actual]
        self.actual_prob = 0.0 if self.log else 1.0
        self.probs = [0.0 if self.log else 1.0]
        self.info = [[]]
        rows = [list(map(float, r)) for r in xy]
        k, _, _, _ = self._node([rows], 0, 0, 1, rows)
        return k, [list(r) for r in self.info[:k]], list(self.probs[:k]), self.actual_prob

    def _frozen_value(self):
        v = self.fv[self.fi]
        self.fi += 1
        return v

    # domain-dependent steps: metric (x) factor, a node's product / sum over its positions
    def _mul(self, p, f):
        return p + f if self.log else p * f

    def _prodnode(self, vals):
        return _npsum(vals) if self.log else _prod(vals)

    def _m(self, row):
        return _marginal_log(row, self.q) if self.log else _marginal(row, self.q)

    def _norm(self, newprobs):
        w = max(newprobs)
        if self.log:
            self.probs = [float(np.float64(p) - np.float64(w)) for p in newprobs]
            return w
        with np.errstate(divide="ignore", invalid="ignore"):  # numpy's x / 0 (the reference divides arrays)
            self.probs = [float(np.float64(p) / np.float64(w)) for p in newprobs]
        return w

    def _scale_actual(self, v, w):
        if self.log:
            self.actual_prob += float(np.float64(v) - np.float64(w))
            return
        with np.errstate(divide="ignore", invalid="ignore"):
            self.actual_prob *= float(np.float64(v) / np.float64(w))

    def _fork(self, cand, lin, ii, div, enc_of, info_of):
        keep = _keep(cand, self.L, self.log)
        info = []
        encs = []
        origin = []
        for c in keep:
            i = c // div if div else c % lin
            row = self.info[i][:ii] + info_of(c)
            info.append(row)
            encs.append(enc_of(c))
            origin.append(i)
        self.info = info
        w = self._norm([cand[c] for c in keep])
        return len(keep), encs, origin, w

    def _node(self, dists, u0, ii, lin, actual_rows):
        q, L = self.q, self.L
        S = len(dists[0])
        nin = sum(1 for j in range(S) if self.frozen[u0 + j] == 0)
        track = self.actual is not None
        if S == 1:
            if nin == 1:
                m = [self._m(dists[i][0]) for i in range(lin)]
                cand = [self._mul(self.probs[c % lin], m[c % lin][c // lin]) for c in range(lin * q)]
                k, encs, origin, w = self._fork(cand, lin, ii, 0, lambda c: [c // lin], lambda c: [c // lin])
                aenc = None
                if track:
                    a = self.actual[ii]
                    self._scale_actual(self._m(actual_rows[0])[a], w)
                    aenc = [a]
                return k, encs, origin, aenc
            fv = self._frozen_value()
            w = self._norm([self._mul(self.probs[i], self._m(dists[i][0])[fv]) for i in range(lin)])
            if track:
                self._scale_actual(self._m(actual_rows[0])[fv], w)
            return lin, [[fv]] * lin, list(range(lin)), [fv]
        if nin == 0:
            enc = polar_qudits(q, [self._frozen_value() for _ in range(S)])
            w = self._norm([self._mul(self.probs[i], self._prodnode([dists[i][j][enc[j]] for j in range(S)]))
                            for i in range(lin)])
            if track:
                self._scale_actual(self._prodnode([actual_rows[j][enc[j]] for j in range(S)]), w)
            return lin, [enc] * lin, list(range(lin)), enc
        if nin == 1:
            kpos = [j for j in range(S) if self.frozen[u0 + j] == 0][0]
            base = [0 if j == kpos else self._frozen_value() for j in range(S)]
            splits = []
            for s in range(q):
                v = list(base)
                v[kpos] = s
                splits.append(polar_qudits(q, v))
            cand = [self._mul(self.probs[c % lin], self._prodnode([dists[c % lin][j][splits[c // lin][j]]
                                                                   for j in range(S)]))
                    for c in range(lin * q)]
            k, encs, origin, w = self._fork(cand, lin, ii, 0, lambda c: splits[c // lin], lambda c: [c // lin])
            aenc = None
            if track:
                aenc = splits[self.actual[ii]]
                self._scale_actual(self._prodnode([actual_rows[j][aenc[j]] for j in range(S)]), w)
            return k, encs, origin, aenc
        if nin == S or nin == S - 1:
            spc = nin == S - 1
            nf, nsel = (3, 4) if spc else (2, 2)
            fork = q ** nf
            fv = self._frozen_value() if spc else 0
            cand = [0.0] * (lin * fork)
            forks = {}
            for i in range(lin):
                rows = dists[i]
                idx = _least_reliable(rows, nsel, self.log)
                const = [j for j in range(S) if j not in idx]
                amax = [max(range(q), key=lambda x, r=rows[j]: (r[x], -x)) for j in range(S)]
                if self.log:  # cur + Python's sum of the maxima (from 0)
                    base = self.probs[i] + sum(max(rows[j]) for j in const)
                else:
                    base = self.probs[i] * (_prod([max(rows[j]) for j in const]) if const else 1.0)
                delta = (fv - sum(amax[j] for j in const)) % q
                for f in range(fork):
                    sym, rem = [0] * nsel, f
                    for t in range(nf - 1, -1, -1):
                        sym[t] = rem % q
                        rem //= q
                    if spc:
                        sym[3] = (delta - sum(sym[:3])) % q
                    sel = [rows[idx[t]][sym[t]] for t in range(nsel)]
                    cand[fork * i + f] = _rowsum(sel) + base if self.log else _prod(sel) * base
                    x = list(amax)
                    for t in range(nsel):
                        x[idx[t]] = sym[t]
                    forks[fork * i + f] = x
            off = 1 if spc else 0
            k, encs, origin, w = self._fork(cand, lin, ii, fork, lambda c: forks[c],
                                            lambda c: polar_qudits(q, forks[c])[off:])
            aenc = None
            if track:
                u = ([fv] if spc else []) + self.actual[ii:ii + S - off]
                aenc = polar_qudits(q, u)
                self._scale_actual(self._prodnode([actual_rows[j][aenc[j]] for j in range(S)]), w)
            return k, encs, origin, aenc
        # general node
        H = S // 2
        mt, pt = (_minus_log, _plus_log) if self.log else (_minus, _plus)
        minus = [mt(d, q) for d in dists]
        amin = mt(actual_rows, q) if track else None
        km, encm, om, aencm = self._node(minus, u0, ii, lin, amin)
        iim = ii + sum(1 for j in range(H) if self.frozen[u0 + j] == 0)
        plus = [pt(dists[om[r]], encm[r], q) for r in range(km)]
        aplus = pt(actual_rows, aencm, q) if track else None
        kp, encp, op, aencp = self._node(plus, u0 + H, iim, km, aplus)
        encs, origin = [], []
        for r in range(kp):
            mi = op[r]
            x = [0] * S
            for h in range(H):
                x[2 * h] = (encm[mi][h] + encp[r][h]) % q
                x[2 * h + 1] = (q - encp[r][h]) % q
            encs.append(x)
            origin.append(om[mi])
        aenc = None
        if track:
            aenc = [0] * S
            for h in range(H):
                aenc[2 * h] = (aencm[h] + aencp[h]) % q
                aenc[2 * h + 1] = (q - aencp[h]) % q
        return kp, encs, origin, aenc


def list_decode(q, frozen_mask, L, xy, frozen_values, actual=None, use_log=False):
    return ListDecoder(q, frozen_mask, L, use_log).decode(xy, frozen_values, actual)


def info_positions(frozen_mask):
    return [i for i, f in enumerate(frozen_mask) if not f]


def merge_info_and_frozen(frozen_mask, info, frozen_values):
    """mergeInfoAndFrozen (:238-242)"""
    u = np.empty(len(frozen_mask), dtype=np.int64)
    fi = [i for i, f in enumerate(frozen_mask) if f]
    ii = info_positions(frozen_mask)
    u[ii] = info
    u[fi] = frozen_values
    return u
