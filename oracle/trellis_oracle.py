"""CPU restatement of the reference's deletion-channel path (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this
module, and only as the checker; the product path never imports it.

What it restates (file:line in the reference tree, snapshot 2025-02-04):
  * guard bands        Guardbands.py:4-44 (add), :47-63 (remove), :66-93 (trim)
  * deletion channel   VectorDistributions/BinaryTrellis.py:441-461
  * trellis build      VectorDistributions/BinaryTrellis.py:309-438
  * minus/plus         VectorDistributions/BinaryTrellis.py:206-258
  * marginal           VectorDistributions/BinaryTrellis.py:260-278
  * normalisation      VectorDistributions/BinaryTrellis.py:280-306
  * collection         VectorDistributions/CollectionOfBinaryTrellises.py:55-103, :106-129
  * memoryless rows    VectorDistributions/BinaryMemorylessVectorDistribution.py:15-87
  * SC recursion       BinaryPolarEncoderDecoder.py:223-325 (decode branch; uniform
                       a-priori tree, so frozen u_i = 0 if 0.5 >= r_i else 1, :258-262)

Floating-point sums follow the reference's iteration order, which is the
insertion order of its vertex and edge dictionaries; this restatement keeps the
same insertion-ordered dictionaries (Python dicts preserve insertion order), so
every sum is formed in the same order.  Pinned by tests/golden/deletion_n8.npz,
produced by running the reference itself (oracle/make_golden.py).
"""
import math


# --------------------------------------------------------------------------- guard bands

def trim(word):
    """Guardbands.py:66-93: the slice between the first and the last 1 (empty if none)."""
    first = next((i for i, b in enumerate(word) if b == 1), -1)
    if first < 0:
        return []
    last = max(i for i, b in enumerate(word) if b == 1)
    return list(word[first:last + 1])


def remove_guard_bands(word, n, n0):
    """Guardbands.py:47-63: trim, halve, recurse until n <= n0."""
    t = trim(word)
    if n <= n0:
        return [t]
    h = len(t) // 2
    return remove_guard_bands(t[:h], n - 1, n0) + remove_guard_bands(t[h:], n - 1, n0)


def add_guard_bands(x, n, n0, xi, ones=0):
    """Guardbands.py:4-44: ln = floor(2^((1-xi)(n-1))) zeros between the two halves."""
    x = list(x)
    if n <= n0:
        return [1] * ones + x + [1] * ones if ones > 0 else x
    assert len(x) % 2 == 0
    ln = math.floor(2 ** ((1 - xi) * (n - 1)))
    h = len(x) // 2
    return add_guard_bands(x[:h], n - 1, n0, xi, ones) + [0] * ln + add_guard_bands(x[h:], n - 1, n0, xi, ones)


def deletion_channel(codeword, p, rng):
    """BinaryTrellis.py:441-461: drop each symbol when rng.random() < p."""
    return [c for c in codeword if not rng.random() < p]


# --------------------------------------------------------------------------- trellis

class _V:
    __slots__ = ("vpos", "prob", "ins", "outs")

    def __init__(self, vpos):
        self.vpos = vpos
        self.prob = -1.0
        self.ins = {}   # (u_vpos, v_vpos, label) -> edge, insertion ordered
        self.outs = {}


class _E:
    __slots__ = ("u", "v", "label", "prob")

    def __init__(self, u, v, label):
        self.u, self.v, self.label, self.prob = u, v, label, 0.0


class Trellis:
    """Single-state trellis; layer l is an insertion-ordered dict vpos -> vertex."""

    def __init__(self, length):
        assert length > 0
        self.length = length
        self.layers = [dict() for _ in range(length + 1)]

    def vertex(self, layer, vpos):
        d = self.layers[layer]
        if vpos not in d:
            d[vpos] = _V(vpos)
        return d[vpos]

    def set_prob(self, layer, vpos, p):
        self.vertex(layer, vpos).prob = p

    def add(self, layer, u, v, label, p):
        """BinaryTrellis.py:128-136, 164-175: from-vertex first, then to-vertex, then the edge."""
        fu = self.vertex(layer, u)
        tv = self.vertex(layer + 1, v)
        key = (u, v, label)
        e = fu.outs.get(key)
        if e is None:
            e = _E(fu, tv, label)
            fu.outs[key] = e
            tv.ins[key] = e
        e.prob += p

    # BinaryTrellis.py:206-258
    def transform(self, decisions=None):
        new = Trellis(self.length // 2)
        if decisions is not None:
            assert len(decisions) == self.length // 2
        for v in self.layers[0].values():
            new.set_prob(0, v.vpos, v.prob)
        for v in self.layers[self.length].values():
            new.set_prob(self.length // 2, v.vpos, v.prob)
        for mid in range(1, self.length + 1, 2):
            j = (mid - 1) // 2
            for w in self.layers[mid].values():
                for ein in w.ins.values():
                    for eout in w.outs.values():
                        p = ein.prob * eout.prob
                        lbl = 1 if ein.label != eout.label else 0
                        if decisions is None:
                            new.add(j, ein.u.vpos, eout.v.vpos, lbl, p)
                        else:
                            if lbl != decisions[j]:
                                continue
                            new.add(j, ein.u.vpos, eout.v.vpos, eout.label, p)
        return new

    # BinaryTrellis.py:260-278 (normalize=False as used by the collection collapse)
    def marginal(self, normalize=True):
        assert self.length == 1
        m = [0.0, 0.0]
        if normalize:
            s = 0.0
            for v in self.layers[0].values():
                for e in v.outs.values():
                    s += v.prob * e.prob * e.v.prob
        else:
            s = 1.0
        for v in self.layers[0].values():
            for e in v.outs.values():
                m[e.label] += v.prob * e.prob * e.v.prob / s
        return m

    # BinaryTrellis.py:280-294
    def normalization(self):
        out = []
        for i in range(self.length):
            t = [0.0, 0.0]
            for v in self.layers[i].values():
                for e in v.outs.values():
                    t[e.label] += e.prob
            out.append(t[0] if t[0] >= t[1] else t[1])
        return out

    # BinaryTrellis.py:297-306
    def normalize(self, norm):
        for i in range(self.length):
            t = norm[i]
            assert t >= 0
            if t == 0:
                t = 1
            for v in self.layers[i].values():
                for e in v.outs.values():
                    e.prob /= t


def build_trellis(word, L, pd, trimmed=True, ones=0):
    """BinaryTrellis.py:309-438, single input state, uniform input (0.5, 0.5)."""
    t = Trellis(L)
    m = len(word)
    dcount = L + 2 * ones - m
    pin = (0.5, 0.5)
    if ones > 0:
        assert trimmed
        for i in range(1 + min(ones, m)):
            t.set_prob(0, i, math.comb(ones, i) * ((1.0 - pd) ** i) * (pd ** (ones - i)))
        for i in range(m, m - min(ones, m) - 1, -1):
            j = m - i
            t.set_prob(L, i, math.comb(ones, j) * ((1.0 - pd) ** j) * (pd ** (ones - j)))
    else:
        t.set_prob(0, 0, 1.0)
        t.set_prob(L, m, 1.0)
    if trimmed:
        assert m == 0 or (word[0] == 1 and word[-1] == 1)
    for l in range(L):
        if ones > 0:
            lo, hi = max(0, l + ones - dcount), min(l + ones, m)
        else:
            lo, hi = max(0, l - dcount), min(l, m)
        for vp in range(lo, hi + 1):
            if vp < m:
                t.add(l, vp, vp + 1, word[vp], pin[word[vp]] * (1.0 - pd))
            if l + 1 + ones - dcount <= vp:
                for lbl in range(2):
                    if (not trimmed) or lbl == 1 or (0 < vp < m):
                        p = pin[lbl] * pd
                    else:
                        p = pin[lbl]
                    t.add(l, vp, vp, lbl, p)
    return t


# --------------------------------------------------------------------------- vector distributions

class Collection:
    """CollectionOfBinaryTrellises.py: T trellises, total input length `length`."""

    def __init__(self, trellises, length):
        self.trellises = trellises
        self.length = length

    def __len__(self):
        return self.length

    def transform(self, decisions=None):  # :55-82
        T = len(self.trellises)
        sub = (len(decisions) // T) if decisions is not None else 0
        kids = [tr.transform(None if decisions is None else decisions[i * sub:(i + 1) * sub])
                for i, tr in enumerate(self.trellises)]
        if self.length // 2 > T:
            return Collection(kids, self.length // 2)
        assert self.length // 2 == T
        return Memoryless([k.marginal(normalize=False) for k in kids])

    def normalize_self(self):  # decoder: calcNormalizationVector + normalizeDistList
        for tr in self.trellises:
            tr.normalize(tr.normalization())


class Memoryless:
    """BinaryMemorylessVectorDistribution.py:15-87 on rows [p0, p1]."""

    def __init__(self, rows):
        self.rows = [list(r) for r in rows]

    def __len__(self):
        return len(self.rows)

    def transform(self, decisions=None):
        out = []
        r = self.rows
        for h in range(len(r) // 2):
            a, b = r[2 * h], r[2 * h + 1]
            if decisions is None:
                out.append([a[0] * b[0] + a[1] * b[1], a[0] * b[1] + a[1] * b[0]])
            elif decisions[h] == 0:
                out.append([a[0] * b[0], a[1] * b[1]])
            else:
                out.append([a[1] * b[0], a[0] * b[1]])
        return Memoryless(out)

    def normalize_self(self):
        for row in self.rows:
            t = row[0] if row[0] >= row[1] else row[1]  # np.maximum (no NaNs arise)
            assert t >= 0
            if t == 0:
                t = 1
            row[0] /= t
            row[1] /= t

    def leaf_decision(self):  # :52-69 + BinaryPolarEncoderDecoder.py:250-252
        p0, p1 = self.rows[0]
        s = 0.0
        s += p0
        s += p1
        m = (p0 / s, p1 / s) if s > 0.0 else (0.5, 0.5)
        return 0 if m[0] >= m[1] else 1, m


def build_collection(word, pd, n, n0, ones=0):
    """CollectionOfBinaryTrellises.py:106-129."""
    segs = remove_guard_bands(word, n, n0)
    return Collection([build_trellis(s, 1 << n0, pd, True, ones) for s in segs], 1 << n)


def sc_decode(vd, frozen, fval, leaf_m=None):
    """BinaryPolarEncoderDecoder.py:223-325, decode branch over one xy vector distribution;
    the uniform a-priori tree only supplies the frozen values fval (:258-262).
    Returns (x_hat list, info list); leaf_m (optional list) receives every leaf's
    marginal in u order (genie export)."""
    info = []
    u = [0]

    def rec(d):
        if len(d) == 1:
            i = u[0]
            u[0] += 1
            dec, m = d.leaf_decision()
            if leaf_m is not None:
                leaf_m.append(m)
            if frozen[i]:
                return [int(fval[i])]
            info.append(dec)
            return [dec]
        mvd = d.transform()
        mvd.normalize_self()
        xm = rec(mvd)
        pvd = d.transform(xm)
        pvd.normalize_self()
        xp = rec(pvd)
        out = []
        for h in range(len(xm)):
            out += [(xm[h] + xp[h]) % 2, xp[h]]
        return out

    x = rec(vd)
    return x, info


def decode_deletion(word, n, n0, pd, frozen, fval, ones=0, leaf_m=None):
    return sc_decode(build_collection(word, pd, n, n0, ones), frozen, fval, leaf_m)
