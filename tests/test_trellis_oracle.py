"""The deletion-channel (trellis) oracle against the reference's own outputs
(tests/golden/deletion_*.npz, made by oracle/make_golden.py from the shimmed
reference).  Pins oracle/trellis_oracle.py before any kernel is compared with it."""
import random

import numpy as np
import pytest

from oracle import trellis_oracle as tro
from tests.conftest import load_golden


def _words(g, pre=""):
    return [list(map(int, w[:l])) for w, l in zip(g[pre + "rx"], g[pre + "rx_len"])]


def deletion_edge_cases():
    g = load_golden("deletion_edge")
    out = []
    for i in range(g["meta"]["cases"]):
        out.append({k.split("_", 1)[1]: v for k, v in g.items() if k.startswith("c%d_" % i)})
    return out


def _check(words, n, n0, pd, ones, frozen, fval, info, xhat, leaf_m):
    for t, w in enumerate(words):
        lm = []
        x, inf = tro.decode_deletion(w, n, n0, pd, frozen, fval, ones=ones, leaf_m=lm)
        assert inf == list(info[t]), t
        assert x == list(xhat[t]), t
        infopos = np.asarray(frozen) == 0
        # marginals at information leaves are the xy marginals the reference decided on
        assert np.array_equal(np.array(lm)[infopos], leaf_m[t][infopos]), t


def test_deletion_c5_matches_reference():
    g = load_golden("deletion_n8")
    m = g["meta"]
    _check(_words(g), m["n"], m["n0"], m["pd"], m["ones"], g["frozen"], g["fval"], g["info"], g["xhat"],
           g["leaf_m"])


@pytest.mark.parametrize("idx", range(11))
def test_deletion_edge_matches_reference(idx):
    c = deletion_edge_cases()[idx]
    n, n0, ones = (int(v) for v in c["shape"])
    _check(_words(c), n, n0, float(c["pd"][0]), ones, c["frozen"], c["fval"], c["info"], c["xhat"], c["leaf_m"])


def test_guard_bands_round_trip():
    """add -> (no deletions) -> remove returns the per-trellis blocks when every block
    starts and ends with a 1 (then no trim moves a split point)."""
    rng = random.Random(3)
    n, n0 = 8, 2
    x = [b if i % 4 in (1, 2) else 1 for i, b in enumerate(rng.randint(0, 1) for _ in range(256))]
    cw = tro.add_guard_bands(x, n, n0, 0.1)
    assert len(cw) == load_golden("deletion_n8")["meta"]["cw_len"]
    segs = tro.remove_guard_bands(cw, n, n0)
    assert len(segs) == 64
    for i, s in enumerate(segs):
        assert s == tro.trim(x[4 * i:4 * i + 4])


def test_reference_mc_line_reproduced():
    """encodeDecodeSimulation's printed line, from the restated pipeline and the reference's seeds."""
    g = load_golden("deletion_n8")
    m = g["meta"]
    n, n0, pd, xi = m["n"], m["n0"], m["pd"], m["xi"]
    N = 1 << n
    frozen = g["genie_frozen"]
    r = random.Random(m["crs"])
    rv = [r.random() for _ in range(N)]
    fval = np.array([0 if 0.5 >= v else 1 for v in rv], np.uint8)
    K = int(N - frozen.sum())
    irng = random.Random(m["info_seed"])
    crng = random.Random(m["channel_seed"])
    errors = 0
    for _ in range(m["mc_trials"]):
        inf = [0 if irng.random() < 0.5 else 1 for _ in range(K)]
        u = np.zeros(N, np.uint8)
        u[frozen == 1] = fval[frozen == 1]
        u[frozen == 0] = inf
        x = _polar(u)
        rx = tro.deletion_channel(tro.add_guard_bands(x, n, n0, xi), pd, crng)
        _, dinf = tro.decode_deletion(rx, n, n0, pd, frozen, fval)
        errors += int(dinf != inf)
    T = m["mc_trials"]
    line = " ".join(str(v) for v in ["Error probability = ", errors, "/", T, " = ", errors / T])
    assert line == m["line"]


def _polar(u):
    """x = polar transform of u in the reference's adjacent-pair convention
    (BinaryPolarEncoderDecoder.py:319-323): encode(u) recursively."""
    u = list(map(int, u))
    if len(u) == 1:
        return u
    h = len(u) // 2
    xm, xp = _polar(u[:h]), _polar(u[h:])
    out = []
    for i in range(h):
        out += [(xm[i] + xp[i]) % 2, xp[i]]
    return out


# -- the C restatement (oracle/trellis_oracle.c): pinned to the same reference outputs and to the
#    Python restatement on random shapes; bench.py times it as the deletion CPU baseline.

def _padded(words):
    W = max([len(w) for w in words] + [1])
    rx = np.zeros((len(words), W), np.uint8)
    for i, w in enumerate(words):
        rx[i, :len(w)] = w
    return rx, np.array([len(w) for w in words], np.int32)


def test_c_oracle_matches_reference():
    from oracle import orc
    g = load_golden("deletion_n8")
    m = g["meta"]
    info, xhat = orc.decode_deletion(g["rx"], g["rx_len"], m["n"], m["n0"], m["pd"], g["frozen"], g["fval"], m["ones"])
    assert np.array_equal(info, g["info"]) and np.array_equal(xhat, g["xhat"])
    for c in deletion_edge_cases():
        n, n0, ones = (int(v) for v in c["shape"])
        info, xhat = orc.decode_deletion(c["rx"], c["rx_len"], n, n0, float(c["pd"][0]), c["frozen"], c["fval"], ones)
        assert np.array_equal(info, c["info"]) and np.array_equal(xhat, c["xhat"])


# (12, 4, 0), (13, 4, 0): main_deletion's own n0 = n // 3 at n = 12, 13 (256 and 512 trellises of
# length 16), the shapes the GPU's n0 = 4 kernels are checked against the C oracle at
@pytest.mark.parametrize("n,n0,ones", [(6, 2, 0), (8, 2, 0), (9, 3, 0), (10, 3, 0), (8, 2, 2), (7, 1, 0), (8, 4, 0),
                                       (5, 5, 1), (12, 4, 0), (13, 4, 0)])
def test_c_oracle_matches_python_oracle(n, n0, ones):
    from oracle import orc
    rng = np.random.default_rng(10 * n + n0 + ones)
    prng = random.Random(n + n0)
    N = 1 << n
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    nw = 5 if n < 12 else 2  # the Python restatement takes ~2 s a word at n = 13
    words = [tro.deletion_channel(tro.add_guard_bands([int(b) for b in rng.integers(0, 2, N)], n, n0, 0.1, ones), 0.1,
                                  prng) for _ in range(nw)]
    words += [[], [1], [0, 0, 1], [1] * (N + 3)]
    rx, ln = _padded(words)
    info, xhat = orc.decode_deletion(rx, ln, n, n0, 0.1, frozen, fval, ones)
    for i, w in enumerate(words):
        x, inf = tro.decode_deletion(w, n, n0, 0.1, frozen, fval, ones)
        assert list(info[i]) == inf and list(xhat[i]) == x, i
