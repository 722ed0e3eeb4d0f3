import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {k: d[k] for k in d.files}
    out["meta"] = json.loads(str(out["meta"]))
    return out


def edge_cases():
    g = load_golden("edge_binary")
    cases = []
    for i in range(g["meta"]["cases"]):
        cases.append({k.split("_", 1)[1]: v for k, v in g.items() if k.startswith("c%d_" % i)})
    return cases


_EDGE_LONG = None


def edge_long_cases():
    """tests/golden/edge_long.npz (oracle/make_golden.py fx_edge_long): the reference's decodes of
    the edge families at N = 1024 / 4096, unpacked to xy [B][N][2], info [B][K], xhat [B][N]."""
    global _EDGE_LONG
    if _EDGE_LONG is None:
        g = load_golden("edge_long")
        cases = []
        for i in range(g["meta"]["cases"]):
            c = {k.split("_", 1)[1]: v for k, v in g.items() if k.startswith("c%d_" % i)}
            N, K = 1 << int(c["n"]), int(c["K"])
            c["xy"] = c["table"][c["idx"]]
            c["info"] = np.unpackbits(c["info_bits"], axis=1)[:, :K]
            c["xhat"] = np.unpackbits(c["xhat_bits"], axis=1)[:, :N]
            c["family_name"] = g["meta"]["families"][int(c["family"])]
            cases.append(c)
        _EDGE_LONG = cases
    return _EDGE_LONG


@pytest.fixture(scope="session")
def golden():
    return load_golden


def blocky_frozen(N, rng):
    """A frozen set with aligned all-frozen (rate-0) and all-information blocks of
    every size from 1 to N/4 plus scattered singles, and random frozen values:
    exercises every rate-0 skip of the decode schedule."""
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    w = N // 4
    while w >= 1:
        for _ in range(2):
            s = int(rng.integers(0, N // w)) * w
            frozen[s:s + w] = int(rng.integers(0, 2))
        w //= 2
    frozen[: N // 8] = 1  # a leading rate-0 block, as in real polar codes
    frozen[-1] = 0
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    return frozen, fval


def awgn_like(B, N, rng, zeros=0.02):
    llr = rng.normal(2.0, 2.0, (B, N)) * np.where(rng.random((B, N)) < 0.5, 1, -1)
    p1 = 1.0 / (1.0 + np.exp(llr))
    xy = np.stack([1.0 - p1, p1], axis=-1) * 0.5
    xy[rng.random((B, N)) < zeros] = 0.0
    return xy
