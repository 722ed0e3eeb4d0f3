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


@pytest.fixture(scope="session")
def golden():
    return load_golden
