"""Tal-Vardy construction against the reference's own
outputs (tests/golden/construct_bin.npz, oracle/make_golden.py::fx_construct_bin):
mergeEquivalentSymbols, degrade(L) with auxiliary letter sets, upgrade(L) and its
AttributeError, and calcFrozenSet_degradingUpgrading's Pe vectors and frozen sets
(test2.py's BSC(0.11), n=7, L=100 among them) -- all bit-exact.  Host library only
(libpolarcub_construct.so), no GPU."""
import builtins

import numpy as np
import pytest

from polarcub_amd import construction, scalar
from tests.conftest import load_golden

G = load_golden("construct_bin")
CASES = G["meta"]["cases"]


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.int64)


def dist(pairs, aux=False):
    d = scalar.BinaryMemorylessDistribution()
    d.probs = [[float(p[0]), float(p[1])] for p in pairs]
    if aux:
        d.auxiliary = [{i} for i in range(len(pairs))]
    return d


def groups(aux, n):
    g = np.full(n, -1, np.int64)
    for j, s in enumerate(aux):
        for i in s:
            g[i] = j
    return g


@pytest.mark.parametrize("case", [c["case"] for c in CASES])
def test_merge_equivalent(case):
    pairs = G[case + "_in"]
    d = dist(pairs, aux=True)
    d.mergeEquivalentSymbols()
    assert np.array_equal(bits(d.probs), bits(G[case + "_merged"]))
    assert np.array_equal(groups(d.auxiliary, len(pairs)), G[case + "_merged_aux"])


@pytest.mark.parametrize("case", [c["case"] for c in CASES])
def test_degrade(case):
    rec = next(c for c in CASES if c["case"] == case)
    pairs = G[case + "_in"]
    for L in rec["deg"]:
        d = dist(pairs, aux=True)
        o = d.degrade(L)
        assert len(o.probs) <= L
        assert np.array_equal(bits(o.probs), bits(G["%s_deg%d" % (case, L)])), L
        assert np.array_equal(groups(o.auxiliary, len(pairs)), G["%s_deg%d_aux" % (case, L)]), L
        # degrade() merges self first, as the reference does
        assert np.array_equal(bits(d.probs), bits(G[case + "_merged"]))


@pytest.mark.parametrize("case", [c["case"] for c in CASES])
def test_upgrade(case):
    rec = next(c for c in CASES if c["case"] == case)
    pairs = G[case + "_in"]
    for L in rec["up"]:
        o = dist(pairs).upgrade(L)
        assert np.array_equal(bits(o.probs), bits(G["%s_up%d" % (case, L)])), L
    for L, exc in rec["up_err"]:
        with pytest.raises(getattr(builtins, exc)):
            dist(pairs).upgrade(L)


@pytest.mark.parametrize("tree", G["meta"]["trees"], ids=lambda t: t["name"])
@pytest.mark.parametrize("threads", [1, 4])
def test_construction_tree(tree, threads):
    name, n, L, bound = tree["name"], tree["n"], tree["L"], tree["bound"]
    src = dist(G[name + "_tree_in"])
    TV, Pe = construction.tv_pe(n, L, None, src.probs, threads)
    assert np.array_equal(bits(Pe), bits(G[name + "_tree_pe"]))
    assert not TV.any()
    fz = scalar.calcFrozenSet_degradingUpgrading(n, L, bound, None, src, threads=threads)
    mask = np.zeros(1 << n, np.uint8)
    mask[sorted(fz)] = 1
    assert np.array_equal(mask, G[name + "_tree_frozen"])


def test_upgrade_tree_bounds_degrade():
    """x-side tree (the reference crashes there): upgraded channels are
    better than degraded ones, so TV of the upgraded x tree is finite and the Pe of the
    upgraded xy tree never exceeds the degraded one's."""
    bsc = scalar.makeBSC(0.11)
    _, pe_deg = construction.tv_pe(6, 16, None, bsc.probs)
    tv, _ = construction.tv_pe(6, 16, bsc.probs, bsc.probs)
    assert np.all(np.isfinite(tv)) and np.all(tv >= 0)
    ups = [bsc]
    for _ in range(6):
        nxt = []
        for d in ups:
            nxt.append(d.minusTransform().upgrade(16))
            nxt.append(d.plusTransform().upgrade(16))
        ups = nxt
    pe_up = np.array([d.errorProb() for d in ups])
    assert np.all(pe_up <= pe_deg + 1e-12)


def test_errors_and_arguments():
    with pytest.raises(IndexError):  # no letter of positive probability (self.probs[0])
        dist([[0.0, 0.0]]).mergeEquivalentSymbols()
    with pytest.raises(ValueError):
        construction.degrade(np.zeros((0, 2)), 4)
    with pytest.raises(ValueError):
        construction.tv_pe(30, 4, None, [[0.5, 0.5]])


def test_test2_construction_printout():
    """The test2.py counterpart's construction prints the reference run's first lines
    (frozen set and rate); the trials themselves run on the GPU (test_gpu_genie.py)."""
    import contextlib
    import io
    g = load_golden("test2_run")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        scalar.calcFrozenSet_degradingUpgrading(7, 100, 0.1, None, scalar.makeBSC(0.11))
    assert buf.getvalue().strip().splitlines() == g["meta"]["lines"][:2]


def test_linked_list_heap_matches_reference():
    """polarcub_amd.heap.LinkedListHeap against the reference's on tied keys: extraction
    order, neighbour key updates, final list and heap array."""
    from polarcub_amd.heap import LinkedListHeap
    keys, upd = G["heap_keys"], G["heap_updates"]
    h = LinkedListHeap([float(k) for k in keys], list(range(len(keys))))
    order, ui = [], 0
    for _ in range(len(G["heap_order"])):
        e = h.extractHeapMin()
        order.append(e.data)
        for nb in (e.leftElementInList, e.rightElementInList):
            if nb is not None:
                h.updateKey(nb, float(upd[ui]))
            ui += 1
    assert order == list(G["heap_order"])
    assert h.returnData() == list(G["heap_final_list"])
    assert [el.data for el in h._heapArray] == list(G["heap_final_array"])
