"""Pin the CPU oracle against the reference's own artifacts.

The reference ships no tests; its only checkable outputs are the 174 configuration
artifacts.  ``tests/golden/reference_artifacts.npz`` (made by ``make_golden.py``) holds the
decoded ``*end2.png`` final states and the ``*wait.txt`` sums.  Pins:

1. the start plans' known answers (|cut|, |B|, populations; App. B.3);
2. every decoded final state is contiguous and inside its population bound under the
   oracle's checkers -- states the reference's chain actually reached;
3. ``single_flip_contiguous`` restated (BFS) agrees with the device's planar local rule on
   every boundary node of every decoded state (the exactness claim of DESIGN.md);
4. the oracle chain, re-run on all 174 reference configurations (every base x pop x
   alignment of both sweeps), reproduces the reference's ``wait.txt`` sums per (base, pop)
   and per base, and its final |cut| / |B| distributions per base match the decoded end
   states (``tests/reference_pin.py``).
"""
import os
import re
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_artifacts.npz")


def _parse(key):
    m = re.match(r"^(\d)B(\d+)P(\d+)$", key)
    return int(m.group(1)), int(m.group(2)), int(m.group(3))


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _to_assign(spec, img, frank=False):
    """Decoded image (row = n[0], col = n[1] (+19 FRANK)) -> district ids in node order."""
    a = np.zeros(spec.n, dtype=np.int8)
    for i, nd in enumerate(spec.nodes):
        v = img[nd[0], nd[1] + (19 if frank else 0)]
        assert v in (-1, 1), (nd, v)
        a[i] = 0 if v == -1 else 1
    return a


def test_start_plan_known_answers(sec11, frank):
    exp = {0: (40, 80, [798, 798]), 1: (40, 80, [798, 798]), 2: (78, 80, [798, 798])}
    for al, (cut, nb, pops) in exp.items():
        a = sec11.assignment_array(G.sec11_plan(al, sec11.nodes), [-1, 1])
        c, b, p = G.cut_and_boundary(sec11, a)
        assert (c, b, sorted(p.tolist())) == (cut, nb, pops)
    exp = {0: (87, 97, [380, 420]), 1: (60, 80, [400, 400]), 2: (20, 40, [380, 420])}
    for al, (cut, nb, pops) in exp.items():
        a = frank.assignment_array(G.frank_plan(al, frank.nodes), [-1, 1])
        c, b, p = G.cut_and_boundary(frank, a)
        assert (c, b, sorted(p.tolist())) == (cut, nb, pops)
    assert (sec11.n, sec11.n_edges, frank.n, frank.n_edges) == (1596, 3116, 800, 1920)


def test_population_bounds_float_semantics():
    # ((1-p)*ideal, (1+p)*ideal) in float64, as Bounds compares them [gc-0.2]
    assert G.population_bounds(800, 2, 0.05) == ((380.0, 420.0), (380, 420))
    assert G.population_bounds(800, 2, 0.1)[0][1] == 440.00000000000006
    assert G.population_bounds(800, 2, 0.9)[1] == (40, 760)
    assert G.population_bounds(1596, 2, 0.01)[1] == (791, 805)


def test_decoded_end_states_valid(gold, cref, sec11, frank):
    for tag, spec, fr in (("sec11", sec11, False), ("frank", frank, True)):
        for key, img in zip(gold[f"{tag}_keys"], gold[f"{tag}_end"]):
            _, _, P = _parse(str(key))
            a = _to_assign(spec, img, fr)
            if not fr:  # the 4 removed corners are the only empty cells
                assert sorted(zip(*np.nonzero(img == 0))) == sorted(G.SEC11_CORNERS)
            assert cref.districts_contiguous(spec, a, 2), key
            _, (lo, hi) = G.population_bounds(spec.n, 2, P / 100)
            pops = np.bincount(a, minlength=2)
            assert lo <= pops.min() and pops.max() <= hi, (key, pops, lo, hi)


def _local_rule(ring, meta, a, v, touch_other):
    """Restatement of the device's contiguity rule (fc_kernels.hip one_run / status)."""
    L = int(meta & 0xFF)
    nbr = int(meta >> 16) & 0xFFFF
    link = int(meta >> 32) & 0xFFFF
    exact = bool(meta >> 8 & 1)
    gam = bool(meta >> 9 & 1)
    inA = [a[ring[i]] == a[v] for i in range(L)]
    ids = [i for i in range(L) if nbr >> i & 1 and inA[i]]
    if not ids:
        return False, True

    def runs(virtual):
        lk = [inA[i] and inA[(i + 1) % L] and bool(link >> i & 1) for i in range(L)]
        if virtual and L >= 2 and inA[0] and inA[L - 1]:
            lk[L - 1] = True
        brk = [not x for x in lk]
        cnt = 0
        for j, s in enumerate(ids):
            e = ids[j + 1] if j + 1 < len(ids) else ids[0] + L
            cnt += any(brk[q % L] for q in range(s, e))
        return cnt <= 1

    single = runs(gam and not touch_other)
    if exact:
        return single, True
    return single, single  # (result, known)


def test_local_rule_exact_on_reference_states(gold, cref, sec11, frank):
    from flipcomplexityempirical_amd.engine import FlipGraph
    checked = 0
    for tag, spec, fr in (("sec11", sec11, False), ("frank", frank, True)):
        ring, meta = FlipGraph(spec).rings()
        gam = np.array([(int(m) >> 9) & 1 for m in meta], dtype=bool)
        for img in gold[f"{tag}_end"][::3]:
            a = _to_assign(spec, img, fr)
            e = spec.edges()
            cutm = a[e[:, 0]] != a[e[:, 1]]
            bnodes = np.unique(e[cutm].reshape(-1))
            for v in bnodes:
                other = 1 - a[v]
                touch = bool(np.any(gam & (a == other)))
                res, known = _local_rule(ring[v], int(meta[v]), a, v, touch)
                assert known
                assert res == cref.flip_contiguous(spec, a, int(v)), (tag, spec.nodes[v])
                checked += 1
    assert checked > 10000


def _pin_run(args):
    (tag, al, base, pct, key), seed = args
    from oracle.flipref import CRef
    import reference_pin as RP
    spec = RP.spec_of(tag)
    _, (lo, hi) = G.population_bounds(spec.n, 2, pct)
    r = CRef().run(spec, RP.start_plan(spec, tag, al), base=base, pop_lo=lo, pop_hi=hi, seed=seed, chain_id=al,
                   n_steps=99999, log1mp=G.log1mp_table(spec.n, 2))
    return r["stats"]["sum_wait"], r["stats"]["cut"], r["stats"]["nb"]


def test_oracle_reproduces_every_reference_artifact():
    """All 174 reference configurations (every base x pop x alignment of both sweeps), two
    seeds each, 100,000 yields (total_steps = 100000, grid_chain_sec11.py:342 -> 99,999 steps
    after S0): wait.txt means per (graph, base, pop) and per (graph, base), and the final
    |cut| / |B| distributions per base against the decoded end2 states (tests/reference_pin.py).
    The device repeats this with eight seeds per configuration (test_reference_pin_gpu.py)."""
    import reference_pin as RP
    cfgs = RP.configs()
    assert len(cfgs) == 174
    jobs = [(c, s) for c in cfgs for s in (2001, 2002)]
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(_pin_run, jobs, chunksize=1))
    worst = RP.check([(c, w, cut, nb) for (c, _), (w, cut, nb) in zip(jobs, res)])
    assert worst["max_abs_z"] < RP.Z_MAX and worst["min_ks_p"] > RP.KS_P_MIN
