"""Distributional agreement under the native random streams (north_star: "KS test on cut-edge
and district-shape statistics under native RNG").

The reference's flip step driven by CPython's Mersenne Twister and numpy's legacy geometric
(oracle.flipref.NativeRngChain; fixture tests/golden/native_rng_c1.npz, made by
tests/golden/make_native.py) against the canonical Philox stream of the C oracle, on
BASELINE config C1 (10x10 grid, k = 2, plan x[0] >= 5, pop tolerance 0.1) at bases 1 and mu,
2000 steps: two-sample KS tests on the end state's |cut edges|, |b_nodes| and district
population, the time-averaged |cut| and |B| of each chain, and the geometric wait.  The
device is held to the same fixture in tests/test_distribution_gpu.py.
"""
import os

import numpy as np
import pytest
from scipy.stats import ks_2samp

from flipcomplexityempirical_amd import graphs as G

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "native_rng_c1.npz")
STATS = ("cut", "nb", "pop1", "wait", "mean_cut", "mean_nb")
P_MIN = 1e-3  # per comparison; the samples are fixed (seeded), so the outcome is deterministic


def c1_setup():
    spec = G.grid_graph(10, 10)
    a0 = spec.assignment_array(G.threshold_plan(spec.nodes, 0, 5), [-1, 1])
    _, (lo, hi) = G.population_bounds(100, 2, 0.1)
    return spec, a0, lo, hi


def summarize(spec, finals, waits, sum_cut, sum_nb, T):
    cut, nb, pop1 = [], [], []
    for a in finals:
        c, b, pops = G.cut_and_boundary(spec, a)
        cut.append(c)
        nb.append(b)
        pop1.append(pops[1])
    return {"cut": np.asarray(cut, float), "nb": np.asarray(nb, float), "pop1": np.asarray(pop1, float),
            "wait": np.asarray(waits, float), "mean_cut": np.asarray(sum_cut, float) / (T + 1),
            "mean_nb": np.asarray(sum_nb, float) / (T + 1)}


def assert_same_distribution(fix, bi, got, label):
    for s in STATS:
        ref = fix[f"b{bi}_{s}"]
        p = ks_2samp(ref, got[s]).pvalue
        assert p > P_MIN, (label, s, p, ref.mean(), got[s].mean())


@pytest.mark.parametrize("bi", [0, 1])
def test_canonical_oracle_matches_native_rng(cref, bi):
    fix = np.load(FIX)
    T, base = int(fix["T"]), float(fix["bases"][bi])
    spec, a0, lo, hi = c1_setup()
    finals, waits, sc, sn = [], [], [], []
    for c in range(600):
        r = cref.run(spec, a0, base=base, pop_lo=lo, pop_hi=hi, seed=0xD15, chain_id=c, n_steps=T,
                     log1mp=G.log1mp_table(100, 2))
        finals.append(r["final"])
        waits.append(r["stats"]["wait_cur"])
        sc.append(r["stats"]["sum_cut"])
        sn.append(r["stats"]["sum_nb"])
    assert_same_distribution(fix, bi, summarize(spec, finals, waits, sc, sn, T), "C oracle")
