"""Distributional agreement under the native random streams (north_star: "KS test on cut-edge
and district-shape statistics under native RNG").

The reference's flip step driven by CPython's Mersenne Twister and numpy's legacy geometric
(oracle.flipref.NativeRngChain; fixtures tests/golden/native_rng_{c1,sec11}.npz, made by
tests/golden/make_native.py) against the canonical Philox stream of the C oracle:
  c1:    BASELINE config C1 (10x10 grid, k = 2, plan x[0] >= 5, pop tolerance 0.1),
         bases 1 and mu, 2000 steps;
  sec11: the headline lattice (grid_chain_sec11.py:186-260), alignment-2 plan, pop
         tolerance 0.1, bases 0.8 and mu, 1000 steps;
  sec11_long: alignment-0 plan, the extreme bases 0.2 and 10, 10,000 steps (long chains far
         from the start state).
Two-sample KS tests on the end state's |cut edges|, |b_nodes| and district population, each
chain's time-averaged |cut| and |B|, and the geometric wait of the end state; for sec11 also
the district-shape statistics of the driver's slope / angle lines (grid_chain_sec11.py:55-78,
371-394): each chain's mean interface angle over its yields and the end state's angle (with
both districts contiguous exactly two frame edges are cut, so the angle does not depend on
the reference's set order).  The device is held to the same fixtures in
tests/test_distribution_gpu.py, with the angles from its own frame-series kernel.
"""
import os

import numpy as np
import pytest
from scipy.stats import ks_2samp

from flipcomplexityempirical_amd import graphs as G

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STATS = ("cut", "nb", "pop1", "wait", "mean_cut", "mean_nb")
SHAPE_STATS = ("angle_mean", "angle_end")  # sec11 only
P_MIN = 1e-3  # per comparison; the samples are fixed (seeded), so the outcome is deterministic
CASES = [("c1", 0), ("c1", 1), ("sec11", 0), ("sec11", 1), ("sec11_long", 0), ("sec11_long", 1)]
ALIGNMENT = {"sec11": 2, "sec11_long": 0}


def fixture(cfg):
    return np.load(os.path.join(GOLD, f"native_rng_{cfg}.npz"))


def setup(cfg):
    if cfg == "c1":
        spec = G.grid_graph(10, 10)
        a0 = spec.assignment_array(G.threshold_plan(spec.nodes, 0, 5), [-1, 1])
    else:
        spec = G.sec11_graph()
        a0 = spec.assignment_array(G.sec11_plan(ALIGNMENT[cfg], spec.nodes), [-1, 1])
    _, (lo, hi) = G.population_bounds(spec.n, 2, 0.1)
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
    names = STATS + tuple(s for s in SHAPE_STATS if s in got)
    if f"b{bi}_angle_mean" in fix.files:
        assert all(s in got for s in SHAPE_STATS), "shape statistics missing"
    for s in names:
        ref = fix[f"b{bi}_{s}"]
        ref, val = ref[np.isfinite(ref)], np.asarray(got[s], float)
        val = val[np.isfinite(val)]
        p = ks_2samp(ref, val).pvalue
        assert p > P_MIN, (label, s, p, ref.mean(), val.mean())


def angle_of(mid_a, mid_b, center=(20.0, 20.0)):
    """The driver's angle line (:391-394) on two frame-edge midpoints."""
    anga = np.asarray(mid_a, float) - center
    angb = np.asarray(mid_b, float) - center
    return float(np.arccos(np.clip(np.dot(anga / np.linalg.norm(anga), angb / np.linalg.norm(angb)), -1, 1)))


def shape_from_events(spec, frame, a0, events, T):
    """(mean angle over the yields with exactly two frame cut edges, end angle) of one chain
    from its accepted flips ``events`` = [(t, v)] (t = the yield the flip creates)."""
    a = a0.copy()
    def state():
        m = np.nonzero(a[frame.eu] != a[frame.ev])[0]
        return (angle_of(frame.mid[m[0]], frame.mid[m[1]]) if m.size == 2 else np.nan)
    vals, ts = [state()], [0]
    for t, v in events:
        a[v] = 1 - a[v]
        vals.append(state())
        ts.append(int(t))
    w = np.diff(np.asarray(ts + [T + 1]))
    vals = np.asarray(vals)
    ok = np.isfinite(vals)
    mean = float(np.sum(vals[ok] * w[ok]) / np.sum(w[ok])) if ok.any() else np.nan
    return mean, vals[-1]


# --- C3: k = 4, the pair proposal (slow_reversible_propose, grid_chain_sec11.py:117-130) -------
C3_STATS = ("cut", "nb", "pop0", "wait", "mean_cut", "mean_nb", "perim0", "radius0")
C3_K, C3_PCT = 4, 0.05


def setup_c3():
    spec = G.sec11_graph()
    a0 = spec.assignment_array(G.quadrant_plan(spec.nodes), list(range(C3_K)))
    _, (lo, hi) = G.population_bounds(spec.n, C3_K, C3_PCT)
    return spec, a0, lo, hi


def summarize_c3(spec, finals, waits, sum_cut, sum_nb, T):
    """The C3 fixture's statistics (tests/golden/make_native.py one_c3) from end states and tallies."""
    import sys
    sys.path.insert(0, GOLD)
    from make_native import c3_shape
    out = {s: [] for s in C3_STATS}
    for a in finals:
        c, b, pops = G.cut_and_boundary(spec, a)
        p0, r0 = c3_shape(spec, a)
        for key, val in (("cut", c), ("nb", b), ("pop0", pops[0]), ("perim0", p0), ("radius0", r0)):
            out[key].append(val)
    out["wait"] = list(waits)
    out["mean_cut"] = np.asarray(sum_cut, float) / (T + 1)
    out["mean_nb"] = np.asarray(sum_nb, float) / (T + 1)
    return {key: np.asarray(v, float) for key, v in out.items()}


def assert_same_distribution_c3(fix, bi, got, label):
    for s in C3_STATS:
        ref = fix[f"b{bi}_{s}"]
        p = ks_2samp(ref, np.asarray(got[s], float)).pvalue
        assert p > P_MIN, (label, s, p, ref.mean(), np.mean(got[s]))


@pytest.mark.parametrize("bi", [0, 1])
def test_c3_canonical_oracle_matches_native_rng_pair(cref, bi):
    """C3 under the canonical PAIR stream (C oracle) against the reference's pair proposal under
    CPython's MT (native_rng_c3.npz): KS on cut, boundary, population and shape statistics."""
    fix = fixture("c3")
    T, base = int(fix["T"]), float(fix["bases"][bi])
    spec, a0, lo, hi = setup_c3()
    finals, waits, sc, sn = [], [], [], []
    for c in range(400):
        r = cref.run(spec, a0, base=base, pop_lo=lo, pop_hi=hi, seed=0xC3, chain_id=c, n_steps=T, k=C3_K,
                     labels=list(range(C3_K)), proposal=1, log1mp=G.log1mp_table(spec.n, C3_K))
        finals.append(r["final"])
        waits.append(r["stats"]["wait_cur"])
        sc.append(r["stats"]["sum_cut"])
        sn.append(r["stats"]["sum_nb"])
    assert_same_distribution_c3(fix, bi, summarize_c3(spec, finals, waits, sc, sn, T), "C oracle c3")


@pytest.mark.parametrize("stream", [0, 1], ids=["node", "band"])
@pytest.mark.parametrize("cfg,bi", CASES)
def test_canonical_oracle_matches_native_rng(cref, cfg, bi, stream):
    """Both node streams (flipref.h FR_STREAM_NODE / FR_STREAM_BAND) sample the reference's
    chain: uniform over b_nodes, whatever superset the draws range over."""
    fix = fixture(cfg)
    T, base = int(fix["T"]), float(fix["bases"][bi])
    spec, a0, lo, hi = setup(cfg)
    from oracle.flipref import events_from_trace
    frame = G.slope_frame(spec, "sec11") if cfg != "c1" else None
    finals, waits, sc, sn, am, ae = [], [], [], [], [], []
    for c in range(600 if T <= 2000 else 150):
        r = cref.run(spec, a0, base=base, pop_lo=lo, pop_hi=hi, seed=0xD15, chain_id=c, n_steps=T,
                     log1mp=G.log1mp_table(spec.n, 2), trace_cap=64 * T if frame is not None else 0,
                     stream=stream)
        finals.append(r["final"])
        waits.append(r["stats"]["wait_cur"])
        sc.append(r["stats"]["sum_cut"])
        sn.append(r["stats"]["sum_nb"])
        if frame is not None:
            assert len(r["trace"]) < 64 * T
            ev = events_from_trace(r["trace"])
            m, e = shape_from_events(spec, frame, a0, ev[:, :2], T)
            am.append(m)
            ae.append(e)
    got = summarize(spec, finals, waits, sc, sn, T)
    if frame is not None:
        got["angle_mean"], got["angle_end"] = np.asarray(am), np.asarray(ae)
    assert_same_distribution(fix, bi, got, f"C oracle {cfg} stream {stream}")
