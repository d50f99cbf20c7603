"""Generate tests/golden/native_rng_c1.npz: end-of-run statistics of the reference's flip step
under its native random streams (oracle.flipref.NativeRngChain: CPython MT random.choice /
random.random, numpy legacy geometric), for the distributional (KS) checks of the canonical
Philox stream (tests/test_distribution.py, tests/test_distribution_gpu.py).

native_rng_c1.npz: config C1 of BASELINE.json: 10x10 grid, k = 2, plan x[0] >= 5, pop
tolerance 0.1, bases 1 and mu = 2.63815853 (grid_chain_sec11.py:33); 400 chains per base,
T = 2000 steps each, chain i seeded 1000 + i.
native_rng_sec11.npz: the sec11 lattice of the headline (grid_chain_sec11.py:186-260),
alignment-2 plan, pop tolerance 0.1, bases 0.8 and mu; 200 chains per base, T = 1000 steps;
plus the district-shape statistics of the driver's slope / angle lines (:371-394): each
chain's mean angle over the yields with exactly two frame cut edges, the end state's angle,
and the fraction of such yields.
native_rng_sec11_long.npz: as sec11 with the alignment-0 plan, the extreme bases 0.2 and 10
and T = 10,000 steps (200 chains per base): long chains far from the start state.
native_rng_c3.npz: BASELINE config C3 -- the sec11 lattice, k = 4 quadrant plan, pop
tolerance 0.05 -- under the reference's pair proposal ``slow_reversible_propose``
(grid_chain_sec11.py:117-130, pairs :151-153; NativeRngChain(pair=True)), bases mu and 1;
256 chains per base, T = 4000 steps, chain i seeded 5000 + i.  Statistics: the end state's
|cut|, |B|, district-0 population, wait, the time-averaged |cut| and |B|, and two district-shape
statistics of the end state: district 0's perimeter (cut edges with an endpoint in it) and the
distance of its centroid from the lattice centre (C3_SHAPE).
Run: python tests/golden/make_native.py [c1 sec11 sec11_long c3]  (c1 + sec11 about 1.5 min on
8 cores, sec11_long about 10 min, c3 about 4 min)."""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CONFIGS = {"c1": ([1.0, 2.63815853], 400, 2000), "sec11": ([0.8, 2.63815853], 200, 1000),
           "sec11_long": ([0.2, 10.0], 200, 10000), "c3": ([2.63815853, 1.0], 256, 4000)}
ALIGNMENT = {"sec11": 2, "sec11_long": 0}  # sec11 start plan (grid_chain_sec11.py:195-214)


SHAPE = ("angle_mean", "angle_end", "frame2_frac")  # sec11 only (the reference's frame)


def _frame_angle(state, frame_edges):
    """The driver's shape lines (grid_chain_sec11.py:371-394) on the reference's own
    ``boundary_slope`` filter (:55-78): (number of frame cut edges, angle when exactly two --
    the only case whose value does not depend on CPython's set order)."""
    from oracle.flipref import slope_angle
    a = state.assignment
    cut = [e for e in frame_edges if a[e[0]] != a[e[1]]]
    if len(cut) != 2:
        return len(cut), float("nan")
    return 2, slope_angle(cut)[1]


C3_SHAPE = ("perim0", "radius0")


def c3_shape(spec, assign):
    """District 0's perimeter and centroid distance from the lattice centre, from a district-id
    array (the C3 shape statistics; tests/test_distribution.py uses the same function)."""
    e = spec.edges()
    a = np.asarray(assign)
    cut = a[e[:, 0]] != a[e[:, 1]]
    perim0 = int(np.count_nonzero(cut & ((a[e[:, 0]] == 0) | (a[e[:, 1]] == 0))))
    xy = np.asarray(spec.nodes, dtype=np.float64)
    c = xy[a == 0].mean(axis=0) - xy.mean(axis=0)
    return perim0, float(np.hypot(c[0], c[1]))


def one_c3(base, i, T):
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import NativeRngChain
    spec = G.sec11_graph()
    plan = G.quadrant_plan(spec.nodes)
    k = 4
    (lo, hi), _ = G.population_bounds(spec.n, k, 0.05)
    ch = NativeRngChain(spec, plan, base=base, pop_bounds=(lo, hi), seed=5000 + i,
                        log1mp=G.log1mp_table(spec.n, k), pair=True)
    ch.run(T)
    s = ch.state
    return (len(s["cut_edges"]), len(s["b_nodes"]), s["population"][0], ch.wait,
            ch.stats["sum_cut"] / (T + 1), ch.stats["sum_nb"] / (T + 1)) + c3_shape(spec, ch.assignment_ids())


def one(args):
    cfg, base, i, T = args
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import NativeRngChain, boundary_slope
    if cfg == "c3":
        return one_c3(base, i, T)
    if cfg == "c1":
        spec = G.grid_graph(10, 10)
        plan = G.threshold_plan(spec.nodes, 0, 5)
    else:
        spec = G.sec11_graph()
        plan = G.sec11_plan(ALIGNMENT[cfg], spec.nodes)
    (lo, hi), _ = G.population_bounds(spec.n, 2, 0.1)
    ch = NativeRngChain(spec, plan, base=base, pop_bounds=(lo, hi), seed=1000 + i, log1mp=G.log1mp_table(spec.n, 2))
    shape = ()
    if cfg == "c1":
        ch.run(T)
    else:
        # every edge boundary_slope can return (its filter over all edges), then per yield
        frame = boundary_slope({tuple(sorted(e)) for e in spec.nx_graph.edges})
        n2, ang = _frame_angle(ch.state, frame)
        ang_sum, n_two = (ang if n2 == 2 else 0.0), int(n2 == 2)
        for _ in range(T):
            acc0 = ch.stats["accepted"]
            ch.step()
            if ch.stats["accepted"] != acc0:
                n2, ang = _frame_angle(ch.state, frame)
            if n2 == 2:
                ang_sum += ang
                n_two += 1
        shape = (ang_sum / n_two if n_two else float("nan"), ang if n2 == 2 else float("nan"), n_two / (T + 1))
    s = ch.state
    return (len(s["cut_edges"]), len(s["b_nodes"]), s["population"][1], ch.wait,
            ch.stats["sum_cut"] / (T + 1), ch.stats["sum_nb"] / (T + 1)) + shape


def main(which=None):
    for cfg, (bases, M, T) in CONFIGS.items():
        if which and cfg not in which:
            continue
        out = {"T": np.int64(T), "bases": np.asarray(bases)}
        with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            for bi, b in enumerate(bases):
                r = np.asarray(list(ex.map(one, [(cfg, b, i, T) for i in range(M)])), dtype=np.float64)
                names = (("cut", "nb", "pop0", "wait", "mean_cut", "mean_nb") + C3_SHAPE if cfg == "c3" else
                         ("cut", "nb", "pop1", "wait", "mean_cut", "mean_nb") + (SHAPE if cfg != "c1" else ()))
                for j, name in enumerate(names):
                    out[f"b{bi}_{name}"] = r[:, j]
        np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"native_rng_{cfg}.npz"), **out)


if __name__ == "__main__":
    main(sys.argv[1:])
