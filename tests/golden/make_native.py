"""Generate tests/golden/native_rng_c1.npz: end-of-run statistics of the reference's flip step
under its native random streams (oracle.flipref.NativeRngChain: CPython MT random.choice /
random.random, numpy legacy geometric), for the distributional (KS) checks of the canonical
Philox stream (tests/test_distribution.py, tests/test_distribution_gpu.py).

native_rng_c1.npz: config C1 of BASELINE.json: 10x10 grid, k = 2, plan x[0] >= 5, pop
tolerance 0.1, bases 1 and mu = 2.63815853 (grid_chain_sec11.py:33); 400 chains per base,
T = 2000 steps each, chain i seeded 1000 + i.
native_rng_sec11.npz: the sec11 lattice of the headline (grid_chain_sec11.py:186-260),
alignment-2 plan, pop tolerance 0.1, bases 0.8 and mu; 200 chains per base, T = 1000 steps.
Run: python tests/golden/make_native.py  (about 1.5 min on 8 cores)."""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CONFIGS = {"c1": ([1.0, 2.63815853], 400, 2000), "sec11": ([0.8, 2.63815853], 200, 1000)}


def one(args):
    cfg, base, i, T = args
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import NativeRngChain
    if cfg == "c1":
        spec = G.grid_graph(10, 10)
        plan = G.threshold_plan(spec.nodes, 0, 5)
    else:
        spec = G.sec11_graph()
        plan = G.sec11_plan(2, spec.nodes)
    (lo, hi), _ = G.population_bounds(spec.n, 2, 0.1)
    ch = NativeRngChain(spec, plan, base=base, pop_bounds=(lo, hi), seed=1000 + i, log1mp=G.log1mp_table(spec.n, 2))
    ch.run(T)
    s = ch.state
    return (len(s["cut_edges"]), len(s["b_nodes"]), s["population"][1], ch.wait,
            ch.stats["sum_cut"] / (T + 1), ch.stats["sum_nb"] / (T + 1))


def main(which=None):
    for cfg, (bases, M, T) in CONFIGS.items():
        if which and cfg not in which:
            continue
        out = {"T": np.int64(T), "bases": np.asarray(bases)}
        with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            for bi, b in enumerate(bases):
                r = np.asarray(list(ex.map(one, [(cfg, b, i, T) for i in range(M)])), dtype=np.float64)
                for j, name in enumerate(("cut", "nb", "pop1", "wait", "mean_cut", "mean_nb")):
                    out[f"b{bi}_{name}"] = r[:, j]
        np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"native_rng_{cfg}.npz"), **out)


if __name__ == "__main__":
    main(sys.argv[1:])
