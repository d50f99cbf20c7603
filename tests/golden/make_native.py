"""Generate tests/golden/native_rng_c1.npz: end-of-run statistics of the reference's flip step
under its native random streams (oracle.flipref.NativeRngChain: CPython MT random.choice /
random.random, numpy legacy geometric), for the distributional (KS) checks of the canonical
Philox stream (tests/test_distribution.py, tests/test_distribution_gpu.py).

Config C1 of BASELINE.json: 10x10 grid, k = 2, plan x[0] >= 5, pop tolerance 0.1, bases 1 and
mu = 2.63815853 (grid_chain_sec11.py:33); 400 chains per base, T = 2000 steps each, chain i
seeded 1000 + i.  Run: python tests/golden/make_native.py  (about 30 s on 8 cores)."""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

BASES = [1.0, 2.63815853]
M, T = 400, 2000


def one(args):
    base, i = args
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import NativeRngChain
    spec = G.grid_graph(10, 10)
    plan = G.threshold_plan(spec.nodes, 0, 5)
    (lo, hi), _ = G.population_bounds(100, 2, 0.1)
    ch = NativeRngChain(spec, plan, base=base, pop_bounds=(lo, hi), seed=1000 + i, log1mp=G.log1mp_table(100, 2))
    ch.run(T)
    s = ch.state
    return (len(s["cut_edges"]), len(s["b_nodes"]), s["population"][1], ch.wait,
            ch.stats["sum_cut"] / (T + 1), ch.stats["sum_nb"] / (T + 1))


def main():
    out = {"T": np.int64(T), "bases": np.asarray(BASES)}
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for bi, b in enumerate(BASES):
            r = np.asarray(list(ex.map(one, [(b, i) for i in range(M)])), dtype=np.float64)
            for j, name in enumerate(("cut", "nb", "pop1", "wait", "mean_cut", "mean_nb")):
                out[f"b{bi}_{name}"] = r[:, j]
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "native_rng_c1.npz"), **out)


if __name__ == "__main__":
    main()
