"""The device, on every reference configuration, against the reference's own outputs.

All 174 configurations of the two sweeps (grid_chain_sec11.py:182-184, Frankenstein_chain.py:
182-184), eight chains each (Philox chain ids 0..7 per configuration), 100,000 yields
(total_steps=100000, :342) on the HIP kernel: the wait.txt sums (:410-411) per (graph, base,
pop) and per (graph, base), and the final |cut| / |B| per base against the decoded end2 states
(:440-450) -- the same pins the C oracle meets with two seeds in test_oracle_golden.py
(tests/reference_pin.py)."""
import numpy as np
import pytest

import reference_pin as RP
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

pytestmark = pytest.mark.gpu

SEEDS = 8


def test_device_reproduces_every_reference_artifact(gpu):
    cfgs = RP.configs()
    assert len(cfgs) == 174
    results = []
    for tag in ("sec11", "frank"):
        spec = RP.spec_of(tag)
        fg = FlipGraph(spec)
        for pct in sorted({c[3] for c in cfgs if c[0] == tag}):
            group = [c for c in cfgs if c[0] == tag and c[3] == pct]
            rows = [(c, s) for c in group for s in range(SEEDS)]
            inits = np.stack([RP.start_plan(spec, tag, c[1]) for c, _ in rows])
            bases = np.asarray([c[2] for c, _ in rows])
            _, (lo, hi) = G.population_bounds(spec.n, 2, pct)
            run = FlipRun(fg, inits, RunConfig(seed=0x9E1 + int(1000 * pct), pop_lo=lo, pop_hi=hi), bases=bases)
            run.steps(99999)
            st = run.stats()
            assert (st["steps"] == 99999).all() and not st["stuck"].any()
            for i, (c, _) in enumerate(rows):
                results.append((c, int(st["sum_wait"][i]), int(st["cut"][i]), int(st["nb"][i])))
            run.close()
    worst = RP.check(results)
    print("reference pin (device, %d runs): max |z| %.2f, min KS p %.3g" % (len(results), worst["max_abs_z"],
                                                                           worst["min_ks_p"]))
