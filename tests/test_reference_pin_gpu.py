"""The device, on every reference configuration, against the reference's own outputs.

All 174 configurations of the two sweeps (grid_chain_sec11.py:182-184, Frankenstein_chain.py:
182-184), eight replicas each, 100,000 yields (total_steps=100000, :342), run through the
product sweep runner (flipcomplexityempirical_amd.sweep: one launch per graph, per-chain bases
and population bounds): the wait.txt sums (:410-411) per (graph, base, pop) and per (graph,
base), and the final |cut| / |B| per base against the decoded end2 states (:440-450) -- the same
pins the C oracle meets with two seeds in test_oracle_golden.py (tests/reference_pin.py)."""
import pytest

import reference_pin as RP
from flipcomplexityempirical_amd.sweep import Sweep, SweepConfig

pytestmark = pytest.mark.gpu

REPLICAS = 8


def test_device_reproduces_every_reference_artifact(gpu):
    cfgs = RP.configs()
    assert len(cfgs) == 174
    results = []
    for tag in ("sec11", "frank"):
        mine = [c for c in cfgs if c[0] == tag]
        sw = Sweep(tag, replicas=REPLICAS, total_steps=100000, seed=0x9E1, series=False, corrected=False,
                   configs=[SweepConfig(tag, al, base, pct) for (_, al, base, pct, _) in mine]).run()
        st = sw._run.stats()
        assert (st["steps"] == 99999).all() and not st["stuck"].any()
        for g in range(sw.n_total):
            c = mine[g % sw.n_configs]
            assert sw.config_of(g).key == c[4]
            results.append((c, int(st["sum_wait"][g]), int(st["cut"][g]), int(st["nb"][g])))
        sw.close()
    worst = RP.check(results)
    print("reference pin (device sweep, %d runs): max |z| %.2f, min KS p %.3g" % (len(results), worst["max_abs_z"],
                                                                                 worst["min_ks_p"]))
