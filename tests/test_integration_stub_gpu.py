"""The reference's whole sec11 sweep (grid_chain_sec11.py:182-184: 5 population tolerances x
10 bases x 3 alignments = 150 configurations) as ONE fc_run -- per-chain bases and per-chain
population bounds (fc_params.chain_pop_bounds) -- through INTEGRATION.md's ctypes stub, executed
verbatim, and through FlipRun with every per-yield tally on.  Each configuration's outputs
(wait sums, cut_times, num_flips / part_sum / last_flipped, histograms), grouped by
configuration with distributed.local_statistics, must be identical to that configuration run
alone, and sampled chains match the C oracle."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib, distributed as D, graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
from test_integration_stub import stub_namespace

pytestmark = pytest.mark.gpu

PER = 2          # chains per configuration
STEPS = 1500
SEED = 31
FULL = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS


def sweep(spec):
    """Chain c runs configuration c // PER; configurations in the reference's loop order."""
    cfgs = [(p, b, al) for p in G.SEC11_POPS for b in G.SEC11_BASES for al in (2, 1, 0)]
    plans = {al: spec.assignment_array(G.sec11_plan(al, spec.nodes), [-1, 1]) for al in range(3)}
    inits, bases, bounds = [], [], []
    for p, b, al in cfgs:
        _, (lo, hi) = G.population_bounds(spec.n, 2, p)
        for _ in range(PER):
            inits.append(plans[al])
            bases.append(b)
            bounds.append((lo, hi))
    groups = np.arange(len(cfgs) * PER) // PER
    return cfgs, np.stack(inits), np.asarray(bases), np.asarray(bounds, dtype=np.int64), groups


def test_stub_runs_the_sweep(gpu, cref, sec11):
    ns = stub_namespace()
    lib = ns["load"](_lib.lib_path())
    cfgs, inits, bases, bounds, _ = sweep(sec11)
    stats = ns["run_sweep"](lib, sec11.n, sec11.row_ptr, sec11.col_idx, sec11.pop,
                            np.asarray(sec11.pos).reshape(-1), inits, bases, bounds, STEPS, seed=SEED)
    got = {f: np.array([getattr(s, f) for s in stats]) for f in ("steps", "proposals", "accepted", "sum_wait",
                                                                "inv_pop", "cut", "nb")}
    assert (got["steps"] == STEPS).all()
    assert got["inv_pop"][bounds[:, 0] == bounds[:, 0].max()].sum() > 0   # the 0.01 tolerance bites
    fr = FlipRun(FlipGraph(sec11), inits, RunConfig(seed=SEED, pop_lo=0, pop_hi=10 ** 6), bases=bases,
                 pop_bounds=bounds)
    fr.steps(STEPS)
    st = fr.stats()
    for f, v in got.items():
        assert np.array_equal(v, st[f]), f
    for c in range(0, len(inits), 37):   # sampled chains against the C oracle
        ref = cref.run(sec11, inits[c], base=float(bases[c]), pop_lo=int(bounds[c, 0]), pop_hi=int(bounds[c, 1]),
                       seed=SEED, chain_id=c, n_steps=STEPS, log1mp=G.log1mp_table(sec11.n, 2))
        for f in ("steps", "proposals", "accepted", "sum_wait", "inv_pop", "cut", "nb"):
            assert int(got[f][c]) == int(ref["stats"][f]), (c, f)


def _arrays(run):
    out = {}
    out["cut_hist"], out["nb_hist"] = run.hist()
    out["cut_times"] = run.cut_times()
    out["num_flips"], out["part_sum"], out["last_flipped"] = run.flips()
    return out


def test_sweep_grouped_equals_each_configuration_alone(gpu, sec11):
    cfgs, inits, bases, bounds, groups = sweep(sec11)
    fg = FlipGraph(sec11)
    cfg = RunConfig(seed=SEED, diag_mask=FULL, pop_lo=0, pop_hi=10 ** 6)
    whole = FlipRun(fg, inits, cfg, bases=bases, pop_bounds=bounds)
    whole.steps(STEPS)
    red = D.local_statistics(whole.stats(), groups, len(cfgs), _arrays(whole))
    whole.close()
    for i, (p, b, al) in enumerate(cfgs):
        sl = slice(i * PER, (i + 1) * PER)
        lo, hi = (int(x) for x in bounds[i * PER])
        alone = FlipRun(fg, inits[sl], RunConfig(seed=SEED, diag_mask=FULL, pop_lo=lo, pop_hi=hi,
                                                 chain_id_offset=i * PER), bases=bases[sl])
        alone.steps(STEPS)
        one = D.local_statistics(alone.stats(), np.zeros(PER, dtype=np.int64), 1, _arrays(alone))
        alone.close()
        for name, arr in one.items():
            assert np.array_equal(red[name][i], arr[0]), (i, (p, b, al), name)
