"""The k = 2 full-diagnostics tallies through the tally log and through its overflow path.

The flip kernel writes each queued state's per-yield tallies (the reference loop body's
histograms, cut_times, num_flips / part_sum / last_flipped and their corrected companions,
grid_chain_sec11.py:367-400) as 16-byte entries to a per-chain log that tally_reduce_kernel
applies after the launch; a chain whose log is full applies the rest of its launch's tallies with
global atomics (the path a device short of memory takes).  FC_FLAG_TALLY_LOG_SMALL caps the log
at 64 entries, so every active chain overflows it in each launch: the arrays must equal those of
the default run bit for bit (the default run itself is pinned to the C oracle in
tests/test_corrected_stats_gpu.py and tests/test_production_gpu.py)."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

pytestmark = pytest.mark.gpu

DIAG = (_lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS
        | _lib.FC_DIAG_FLIPS_EXACT | _lib.FC_DIAG_SERIES)


def _run(spec, flags, launches, steps):
    n_chains = 64
    inits = np.stack([spec.assignment_array(G.sec11_plan(c % 3, spec.nodes), [-1, 1]) for c in range(n_chains)])
    bases = np.asarray([G.SEC11_BASES[c % 10] for c in range(n_chains)])
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), 2, 0.1)
    cfg = RunConfig(seed=77, pop_lo=lo, pop_hi=hi, diag_mask=DIAG, event_cap=launches * steps + 1, flags=flags)
    run = FlipRun(FlipGraph(spec), inits, cfg, bases=bases)
    for _ in range(launches):
        run.steps(steps)
    return run


@pytest.mark.parametrize("launches", [1, 3])
def test_tally_log_overflow_path_equals_log(gpu, sec11, launches):
    a = _run(sec11, 0, launches, 3000)
    b = _run(sec11, _lib.FC_FLAG_TALLY_LOG_SMALL, launches, 3000)
    sa, sb = a.stats(), b.stats()
    assert np.array_equal(sa["steps"], sb["steps"]) and np.array_equal(sa["accepted"], sb["accepted"])
    assert int(sa["accepted"].min()) > 64  # every chain overflowed the small log
    for x, y in zip(a.hist(), b.hist()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.cut_times(), b.cut_times())
    for x, y in zip(a.flips(), b.flips()):
        assert np.array_equal(x, y)
    for x, y in zip(a.flips_exact(), b.flips_exact()):
        assert np.array_equal(x, y)
    for c in (0, 17, 63):  # the event log does not go through the tally log
        assert np.array_equal(a.events(c), b.events(c))
