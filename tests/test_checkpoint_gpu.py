"""Checkpoint / resume through the C-ABI (fc_run_checkpoint / fc_run_restore): a run
checkpointed mid-way and restored into a fresh run with the same graph and parameters continues
bit for bit -- counters, sums, waits, state, populations, histograms, cut_times, flips and the
series event log -- for the k = 2 kernel, the k > 2 kernel with its district-graph tables, and
ReCom."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

pytestmark = pytest.mark.gpu

ALL = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS | _lib.FC_DIAG_SERIES
KEYS = ("steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb", "sum_wait",
        "sum_cut2", "sum_nb2", "wait_cur", "cut", "nb", "last_flip", "hit_time", "events", "series_t0")


def _same(a, b, diag=True, k=2):
    sa, sb = a.stats(), b.stats()
    for key in KEYS:
        assert np.array_equal(sa[key], sb[key]), key
    assert np.array_equal(a.state(), b.state())
    assert np.array_equal(a.pops(), b.pops())
    if diag:
        for x, y in zip(a.hist(), b.hist()):
            assert np.array_equal(x, y)
        assert np.array_equal(a.cut_times(), b.cut_times())
        for x, y in zip(a.flips(), b.flips()):
            assert np.array_equal(x, y)
        for c in range(a.n_chains):
            assert np.array_equal(a.events(c), b.events(c))


@pytest.mark.parametrize("case", ["k2_sec11", "k4_sec11"])
def test_checkpoint_resume_bit_exact(gpu, sec11, case):
    if case == "k2_sec11":
        k, labels, prop, pct = 2, (-1, 1), _lib.FC_PROPOSE_BI_SIGN, 0.1
        inits = np.stack([sec11.assignment_array(G.sec11_plan(c % 3, sec11.nodes), [-1, 1]) for c in range(24)])
        bases = np.asarray([G.SEC11_BASES[c % 10] for c in range(24)])
    else:
        k, labels, prop, pct = 4, (0, 1, 2, 3), _lib.FC_PROPOSE_PAIR, 0.05
        inits = np.stack([sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(4)))] * 16)
        bases = np.asarray([[0.5, 1.0, G.SEC11_MU, 4.0][c % 4] for c in range(16)])
    _, (lo, hi) = G.population_bounds(sec11.n, k, pct)
    fg = FlipGraph(sec11)
    cfg = RunConfig(k=k, labels=labels, proposal=prop, seed=77, pop_lo=lo, pop_hi=hi, diag_mask=ALL,
                    event_cap=20000, hit_lo=0, hit_hi=30)
    a = FlipRun(fg, inits, cfg, bases=bases)
    a.steps(1700)
    blob = a.checkpoint()
    a.steps(2300)
    b = FlipRun(fg, inits, cfg, bases=bases)
    b.steps(11)  # diverge first: the restore must overwrite everything that matters
    b.restore(blob)
    b.steps(2300)
    _same(a, b, k=k)
    # a restore into a run with other parameters is refused
    other = FlipRun(fg, inits, RunConfig(k=k, labels=labels, proposal=prop, seed=77, pop_lo=lo, pop_hi=hi),
                    bases=bases)
    with pytest.raises(ValueError):
        other.restore(blob)
    # a blob written under another random-stream version (the round-3 magic, or a changed version
    # field) is refused, never continued on this build's stream
    assert blob[:8] == b"FCCKPT03"
    with pytest.raises(ValueError, match="earlier random stream"):
        b.restore(b"FCCKPT02" + blob[8:])
    with pytest.raises(ValueError, match="random-stream version"):
        b.restore(blob[:8] + (2).to_bytes(4, "little") + blob[12:])


def test_checkpoint_resume_recom(gpu, sec11):
    _, (lo, hi) = G.population_bounds(sec11.n, 2, 0.1)
    inits = np.stack([sec11.assignment_array(G.sec11_plan(c % 3, sec11.nodes), [-1, 1]) for c in range(8)])
    cfg = RunConfig(proposal=_lib.FC_PROPOSE_RECOM, seed=5, pop_lo=lo, pop_hi=hi, base=1.0,
                    recom_pop_target=sec11.n / 2, recom_epsilon=0.1, recom_node_repeats=2)
    fg = FlipGraph(sec11)
    a = FlipRun(fg, inits, cfg)
    a.steps(30)
    blob = a.checkpoint()
    a.steps(40)
    b = FlipRun(fg, inits, cfg)
    b.restore(blob)
    b.steps(40)
    _same(a, b, diag=False)
