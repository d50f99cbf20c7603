"""The k = 2 full-diagnostics instance applies its per-flip tallies from the deferred queue
(fc_flip2.hip tally_flush; DESIGN §4 "Batch (k = 2)"): queue lengths 1 (a drain at every batch
that accepts), 5 and 64, launches of uneven length (a queued state's run crosses batches and
launches), with and without geometric waits.  The |cut| / |B| histograms, cut_times, the quirk
and corrected flip tallies, the accepted-flip log, the hitting time and the scalars match the C
oracle bit for bit (the driver's loop body, grid_chain_sec11.py:367-400).  No chain is traced and
there is no tape, so the kernel is the diagnostics instance without XTRA code."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
from oracle.flipref import events_from_trace, hitting_time, yield_series

pytestmark = pytest.mark.gpu

TALLIES = (_lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS | _lib.FC_DIAG_FLIPS_EXACT |
           _lib.FC_DIAG_SERIES)
LAUNCHES = (7, 300, 1693)


@pytest.mark.parametrize("wait_queue,waits", [(1, True), (5, True), (64, True), (64, False)])
def test_k2_tally_queue(gpu, cref, sec11, wait_queue, waits):
    n_chains, steps, seed = 12, sum(LAUNCHES), 37
    bases = np.asarray([[0.1, 0.5, 1.0, G.SEC11_MU, 4.0, 10.0][c % 6] for c in range(n_chains)])
    inits = np.stack([sec11.assignment_array(G.sec11_plan(c % 3, sec11.nodes), [-1, 1]) for c in range(n_chains)])
    _, (lo, hi) = G.population_bounds(int(sec11.pop.sum()), 2, 0.1)
    x0 = [G.cut_and_boundary(sec11, inits[c])[0] for c in range(n_chains)]
    hit = (min(x0) + 25, 10 ** 6)
    diag = TALLIES | (_lib.FC_DIAG_WAIT if waits else 0)
    cfg = RunConfig(k=2, labels=(-1, 1), proposal=_lib.FC_PROPOSE_BI_SIGN, seed=seed, pop_lo=lo, pop_hi=hi,
                    diag_mask=diag, event_cap=steps + 1, hit_lo=hit[0], hit_hi=hit[1],
                    tune={"wait_queue": wait_queue})
    run = FlipRun(FlipGraph(sec11), inits, cfg, bases=bases)
    for n in LAUNCHES:
        run.steps(n)
    assert run.kernel_name().startswith("fc::flip2_kernel<8, 4, true, false, false, false>"), run.kernel_name()
    st = run.stats()
    ch, nh = run.hist()
    ct = run.cut_times()
    nf, ps, lf = run.flips()
    xf, xo, xl = run.flips_exact()
    keys = ["steps", "accepted", "sum_cut", "sum_nb", "cut", "nb"] + (["sum_wait", "wait_cur"] if waits else [])
    for c in range(n_chains):
        ref = cref.run(sec11, inits[c], base=float(bases[c]), pop_lo=lo, pop_hi=hi, seed=seed, chain_id=c,
                       n_steps=steps, log1mp=G.log1mp_table(sec11.n, 2), trace_cap=400000, want_hist=True,
                       want_edges=True, want_flips=True, want_exact_flips=True)
        for key in keys:
            assert int(st[key][c]) == int(ref["stats"][key]), (wait_queue, c, key)
        assert np.array_equal(ch[c], ref["cut_hist"]) and np.array_equal(nh[c], ref["nb_hist"]), c
        assert np.array_equal(ct[c], ref["cut_times"]), c
        assert np.array_equal(nf[c], ref["num_flips"]) and np.array_equal(ps[c], ref["part_sum"]), c
        assert np.array_equal(lf[c], ref["last_flipped"]), c
        assert np.array_equal(xf[c], ref["flip_count"]) and np.array_equal(xo[c], ref["occupancy"]), c
        assert np.array_equal(xl[c], ref["last_accept"]), c
        ev = run.events(c)
        exp = events_from_trace(ref["trace"])
        assert len(ev) == len(exp) == st["events"][c], c
        got = np.stack([ev["t"], ev["v"], ev["cut"], ev["nb"], ev["target"]], axis=1).astype(np.int64)
        assert np.array_equal(got, exp), c
        assert st["hit_time"][c] == hitting_time(yield_series(ref["trace"], x0[c]), *hit), c
