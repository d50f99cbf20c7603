"""GPU parity of the corrected companions (FC_DIAG_FLIPS_EXACT, fc_run_read_wait_expected;
SURVEY App. A.6) beside the quirk forms: k = 2 (flip2_kernel, segment-parallel commits, chunked
launches) and k = 4 PAIR (flip_kernel) against the C oracle, bit-exact; the expected-wait sum
against the oracle's |B| histogram; checkpoint / restore carries the new accumulators."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

pytestmark = pytest.mark.gpu

DIAG = (_lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_FLIPS | _lib.FC_DIAG_FLIPS_EXACT)


def _run(spec, inits, bases, k, labels, proposal, pct, steps, chunks, seed=31):
    fg = FlipGraph(spec)
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    cfg = RunConfig(k=k, labels=tuple(labels), proposal=proposal, seed=seed, pop_lo=lo, pop_hi=hi,
                    diag_mask=DIAG)
    run = FlipRun(fg, inits, cfg, bases=bases)
    per = steps // chunks
    for i in range(chunks):
        run.steps(per if i < chunks - 1 else steps - per * (chunks - 1))
    return run, lo, hi


def _check(cref, spec, run, inits, bases, k, labels, proposal, lo, hi, steps, seed=31):
    xf, xo, xl = run.flips_exact()
    nf, ps, lf = run.flips()
    _, nh = run.hist()
    we = run.wait_expected()
    M = float(spec.n) ** k - 1.0
    for c in range(inits.shape[0]):
        ref = cref.run(spec, inits[c], base=float(bases[c]), pop_lo=lo, pop_hi=hi, seed=seed, chain_id=c,
                       n_steps=steps, k=k, labels=list(labels), log1mp=G.log1mp_table(spec.n, k),
                       want_hist=True, want_flips=True, want_exact_flips=True, proposal=proposal)
        assert np.array_equal(xf[c], ref["flip_count"]), c
        assert np.array_equal(xo[c], ref["occupancy"]), c
        assert np.array_equal(xl[c], ref["last_accept"]), c
        assert np.array_equal(nf[c], ref["num_flips"]) and np.array_equal(ps[c], ref["part_sum"]), c
        assert np.array_equal(lf[c], ref["last_flipped"]), c
        assert int(xf[c].sum()) == int(run.stats()["accepted"][c])
        h = ref["nb_hist"]
        assert np.array_equal(nh[c], h)
        b = np.arange(spec.n + 1)[1:]
        want = float((h[1:] * (M / b - 1.0)).sum())
        assert we[c] == pytest.approx(want, rel=1e-12), c


@pytest.mark.parametrize("chunks", [1, 3])
def test_k2_corrected_flips(gpu, cref, sec11, chunks):
    n_chains, steps = 20, 3000
    inits = np.stack([sec11.assignment_array(G.sec11_plan(c % 3, sec11.nodes), [-1, 1]) for c in range(n_chains)])
    bases = np.asarray([G.SEC11_BASES[c % 10] for c in range(n_chains)])
    run, lo, hi = _run(sec11, inits, bases, 2, (-1, 1), _lib.FC_PROPOSE_BI_SIGN, 0.1, steps, chunks)
    _check(cref, sec11, run, inits, bases, 2, (-1, 1), 0, lo, hi, steps)


def test_k4_corrected_flips(gpu, cref, sec11):
    k, n_chains, steps = 4, 12, 2000
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    inits = np.stack([a0] * n_chains)
    bases = np.asarray([[G.SEC11_MU, 1.0, 0.5, 4.0][c % 4] for c in range(n_chains)])
    labels = (3, -2, 7, 0)
    run, lo, hi = _run(sec11, inits, bases, k, labels, _lib.FC_PROPOSE_PAIR, 0.05, steps, 2)
    _check(cref, sec11, run, inits, bases, k, labels, 1, lo, hi, steps)


def test_corrected_flips_checkpoint(gpu, sec11):
    """A run restored from a checkpoint taken half-way ends with the same corrected tallies."""
    n_chains = 8
    inits = np.stack([sec11.assignment_array(G.sec11_plan(c % 3, sec11.nodes), [-1, 1]) for c in range(n_chains)])
    bases = np.asarray([G.SEC11_BASES[(3 * c) % 10] for c in range(n_chains)])
    a, lo, hi = _run(sec11, inits, bases, 2, (-1, 1), 0, 0.1, 2000, 1)
    blob = a.checkpoint()
    a.steps(1000)
    b, _, _ = _run(sec11, inits, bases, 2, (-1, 1), 0, 0.1, 1, 1)
    b.restore(blob)
    b.steps(1000)
    for x, y in zip(a.flips_exact(), b.flips_exact()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.wait_expected(), b.wait_expected())


def test_recom_rejects_exact_flips(gpu, sec11):
    fg = FlipGraph(sec11)
    inits = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])[None]
    cfg = RunConfig(proposal=_lib.FC_PROPOSE_RECOM, diag_mask=_lib.FC_DIAG_FLIPS_EXACT, recom_pop_target=798.0,
                    recom_epsilon=0.1, pop_lo=0, pop_hi=10 ** 6)
    with pytest.raises(Exception, match="FLIPS_EXACT"):
        FlipRun(fg, inits, cfg, bases=np.asarray([1.0]))
