"""The device replays the reference's own flip-step trajectories (node tape):
``NativeRngChain`` (CPython / numpy Mersenne Twisters, ``random.choice(list(b_nodes))`` at
grid_chain_sec11.py:143) records its draws as tape words; ``fc_run_set_tape`` +
``fc_run_set_initial_wait`` feed them to the HIP kernel, which must reproduce every proposal
(node, valid / accepted / invalid reason, |cut|, |B|, geometric wait), the per-yield sums and
the final assignment bit for bit.  Several recorded chains of different lengths share one
launch (tapes zero-padded to the longest)."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

from test_node_tape import FIELDS, PAIR_CASES, record, wrap64

pytestmark = pytest.mark.gpu

STATS = ("steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb", "sum_wait", "cut", "nb")


def _replay(spec, plans, bases, pct, steps, seeds, *, lean=False, chunks=(None,), k=2, tune=None):
    chains = [record(spec, plans[i], bases[i], pct, seeds[i], steps, k=k) for i in range(len(plans))]
    tapes = [ch.node_tape() for ch in chains]
    L = max(t.size for t in tapes)
    tape = np.zeros((len(chains), L), dtype=np.uint32)
    for i, t in enumerate(tapes):
        tape[i, :t.size] = t
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    labels = [-1, 1] if k == 2 else list(range(k))
    inits = np.stack([spec.assignment_array(p, labels) for p in plans])
    n_trace = 0 if lean else len(chains)
    cfg = RunConfig(k=k, labels=tuple(labels), proposal=_lib.FC_PROPOSE_BI_SIGN if k == 2 else _lib.FC_PROPOSE_PAIR,
                    seed=1, pop_lo=lo, pop_hi=hi, trace_chains=n_trace,
                    trace_cap=0 if lean else max(len(ch.trace) for ch in chains) + 64,
                    diag_mask=_lib.FC_DIAG_WAIT if lean else _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST, tune=tune)
    run = FlipRun(FlipGraph(spec), inits, cfg, bases=np.asarray(bases, dtype=np.float64))
    run.set_tape(tape)
    run.set_initial_wait(np.asarray([ch.wait0_words for ch in chains], dtype=np.uint32))
    done = 0
    for n in chunks:
        n = steps - done if n is None else n
        run.steps(n)
        done += n
    assert done == steps
    return chains, run


def _compare(chains, run, lean):
    st = run.stats()
    fin = run.state()
    for c, ch in enumerate(chains):
        for k in STATS:
            ref = ch.stats[k] if k in ch.stats else None
            if k == "cut":
                ref = len(ch.state["cut_edges"])
            elif k == "nb":
                ref = len(ch.state["b_nodes"])
            assert int(st[k][c]) == wrap64(ref), (c, k, int(st[k][c]), ref)
        assert int(st["wait_cur"][c]) == int(ch.wait), c
        assert np.array_equal(fin[c], ch.assignment_ids()), c
        if not lean:
            got, exp = run.trace(c), ch.trace_array()
            assert len(got) == len(exp), (c, len(got), len(exp))
            for f in FIELDS:
                bad = np.nonzero(got[f] != exp[f])[0]
                assert bad.size == 0, (c, f, bad[:5])


@pytest.mark.parametrize("lean", [False, True])
def test_device_replays_native_rng_sec11(gpu, sec11, lean):
    """sec11 lattice, the three start plans, bases across the phase transition."""
    plans = [G.sec11_plan(al, sec11.nodes) for al in (0, 1, 2, 0, 1, 2)]
    bases = [0.2, 0.8, 1.0, G.SEC11_MU, 4.0, 10.0]
    chains, run = _replay(sec11, plans, bases, 0.1, 1200, seeds=[91 + i for i in range(6)], lean=lean,
                          chunks=(1, 250, None))
    _compare(chains, run, lean)


def test_device_replays_native_rng_c1_and_frank(gpu, frank):
    """C1 (10 x 10 grid, lambda = 1 and mu) for 4000 steps, and FRANK (ring length 6 cells,
    tight population bound)."""
    c1 = G.grid_graph(10, 10)
    plan = G.threshold_plan(c1.nodes, 0, 5)
    chains, run = _replay(c1, [plan] * 4, [1.0, 1.0, G.SEC11_MU, 0.5], 0.1, 4000, seeds=[5, 6, 7, 8])
    _compare(chains, run, False)
    plans = [G.frank_plan(al, frank.nodes) for al in range(3)]
    chains, run = _replay(frank, plans, [0.3, 1 / 0.3, 1.0], 0.05, 1500, seeds=[11, 12, 13])
    _compare(chains, run, False)


@pytest.mark.parametrize("chunks", [(None,), (1, 400, None)], ids=["1launch", "3launches"])
@pytest.mark.parametrize("name", sorted(PAIR_CASES))
def test_device_replays_native_rng_pair(gpu, name, chunks):
    """k > 2: the reference's pair proposal ``slow_reversible_propose`` (:117-130) under CPython's
    MT, replayed on the general-k kernel with the multi-flip commit forced on (several
    independent accepted flips per ring pass): every proposal (node, target district, verdict,
    |cut|, |B|, wait), the tallies and the end state, in one launch and in three.  Four
    recorded chains of different bases and seeds share each launch."""
    mk, plan_of, k, base, pct, steps = PAIR_CASES[name]
    spec = mk()
    plan = plan_of(spec)
    bases = [base, 1.0, 0.5, 3.0]
    chains, run = _replay(spec, [plan] * 4, bases, pct, steps, seeds=[4100 + i for i in range(4)], k=k,
                          chunks=chunks, tune={"multi_flip": 1})
    name_k = run.kernel_name()
    assert name_k.startswith("fc::flip_kernel<") and name_k.endswith((", true, 1>", ", true, 2>")), name_k
    _compare(chains, run, False)


def test_initial_wait_only_before_stepping(gpu, sec11):
    _, (lo, hi) = G.population_bounds(sec11.n, 2, 0.1)
    a0 = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])
    run = FlipRun(FlipGraph(sec11), a0[None, :], RunConfig(seed=3, pop_lo=lo, pop_hi=hi))
    run.steps(5)
    with pytest.raises(ValueError, match="stepped"):
        run.set_initial_wait(np.zeros((1, 2), dtype=np.uint32))
