"""GPU parity of the accept / constraint variants against the C oracle.

The reference builds, but does not run, ``uniform_accept`` (``grid_chain_sec11.py:159-165``),
``annealing_cut_accept_backwards`` (``:81-110``, with its ``|B'|/|B|`` Hastings factor),
``boundary_condition`` (``:43-52``) and ``fixed_endpoints`` (``:39-40``).  The device
evaluates boundary_condition from its outer-face counts and fixed_endpoints as frozen
endpoints; the oracle restates the reference literally (scan of the boundary_node set,
check of the pinned edges after the flip, |B'| by flipping).  Trajectories, per-proposal
traces (incl. the rejection reasons) and statistics must agree bit for bit, with the
Validator members re-drawing and the accept callable's constraints rejecting steps.
"""
import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd import chain as fc
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
from oracle import flipref as F

pytestmark = pytest.mark.gpu

C, P, B, X = _lib.FC_CON_CONTIG, _lib.FC_CON_POP, _lib.FC_CON_BOUNDARY, _lib.FC_CON_FIXED
PINNED = [((19, 0), (20, 0)), ((19, 39), (20, 39))]

CASES = {
    # name: (accept, con_valid, con_accept, base, beta, alignment, pct)
    "cut+boundary+fixed": (_lib.FC_ACCEPT_CUT, C | P | B | X, 0, 1 / G.SEC11_MU, 0.0, 0, 0.1),
    "uniform, pop validator": (_lib.FC_ACCEPT_UNIFORM, P, C | P | B, 1.0, 0.0, 1, 0.1),
    "uniform, contig validator": (_lib.FC_ACCEPT_UNIFORM, C, C | P | B, 1.0, 0.0, 2, 0.05),
    "anneal, validator": (_lib.FC_ACCEPT_ANNEAL, C | P, C | P, 0.1, 5.0, 0, 0.1),
    "anneal, accept only": (_lib.FC_ACCEPT_ANNEAL, 0, C | P, 0.8, 1.0, 2, 0.5),
}


def _frame_flags(spec):
    return np.asarray([1 if (0 in nd or 39 in nd) else 0 for nd in spec.nodes], dtype=np.uint8)  # :228-234


@pytest.mark.parametrize("case", list(CASES))
def test_variant_trajectories_match_oracle(gpu, cref, sec11, case):
    accept, cv, ca, base, beta, al, pct = CASES[case]
    fg = FlipGraph(sec11)
    a0 = sec11.assignment_array(G.sec11_plan(al, sec11.nodes), [-1, 1])
    _, (lo, hi) = G.population_bounds(sec11.n, 2, pct)
    pinned = [(sec11.index[u], sec11.index[w]) for u, w in PINNED] if cv & X else []
    frozen = sorted({x for e in pinned for x in e})
    n_chains, steps = 4, 3000
    cv = cv or _lib.FC_CON_EMPTY  # Validator([])
    cfg = RunConfig(seed=77, pop_lo=lo, pop_hi=hi, base=base, accept=accept, con_valid=cv,
                    con_accept=ca, beta=beta, frozen=tuple(frozen), trace_chains=n_chains, trace_cap=200000,
                    diag_mask=_lib.FC_DIAG_WAIT)
    run = FlipRun(fg, np.stack([a0] * n_chains), cfg)
    run.steps(steps)
    st, fin = run.stats(), run.state()
    for c in range(n_chains):
        ref = cref.run(sec11, a0, base=base, pop_lo=lo, pop_hi=hi, seed=77, chain_id=c, n_steps=steps,
                       log1mp=G.log1mp_table(sec11.n, 2), trace_cap=200000, accept=accept,
                       con_valid=cv, con_accept=ca, beta=beta, boundary=_frame_flags(sec11),
                       pinned=np.asarray(pinned, dtype=np.int32) if pinned else None)
        tr = run.trace(c)
        rt = ref["trace"]
        assert len(tr) == len(rt), (case, c)
        for f in ("draw", "v", "flags", "cut", "nb", "wait"):
            assert np.array_equal(tr[f], rt[f]), (case, c, f)
        assert np.array_equal(fin[c], ref["final"]), (case, c)
        for k in ("steps", "proposals", "accepted", "inv_contig", "inv_pop", "sum_wait", "sum_cut", "cut", "nb"):
            assert int(st[k][c]) == int(ref["stats"][k]), (case, c, k)
        assert st["accepted"][c] > 0


def _sec11_partition(alignment, pop1, extra_updaters=None):
    graph = G.sec11_nx()
    cddict = G.sec11_plan(alignment, sorted(graph.nodes()))
    bnodes = [x for x in graph.nodes() if 0 in x or 39 in x]

    def bnodes_p(partition):
        return bnodes

    updaters = {"population": fc.Tally("population"), "cut_edges": fc.cut_edges, "b_nodes": fc.b_nodes_bi,
                "boundary": bnodes_p, "base": lambda q: 1.0, "geom": fc.geom_wait}
    part = fc.Partition(graph, assignment=cddict, updaters=updaters)
    return part, fc.within_percent_of_ideal_population(part, pop1)


def test_markov_chain_uniform_accept_and_fixed_endpoints(gpu, cref, sec11):
    """The reference-shaped construction compiles onto the device and agrees with the oracle."""
    part, popbound = _sec11_partition(0, 0.1)
    chain = fc.MarkovChain(fc.slow_reversible_propose_bi,
                           fc.Validator([fc.single_flip_contiguous, popbound, fc.fixed_endpoints]),
                           accept=fc.UniformAccept(popbound), initial_state=part, total_steps=2001, seed=3)
    cs = chain.cspec
    assert (cs.accept, cs.con_valid, cs.con_accept) == (_lib.FC_ACCEPT_UNIFORM, C | P | X, C | P | B)
    res = chain.run(series=False)
    pinned = np.asarray([(cs.spec.index[u], cs.spec.index[w]) for u, w in cs.pinned], dtype=np.int32)
    ref = cref.run(cs.spec, cs.init, base=1.0, pop_lo=cs.pop_lo, pop_hi=cs.pop_hi, seed=3, chain_id=0,
                   n_steps=2000, log1mp=G.log1mp_table(cs.spec.n, 2), accept=_lib.FC_ACCEPT_UNIFORM,
                   con_valid=C | P | X, con_accept=C | P | B, boundary=_frame_flags(cs.spec), pinned=pinned)
    for k in ("steps", "proposals", "accepted", "inv_contig", "inv_pop", "sum_wait", "sum_cut"):
        assert res.stats[k] == int(ref["stats"][k]), k
    fin = ref["final"]
    for i, nd in enumerate(cs.spec.nodes):
        assert res.final_assignment[nd] == cs.labels[fin[i]]
    for u, w in fc.fixed_endpoints.pinned:
        assert res.final_assignment[u] != res.final_assignment[w]
