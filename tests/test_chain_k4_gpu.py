"""The reference's k > 2 chain through the plugin API.

A k > 2 driver built the way grid_chain_sec11.py builds its chain (:299-342), with the two lines
a k > 2 run changes: the proposal is ``slow_reversible_propose`` (:117-130) and the ``"b_nodes"``
updater is the pair updater ``b_nodes`` (:151-153) that proposal reads.  On the C3 shape (sec11,
the k = 4 quadrant plan, population tolerance 0.05, cut_accept with base mu) the device-backed
``chain.MarkovChain``:

* iterated by the driver's loop body (:366-402 restated: rce, rbn, waits, cut_times, num_flips /
  part_sum / last_flipped) equals its own fast path ``run()`` bit for bit;
* equals the C oracle on the same canonical stream with |b_nodes| counted as pairs
  (``fr_params.nb_pairs``): sum of waits, rce / rbn sums, proposals, final state;
* counts |b_nodes| as the pairs (len(part["b_nodes"]) of the pair updater), so geom_wait's p
  (:147-148) and rbn are the reference's own for this driver.
"""
import math

import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd import chain as fc
from flipcomplexityempirical_amd import graphs as G

pytestmark = pytest.mark.gpu


def build_k4_chain(base, pop1, total_steps, seed=31, chain_id=0):
    graph = G.sec11_nx()
    cddict = G.quadrant_plan(sorted(graph.nodes()))

    def new_base(partition):
        return base

    updaters = {"population": fc.Tally("population"), "cut_edges": fc.cut_edges, "b_nodes": fc.b_nodes,
                "base": new_base, "geom": fc.geom_wait}
    part0 = fc.Partition(graph, assignment=cddict, updaters=updaters)
    popbound = fc.within_percent_of_ideal_population(part0, pop1)
    exp_chain = fc.MarkovChain(fc.slow_reversible_propose, fc.Validator([fc.single_flip_contiguous, popbound]),
                               accept=fc.cut_accept, initial_state=part0, total_steps=total_steps,
                               seed=seed, chain_id=chain_id)
    return graph, exp_chain


def driver_loop(graph, exp_chain):
    """grid_chain_sec11.py:366-419 without the two-district slope / angle lines."""
    rce, rbn, waits = [], [], []
    for e in graph.edges():
        graph.edges[e]["cut_times"] = 0
    for n in graph.nodes():
        graph.nodes[n]["part_sum"] = exp_chain.initial_state.assignment[n]
        graph.nodes[n]["last_flipped"] = 0
        graph.nodes[n]["num_flips"] = 0
    t = 0
    for part in exp_chain:
        rce.append(len(part["cut_edges"]))
        waits.append(part["geom"])
        rbn.append(len(list(part["b_nodes"])))
        for edge in part["cut_edges"]:
            graph.edges[edge]["cut_times"] += 1
        if part.flips is not None:
            f = list(part.flips.keys())[0]
            graph.nodes[f]["part_sum"] = graph.nodes[f]["part_sum"] - part.assignment[f] * (t - graph.nodes[f]["last_flipped"])
            graph.nodes[f]["last_flipped"] = t
            graph.nodes[f]["num_flips"] = graph.nodes[f]["num_flips"] + 1
        t += 1
    for n in graph.nodes():
        if graph.nodes[n]["last_flipped"] == 0:
            graph.nodes[n]["part_sum"] = t * part.assignment[n]
        graph.nodes[n]["lognum_flips"] = math.log(graph.nodes[n]["num_flips"] + 1)
    return rce, rbn, waits, t, part


@pytest.mark.parametrize("base,pop1,chain_id", [(G.SEC11_MU, 0.05, 0), (1.0, 0.05, 5), (0.5, 0.2, 9)])
def test_k4_driver_loop_matches_fast_path_and_oracle(gpu, cref, base, pop1, chain_id):
    T = 3000
    graph, chain = build_k4_chain(base, pop1, T, chain_id=chain_id)
    cs = chain.cspec
    assert cs.proposal == _lib.FC_PROPOSE_PAIR and cs.nb_pairs and cs.labels == [0, 1, 2, 3]
    rce, rbn, waits, t, last = driver_loop(graph, chain)
    assert t == T
    # rbn counts the pair updater's pairs: more than the boundary nodes once a node touches two
    # foreign districts
    nodes_b = {x for e in last["cut_edges"] for x in e}
    assert rbn[-1] == len(last["b_nodes"]) >= len(nodes_b)
    res = chain.run()
    assert res.steps == T - 1
    assert res.waits_sum == sum(waits)
    assert res.rce_sum == sum(rce) and res.rbn_sum == sum(rbn)
    assert np.array_equal(res.rce, rce) and np.array_equal(res.rbn, rbn)
    assert np.array_equal(res.cut_hist, np.bincount(rce, minlength=res.cut_hist.size))
    assert np.array_equal(res.nb_hist, np.bincount(rbn, minlength=res.nb_hist.size))
    for e in graph.edges():
        assert graph.edges[e]["cut_times"] == res.cut_times[tuple(sorted(e))], e
    for n in graph.nodes():
        assert graph.nodes[n]["num_flips"] == res.num_flips[n], n
        assert graph.nodes[n]["part_sum"] == res.part_sum[n], n
        assert graph.nodes[n]["lognum_flips"] == res.lognum_flips[n]
        assert last.assignment[n] == res.final_assignment[n]
    # the C oracle on the same stream, |b_nodes| as pairs
    ref = cref.run(cs.spec, cs.init, base=cs.base, pop_lo=cs.pop_lo, pop_hi=cs.pop_hi, seed=31, chain_id=chain_id,
                   n_steps=T - 1, k=4, labels=[0, 1, 2, 3], proposal=1, nb_pairs=True,
                   log1mp=G.log1mp_table(cs.spec.n, 4, G.nb_width(cs.spec, 4, True)))
    for key, val in (("sum_wait", res.waits_sum), ("sum_cut", res.rce_sum), ("sum_nb", res.rbn_sum),
                     ("proposals", res.proposals), ("accepted", res.accepted)):
        assert ref["stats"][key] == val, key
    fin = np.asarray([cs.labels.index(res.final_assignment[nd]) for nd in cs.spec.nodes], dtype=np.int8)
    assert np.array_equal(ref["final"], fin)


def test_k4_pairs_launches_against_oracle(gpu, cref):
    """FC_FLAG_NB_PAIRS through the lean and full k > 2 instances at production width (256 chains,
    bases with high and low acceptance), in three launches, against the oracle per chain.  Such
    runs commit one flip at a time (the multi-flip pass counts |B| as nodes only)."""
    from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
    sec11 = G.sec11_graph()
    k = 4
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    _, (lo, hi) = G.population_bounds(sec11.n, k, 0.05)
    W = G.nb_width(sec11, k, True)
    bases = np.asarray([1.0, G.SEC11_MU, 0.5, 2.0] * 64)
    for diag in (_lib.FC_DIAG_WAIT, _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST):
        cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=7, pop_lo=lo, pop_hi=hi,
                        flags=_lib.FC_FLAG_NB_PAIRS, diag_mask=diag)
        run = FlipRun(FlipGraph(sec11), np.broadcast_to(a0, (256, sec11.n)), cfg, bases=bases)
        assert run.nb_width() == W
        for n in (700, 1, 1299):
            run.steps(n)
        assert run.kernel_name().endswith(", 0>"), run.kernel_name()  # no multi-flip instance
        st, fin = run.stats(), run.state()
        nh = run.hist()[1] if diag & _lib.FC_DIAG_HIST else None
        for c in range(0, 256, 17):
            ref = cref.run(sec11, a0, base=bases[c], pop_lo=lo, pop_hi=hi, seed=7, chain_id=c, n_steps=2000, k=k,
                           labels=list(range(k)), proposal=1, nb_pairs=True, want_hist=nh is not None,
                           log1mp=G.log1mp_table(sec11.n, k, W))
            assert np.array_equal(fin[c], ref["final"]), c
            for key in ("steps", "proposals", "accepted", "sum_cut", "sum_nb", "sum_wait", "wait_cur", "cut", "nb"):
                assert int(st[key][c]) == int(ref["stats"][key]), (c, key)
            if nh is not None:
                assert np.array_equal(nh[c], ref["nb_hist"]), c
        run.close()
