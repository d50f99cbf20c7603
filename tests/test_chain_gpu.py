"""The reference's chain construction and driver loop, run unchanged in shape against the
device-backed MarkovChain (grid_chain_sec11.py:299-419, with networkx-3 attribute access).

Checks: the per-step iterator equals the fast path and the oracle; every driver output
(wait.txt sum, cut_times, num_flips, part_sum, lognum_flips) agrees.
"""
import math

import numpy as np
import pytest

from flipcomplexityempirical_amd import chain as fc
from flipcomplexityempirical_amd import graphs as G
from oracle.flipref import boundary_slope as _oracle_boundary_slope

pytestmark = pytest.mark.gpu


def boundary_slope(partition):
    """The reference's updater (grid_chain_sec11.py:55-78), via the oracle's restatement."""
    return _oracle_boundary_slope(partition["cut_edges"], "sec11")


def build_chain(alignment, base, pop1, total_steps, seed=21):
    graph = G.sec11_nx()
    cddict = G.sec11_plan(alignment, sorted(graph.nodes()))

    def new_base(partition):
        return base

    updaters = {"population": fc.Tally("population"), "cut_edges": fc.cut_edges, "b_nodes": fc.b_nodes_bi,
                "base": new_base, "geom": fc.geom_wait, "slope": boundary_slope}
    grid_partition = fc.Partition(graph, assignment=cddict, updaters=updaters)
    popbound = fc.within_percent_of_ideal_population(grid_partition, pop1)
    exp_chain = fc.MarkovChain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous, popbound]),
                               accept=fc.cut_accept, initial_state=grid_partition, total_steps=total_steps,
                               seed=seed, chain_id=alignment)
    return graph, exp_chain


def driver_loop(graph, exp_chain):
    """The body of grid_chain_sec11.py:366-419 (rce / waits / rbn, slopes / angles,
    cut_times, flips)."""
    rce, rbn, waits, slopes, angles = [], [], [], [], []
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
        temp = part["slope"]
        enda = ((temp[0][0][0] + temp[0][1][0]) / 2, (temp[0][0][1] + temp[0][1][1]) / 2)
        endb = ((temp[1][0][0] + temp[1][1][0]) / 2, (temp[1][0][1] + temp[1][1][1]) / 2)
        if endb[0] != enda[0]:
            slope = (endb[1] - enda[1]) / (endb[0] - enda[0])
        else:
            slope = np.inf
        slopes.append(slope)
        for edge in part["cut_edges"]:
            graph.edges[edge]["cut_times"] += 1
        anga = (enda[0] - 20, enda[1] - 20)
        angb = (endb[0] - 20, endb[1] - 20)
        angles.append(np.arccos(np.clip(np.dot(anga / np.linalg.norm(anga), angb / np.linalg.norm(angb)), -1, 1)))
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
    driver_loop.series = (slopes, angles)
    return rce, rbn, waits, t, part


@pytest.mark.parametrize("alignment,base,pop1", [(2, 0.2, 0.1), (0, 1.0, 0.05), (1, G.SEC11_MU, 0.5), (2, 10, 0.01)])
def test_driver_loop_matches_fast_path_and_oracle(gpu, cref, alignment, base, pop1, tmp_path):
    T = 2500
    graph, chain = build_chain(alignment, base, pop1, T)
    rce, rbn, waits, t, last = driver_loop(graph, chain)
    assert t == T and len(rce) == T
    res = chain.run()
    assert res.steps == T - 1
    assert res.waits_sum == sum(waits)
    assert res.rce_sum == sum(rce) and res.rbn_sum == sum(rbn)
    assert np.array_equal(res.cut_hist, np.bincount(rce, minlength=res.cut_hist.size))
    # per-yield lists: rce / rbn exact, slopes exact (== : the sign of a zero slope follows
    # set order), angles within 1e-6 (arccos of a cosine that may differ by an ulp)
    slopes, angles = driver_loop.series
    assert np.array_equal(res.rce, rce) and np.array_equal(res.rbn, rbn)
    assert res.slopes.size == T and np.all(res.slopes == np.asarray(slopes))
    assert np.max(np.abs(res.angles - np.asarray(angles))) <= 1e-6
    # the sweep's per-configuration outputs, as data (grid_chain_sec11.py:410-528)
    prefix = f"{alignment}B{int(100 * base)}P{int(100 * pop1)}"
    res.write_outputs(str(tmp_path), prefix)
    assert (tmp_path / f"{prefix}wait.txt").read_text() == str(sum(waits))
    A2 = np.load(tmp_path / f"{prefix}end2.npy")
    for n in graph.nodes():
        assert A2[n[0], n[1]] == last.assignment[n]
    assert np.array_equal(np.load(tmp_path / f"{prefix}rce.npy"), rce)
    for e in graph.edges():
        assert graph.edges[e]["cut_times"] == res.cut_times[tuple(sorted(e))], e
    for n in graph.nodes():
        assert graph.nodes[n]["num_flips"] == res.num_flips[n], n
        assert graph.nodes[n]["part_sum"] == res.part_sum[n], n
        assert graph.nodes[n]["lognum_flips"] == res.lognum_flips[n]
        assert last.assignment[n] == res.final_assignment[n]
    # and the oracle, from the same compiled chain
    cs = chain.cspec
    ref = cref.run(cs.spec, cs.init, base=cs.base, pop_lo=cs.pop_lo, pop_hi=cs.pop_hi, seed=21,
                   chain_id=alignment, n_steps=T - 1, log1mp=G.log1mp_table(cs.spec.n, 2))
    assert ref["stats"]["sum_wait"] == res.waits_sum
    assert ref["stats"]["sum_cut"] == res.rce_sum
    assert ref["stats"]["proposals"] == res.proposals


def test_invalid_initial_state(gpu):
    graph = G.sec11_nx()
    cddict = G.sec11_plan(0, sorted(graph.nodes()))
    cddict[(0, 5)] = 1
    p = fc.Partition(graph, assignment=cddict, updaters={"population": fc.Tally("population"),
                                                           "base": lambda q: 1.0})
    with pytest.raises(ValueError):
        fc.MarkovChain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous]),
                       accept=fc.cut_accept, initial_state=p, total_steps=10)


def test_stuck_chain_reports(gpu, sec11):
    """An unsatisfiable population bound: the chain cannot take a step; the device stops at
    max_draws and flags it (the reference would spin forever)."""
    from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
    fg = FlipGraph(sec11)
    a0 = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])
    run = FlipRun(fg, a0[None, :], RunConfig(pop_lo=798, pop_hi=798))
    run.steps(10, max_draws=20000)
    st = run.stats()
    assert st["stuck"][0] == 1 and st["steps"][0] == 0 and st["inv_pop"][0] > 0
    assert st["draws"][0] <= 20000 + 64
