"""gerrychain-shaped API: host helpers and the compilation of the reference's callables
into device parameters (no GPU needed)."""
import pytest

from flipcomplexityempirical_amd import chain as fc
from flipcomplexityempirical_amd import graphs as G


def _sec11_partition(alignment=0, base=0.1):
    g = G.sec11_nx()
    plan = G.sec11_plan(alignment, sorted(g.nodes()))
    ups = {"population": fc.Tally("population"), "cut_edges": fc.cut_edges, "b_nodes": fc.b_nodes_bi,
           "base": lambda p: base, "geom": fc.geom_wait}
    return fc.Partition(g, assignment=plan, updaters=ups)


def test_partition_updaters_known_answers():
    p = _sec11_partition(2)
    assert len(p["cut_edges"]) == 78 and len(p["b_nodes"]) == 80
    assert sorted(p["population"].values()) == [798, 798]
    assert len(p) == 2 and set(p.parts) == {-1, 1}
    q = p.flip({(20, 20): -1 * p.assignment[(20, 20)]})
    assert q.parent is p and q.flips == {(20, 20): -p.assignment[(20, 20)]}
    assert fc.single_flip_contiguous(q) in (True, False)


def test_bounds_and_validator():
    p = _sec11_partition(0)
    b = fc.within_percent_of_ideal_population(p, 0.1)
    assert b.bounds == (718.2, 877.8000000000001)
    assert b(p) is True
    v = fc.Validator([fc.single_flip_contiguous, b])
    assert v(p) is True
    with pytest.raises(TypeError):
        fc.Validator([lambda part: 1])(p)


def test_compile_reference_chain():
    p = _sec11_partition(1, base=4)
    pb = fc.within_percent_of_ideal_population(p, 0.05)
    cs = fc.compile_chain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous, pb]),
                          fc.cut_accept, p)
    assert cs.base == 4.0 and (cs.pop_lo, cs.pop_hi) == (759, 837)
    assert cs.labels == [-1, 1] and cs.spec.n == 1596 and cs.contig_first
    assert int(cs.init.sum()) == 798


def test_compile_accepts_reference_named_callbacks():
    """The driver's own functions (same names) are recognised, e.g. its cut_accept."""
    def slow_reversible_propose_bi(partition):
        return partition

    def cut_accept(partition):
        return True

    p = _sec11_partition(0, base=0.2)
    cs = fc.compile_chain(slow_reversible_propose_bi, [fc.single_flip_contiguous], cut_accept, p)
    assert cs.base == 0.2 and cs.pop_lo < 0


def test_compile_k4_pair_chain():
    """the reference's k > 2 proposal (slow_reversible_propose,
    grid_chain_sec11.py:117-130) over the pair updater b_nodes (:151-153) compiles to the PAIR
    kernel with the plan's district ids and |b_nodes| counted as pairs; with the node updater
    b_nodes_bi it would draw nodes as (node, district) pairs, so it is refused."""
    def slow_reversible_propose(partition):  # the driver's own function, same name
        flip = partition["b_nodes"]
        return flip

    g = G.sec11_nx()
    plan = G.quadrant_plan(sorted(g.nodes()))
    ups = {"population": fc.Tally("population"), "cut_edges": fc.cut_edges, "b_nodes": fc.b_nodes,
           "base": lambda p: 2.5, "geom": fc.geom_wait}
    p = fc.Partition(g, assignment=plan, updaters=ups)
    pb = fc.within_percent_of_ideal_population(p, 0.05)
    from flipcomplexityempirical_amd import _lib
    for prop in (fc.slow_reversible_propose, slow_reversible_propose):
        cs = fc.compile_chain(prop, fc.Validator([fc.single_flip_contiguous, pb]), fc.cut_accept, p)
        assert cs.proposal == _lib.FC_PROPOSE_PAIR and cs.nb_pairs and cs.labels == [0, 1, 2, 3]
        assert cs.dev_labels == [0, 1, 2, 3] and cs.base == 2.5 and (cs.pop_lo, cs.pop_hi) == (380, 418)
    # the pair set |b_nodes| = sum of foreign districts per node
    a = p.assignment
    nf = sum(len({a[w] for w in g.neighbors(u)} - {a[u]}) for u in g.nodes())
    assert len(p["b_nodes"]) == nf > len(fc.b_nodes_bi(p))
    assert G.nb_width(G.sec11_graph(), 4, True) - 1 >= nf
    p_bi = fc.Partition(g, assignment=plan, updaters=dict(ups, **{"b_nodes": fc.b_nodes_bi}))
    with pytest.raises(NotImplementedError, match="pair updater"):
        fc.compile_chain(fc.slow_reversible_propose, [fc.single_flip_contiguous], fc.cut_accept, p_bi)
    p_none = fc.Partition(g, assignment=plan, updaters={k: v for k, v in ups.items() if k != "b_nodes"})
    with pytest.raises(ValueError, match="b_nodes"):
        fc.compile_chain(fc.slow_reversible_propose, [fc.single_flip_contiguous], fc.cut_accept, p_none)
    # k > 2 runs the reference's Validator + cut_accept chain only
    with pytest.raises(NotImplementedError, match="k > 2"):
        fc.compile_chain(fc.slow_reversible_propose, [fc.single_flip_contiguous], fc.UniformAccept(pb), p)
    # k = 2 with the pair updater: PAIR proposals, pairs == nodes (no flag needed)
    p2 = fc.Partition(g, assignment=G.sec11_plan(0, sorted(g.nodes())), updaters=ups)
    cs2 = fc.compile_chain(fc.slow_reversible_propose, [fc.single_flip_contiguous], fc.cut_accept, p2)
    assert cs2.proposal == _lib.FC_PROPOSE_PAIR and not cs2.nb_pairs and cs2.labels == [-1, 1]


def test_unsupported_callables_raise():
    p = _sec11_partition(0)
    with pytest.raises(NotImplementedError):
        fc.compile_chain(lambda part: part, [fc.single_flip_contiguous], fc.cut_accept, p)
    with pytest.raises(NotImplementedError):
        fc.compile_chain(fc.slow_reversible_propose_bi, [fc.single_flip_contiguous, lambda part: True],
                         fc.cut_accept, p)
    with pytest.raises(NotImplementedError):
        fc.compile_chain(fc.slow_reversible_propose_bi, [fc.within_percent_of_ideal_population(p, .1)],
                         fc.cut_accept, p)
    with pytest.raises(NotImplementedError):
        fc.compile_chain(fc.slow_reversible_propose_bi, [fc.single_flip_contiguous], lambda part: True, p)


def test_variant_callables_compile(sec11):
    """uniform_accept / annealing_cut_accept_backwards / boundary_condition /
    fixed_endpoints map onto the device parameters; the device forms'
    preconditions are checked (boundary set = outer face, pinned edges cut at the start)."""
    from flipcomplexityempirical_amd import _lib
    from flipcomplexityempirical_amd import chain as fc
    from flipcomplexityempirical_amd import graphs as G
    graph = G.sec11_nx()
    bnodes = [x for x in graph.nodes() if 0 in x or 39 in x]

    def bnodes_p(partition):
        return bnodes

    ups = {"population": fc.Tally("population"), "cut_edges": fc.cut_edges, "b_nodes": fc.b_nodes_bi,
           "boundary": bnodes_p, "base": lambda q: 1.0}
    part = fc.Partition(graph, assignment=G.sec11_plan(0, sorted(graph.nodes())), updaters=ups)
    pb = fc.within_percent_of_ideal_population(part, 0.1)
    cs = fc.compile_chain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous, fc.boundary_condition]),
                          fc.AnnealingCutAcceptBackwards(pb), part)
    assert (cs.accept, cs.con_valid, cs.con_accept, cs.base, cs.beta) == (
        _lib.FC_ACCEPT_ANNEAL, _lib.FC_CON_CONTIG | _lib.FC_CON_BOUNDARY, _lib.FC_CON_CONTIG | _lib.FC_CON_POP, 0.1, 5.0)
    cs = fc.compile_chain(fc.slow_reversible_propose_bi, fc.Validator([]), fc.UniformAccept(pb), part)
    assert cs.con_valid == _lib.FC_CON_EMPTY and cs.con_accept == 7
    # MarkovChain checks the device preconditions on the host (no GPU needed)
    chain = fc.MarkovChain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous, pb, fc.fixed_endpoints,
                                                                        fc.boundary_condition]),
                           accept=fc.cut_accept, initial_state=part, total_steps=10)
    assert chain.cspec.con_valid == 15 and len(chain.cspec.frozen) == 4
    # alignment 1 leaves the pinned edges uncut: the reference's own validation raises
    part1 = fc.Partition(graph, assignment=G.sec11_plan(1, sorted(graph.nodes())), updaters=ups)
    with pytest.raises(ValueError):
        fc.MarkovChain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous, fc.fixed_endpoints]),
                       accept=fc.cut_accept, initial_state=part1, total_steps=10)
    # a boundary set that is not the outer face has no device form
    ups2 = dict(ups, boundary=lambda q: bnodes[::2])
    part2 = fc.Partition(graph, assignment=G.sec11_plan(0, sorted(graph.nodes())), updaters=ups2)
    with pytest.raises(NotImplementedError):
        fc.MarkovChain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous, fc.boundary_condition]),
                       accept=fc.cut_accept, initial_state=part2, total_steps=10)
    with pytest.raises(NotImplementedError):  # contiguity nowhere
        fc.compile_chain(fc.slow_reversible_propose_bi, fc.Validator([pb]), fc.cut_accept, part)


def test_recom_partial_compiles_and_host_recom_is_valid():
    """``partial(recom, pop_col="population", pop_target=ideal, epsilon=0.05, node_repeats=1)``
    (grid_chain_sec11.py:328-335) compiles to FC_PROPOSE_RECOM; the host restatement of
    recom returns a balanced, contiguous two-district plan."""
    import functools
    import random as _random
    from flipcomplexityempirical_amd import _lib
    from flipcomplexityempirical_amd import chain as fc
    from flipcomplexityempirical_amd import graphs as G
    graph = G.sec11_nx()
    part = fc.Partition(graph, assignment=G.sec11_plan(0, sorted(graph.nodes())),
                        updaters={"population": fc.Tally("population"), "cut_edges": fc.cut_edges})
    ideal = sum(part["population"].values()) / len(part)
    tree_proposal = functools.partial(fc.recom, pop_col="population", pop_target=ideal, epsilon=0.05, node_repeats=1)
    pb = fc.within_percent_of_ideal_population(part, 0.1)
    cs = fc.compile_chain(tree_proposal, fc.Validator([pb]), fc.always_accept, part)
    assert cs.proposal == _lib.FC_PROPOSE_RECOM and cs.recom == {"pop_col": "population", "pop_target": ideal,
                                                                 "epsilon": 0.05, "node_repeats": 1}
    _random.seed(3)
    nxt = tree_proposal(part)
    assert fc.contiguous(nxt)
    pops = list(nxt["population"].values())
    assert all(abs(p_ - ideal) < 0.05 * ideal for p_ in pops)
