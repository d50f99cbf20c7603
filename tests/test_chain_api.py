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
