"""CPU checks of the frame-edge set behind the slope / angle diagnostic (row A13).

* ``graphs.slope_frame`` (the product's host setup) selects exactly the edges the oracle's
  restatement of ``boundary_slope`` (``grid_chain_sec11.py:55-78``,
  ``Frankenstein_chain.py:55-78``) keeps when every edge is cut.
* On all 174 decoded reference end states (``tests/golden``) exactly two frame edges are
  cut, so the reference's set order cannot change the slope's magnitude or the angle --
  the premise of DESIGN.md's "first two in canonical order" rule.
"""
import numpy as np

from flipcomplexityempirical_amd import graphs as G
from oracle.flipref import boundary_slope, cut_edge_labels, slope_angle
from tests.test_oracle_golden import GOLD, _to_assign


def _all_edges(spec):
    return {tuple(sorted((spec.nodes[u], spec.nodes[v]))) for u, v in spec.edges()}


def test_frame_equals_boundary_slope_filter(sec11, frank):
    for spec, kind, n_exp in ((sec11, "sec11", 152), (frank, "frank", None)):
        fr = G.slope_frame(spec, kind)
        got = {tuple(sorted((spec.nodes[u], spec.nodes[v]))) for u, v in zip(fr.eu, fr.ev)}
        assert got == set(boundary_slope(_all_edges(spec), kind))
        if n_exp is not None:
            assert len(got) == n_exp
        for (u, v), m in zip(zip(fr.eu, fr.ev), fr.mid):
            a, b = spec.nodes[u], spec.nodes[v]
            assert tuple(m) == ((a[0] + b[0]) / 2, (a[1] + b[1]) / 2)


def test_reference_end_states_have_two_frame_cut_edges(sec11, frank):
    gold = np.load(GOLD)
    for tag, spec, kind in (("sec11", sec11, "sec11"), ("frank", frank, "frank")):
        for img in gold[f"{tag}_end"]:
            a = _to_assign(spec, img, frank=(tag == "frank"))
            temp = boundary_slope(cut_edge_labels(spec, a), kind)
            assert len(temp) == 2
            s, ang = slope_angle(temp)
            s2, ang2 = slope_angle(temp[::-1])
            assert s == s2 and ang == ang2  # order-independent with two edges
