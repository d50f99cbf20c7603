"""Native ring builder (fc_graph_create, host-only): rings, link bits, exactness flags, and
the planar local contiguity rule against BFS on random states of several graph families."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph
from tests.test_oracle_golden import _local_rule


def _check_rings(spec, fg):
    ring, meta = fg.rings()
    adj = [set(spec.neighbors(u).tolist()) for u in range(spec.n)]
    for v in range(spec.n):
        L = int(meta[v]) & 0xFF
        nbr = (int(meta[v]) >> 16) & 0xFFFF
        link = (int(meta[v]) >> 32) & 0xFFFF
        ents = ring[v][:L].tolist()
        nb = [ents[i] for i in range(L) if nbr >> i & 1]
        assert sorted(nb) == sorted(adj[v]), v              # every neighbour exactly once
        assert v not in ents
        assert all(ring[v][L:] == v)                        # padding
        for i in range(L):
            if link >> i & 1:                              # links are real edges
                assert ents[(i + 1) % L] in adj[ents[i]], (v, i)


@pytest.mark.parametrize("name", ["sec11", "frank", "grid10", "tri"])
def test_lattice_rings(name):
    spec = {"sec11": G.sec11_graph, "frank": G.frank_graph, "grid10": lambda: G.grid_graph(10, 10),
            "tri": lambda: G.triangular_graph(12, 20)}[name]()
    fg = FlipGraph(spec)
    _check_rings(spec, fg)
    info = fg.info
    assert info["planar"] == 1 and info["outer_simple"] == 1 and info["n_exact"] == spec.n


def test_sec11_outer_face_and_corners(sec11):
    fg = FlipGraph(sec11)
    ring, meta = fg.rings()
    gam = {sec11.nodes[i] for i in range(sec11.n) if int(meta[i]) >> 9 & 1}
    frame = {nd for nd in sec11.nodes if 0 in nd or 39 in nd}
    assert gam == frame and len(gam) == 152
    v = sec11.index[(0, 1)]                                # corner with the added diagonal
    L = int(meta[v]) & 0xFF
    assert [sec11.nodes[x] for x in ring[v][:L]] == [(1, 0), (1, 1), (1, 2), (0, 2)]


def test_no_positions_and_nonplanar_are_not_exact(sec11):
    assert FlipGraph(sec11, use_positions=False).info["n_exact"] == 0
    bad = G.GraphSpec(nodes=sec11.nodes, row_ptr=sec11.row_ptr, col_idx=sec11.col_idx, pop=sec11.pop,
                      pos=sec11.pos[np.random.default_rng(0).permutation(sec11.n)], index=sec11.index)
    fg = FlipGraph(bad)
    assert fg.info["planar"] == 0 and fg.info["n_exact"] == 0
    _check_rings(bad, fg)
    assert FlipGraph(sec11, exact=False).info["n_exact"] == 0


def test_bad_csr_rejected():
    from flipcomplexityempirical_amd import _lib
    spec = G.grid_graph(3, 3)
    col = spec.col_idx.copy()
    col[0] = 0  # self loop
    bad = G.GraphSpec(nodes=spec.nodes, row_ptr=spec.row_ptr, col_idx=col, pop=spec.pop)
    with pytest.raises(ValueError):
        FlipGraph(bad)
    assert _lib.FC_ERR_ARG == -1


def _delaunay_spec(n_pts, seed):
    from scipy.spatial import Delaunay
    import networkx as nx
    rng = np.random.default_rng(seed)
    pts = rng.random((n_pts, 2))
    tri = Delaunay(pts)
    g = nx.Graph()
    for s in tri.simplices:
        for i in range(3):
            g.add_edge(int(s[i]), int(s[(i + 1) % 3]))
    for i in range(n_pts):
        g.nodes[i]["population"] = 1
    return G.from_networkx(g, pos={i: tuple(pts[i]) for i in range(n_pts)})


def _random_two_district_states(spec, cref, rng, n_states, base=1.0, steps=400):
    """Reachable k=2 states: run the oracle chain from a half-plane plan."""
    order = np.argsort(spec.pos[:, 0]) if spec.pos is not None else np.arange(spec.n)
    a0 = np.zeros(spec.n, dtype=np.int8)
    a0[order[spec.n // 2:]] = 1
    if not cref.districts_contiguous(spec, a0, 2):
        pytest.skip("half-plane plan not contiguous for this sample")
    out = []
    for s in range(n_states):
        r = cref.run(spec, a0, base=base, pop_lo=0, pop_hi=10 ** 6, seed=int(rng.integers(1 << 30)), chain_id=s,
                     n_steps=steps)
        out.append(r["final"])
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_local_rule_exact_on_delaunay(cref, seed):
    spec = _delaunay_spec(300, seed)
    fg = FlipGraph(spec)
    assert fg.info["planar"] == 1
    ring, meta = fg.rings()
    gam = np.array([(int(m) >> 9) & 1 for m in meta], dtype=bool)
    rng = np.random.default_rng(seed)
    checked = exact_checked = 0
    for a in _random_two_district_states(spec, cref, rng, 6, base=0.5):
        e = spec.edges()
        cutm = a[e[:, 0]] != a[e[:, 1]]
        for v in np.unique(e[cutm].reshape(-1)):
            touch = bool(np.any(gam & (a == 1 - a[v])))
            res, known = _local_rule(ring[v], int(meta[v]), a, int(v), touch)
            truth = cref.flip_contiguous(spec, a, int(v))
            if known:
                assert res == truth, v
                exact_checked += 1
            else:
                assert not res  # the sufficient direction never claims a disconnected flip valid
            checked += 1
    assert checked > 300 and exact_checked > 0.8 * checked


@pytest.mark.parametrize("name", ["sec11", "frank", "tri", "delaunay", "nopos"])
def test_ring_relation_is_symmetric(name):
    """x in R(y) <=> y in R(x): the device's conflict test relies on it."""
    if name == "delaunay":
        spec, kw = _delaunay_spec(250, 3), {}
    elif name == "nopos":
        spec, kw = G.sec11_graph(), {"use_positions": False}
    else:
        spec = {"sec11": G.sec11_graph, "frank": G.frank_graph, "tri": lambda: G.triangular_graph(10, 16)}[name]()
        kw = {}
    ring, meta = FlipGraph(spec, **kw).rings()
    R = [set(ring[v][:int(meta[v]) & 0xFF].tolist()) for v in range(spec.n)]
    for v in range(spec.n):
        for x in R[v]:
            assert v in R[x], (v, x)


def test_from_json_round_trips(tmp_path):
    """gerrychain / networkx JSON ingestion gives the same CSR, populations
    and positions as building from the networkx graph directly."""
    import json
    from networkx.readwrite import json_graph
    from flipcomplexityempirical_amd import graphs as G
    ref = G.sec11_graph()
    g = G.sec11_nx()
    for kind, data in (("adjacency", json_graph.adjacency_data(g)), ("node_link", json_graph.node_link_data(g, edges="links"))):
        p = tmp_path / f"sec11_{kind}.json"
        p.write_text(json.dumps(data))
        spec = G.from_json(str(p))
        assert spec.nodes == ref.nodes
        assert np.array_equal(spec.row_ptr, ref.row_ptr) and np.array_equal(spec.col_idx, ref.col_idx)
        assert np.array_equal(spec.pop, ref.pop) and np.array_equal(spec.pos, ref.pos)
    # triangular lattice: positions from the 'pos' attribute
    t = G.triangular_graph(6, 10)
    data = json_graph.adjacency_data(t.nx_graph)
    spec = G.from_json(data)
    assert np.array_equal(spec.col_idx, t.col_idx) and np.allclose(spec.pos, t.pos)
