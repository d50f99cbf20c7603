"""Host-side graph and initial-plan builders: the input side of the flip-walk hot path.

These reproduce the lattices and start plans the reference drivers build before they
construct the gerrychain ``Partition``:

* ``sec11_graph`` / ``sec11_plan``   -- ``grid_chain_sec11.py:186-260``
  (40x40 grid, 4 corner nodes removed, 4 corner diagonals added; plans by alignment).
* ``frank_graph`` / ``frank_plan``   -- ``Frankenstein_chain.py:186-246``
  (20x20 square grid glued to a triangular lattice along y = 0).
* ``grid_graph`` / ``threshold_plan`` -- the C1 config (10x10 grid, plan ``x[0] >= 5``).

Everything is converted to a :class:`GraphSpec` -- CSR adjacency with a canonical node
order (sorted node keys), integer node populations and planar positions. The positions
feed the native ring builder (``fc_graph_create``), which derives the per-node link rings
used by the on-device contiguity test. networkx is only used here, on the host.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, Hashable, List, Optional, Sequence

import numpy as np

try:  # networkx is a host-side dependency of the builders only
    import networkx as nx
except ImportError:  # pragma: no cover - the image ships networkx
    nx = None


@dataclass
class GraphSpec:
    """CSR view of a node-labelled graph (canonical node order = ``nodes``)."""

    nodes: List[Hashable]
    row_ptr: np.ndarray  # int32 [n+1]
    col_idx: np.ndarray  # int32 [2E], neighbours of each row sorted ascending
    pop: np.ndarray  # int32 [n]
    pos: Optional[np.ndarray] = None  # float64 [n, 2]
    nx_graph: object = None
    index: Dict[Hashable, int] = field(default_factory=dict)

    @property
    def n(self) -> int:
        return len(self.nodes)

    @property
    def n_edges(self) -> int:
        return int(self.col_idx.shape[0] // 2)

    def edges(self) -> np.ndarray:
        """Canonical edge list ``(u, v)`` with ``u < v`` in CSR order (the order of
        per-edge statistics such as ``cut_times``)."""
        out = []
        for u in range(self.n):
            for w in self.col_idx[self.row_ptr[u]:self.row_ptr[u + 1]]:
                if w > u:
                    out.append((u, int(w)))
        return np.asarray(out, dtype=np.int32).reshape(-1, 2)

    def neighbors(self, u: int) -> np.ndarray:
        return self.col_idx[self.row_ptr[u]:self.row_ptr[u + 1]]

    def degree(self) -> np.ndarray:
        return np.diff(self.row_ptr).astype(np.int32)

    def assignment_array(self, assignment: Dict[Hashable, int], labels: Sequence[int]) -> np.ndarray:
        """Map a ``{node: label}`` plan to district ids (index into ``labels``) in canonical order."""
        lut = {lab: i for i, lab in enumerate(labels)}
        return np.asarray([lut[assignment[nd]] for nd in self.nodes], dtype=np.int8)


def from_networkx(g, pop_attr: str = "population", pos: Optional[Dict] = None) -> GraphSpec:
    """Build a :class:`GraphSpec` from a networkx graph (nodes sorted for a canonical order)."""
    nodes = sorted(g.nodes())
    index = {nd: i for i, nd in enumerate(nodes)}
    n = len(nodes)
    row_ptr = np.zeros(n + 1, dtype=np.int32)
    cols: List[int] = []
    for i, nd in enumerate(nodes):
        nb = sorted(index[w] for w in g.neighbors(nd) if w != nd)
        cols.extend(nb)
        row_ptr[i + 1] = len(cols)
    col_idx = np.asarray(cols, dtype=np.int32)
    popv = np.asarray([int(g.nodes[nd].get(pop_attr, 1)) for nd in nodes], dtype=np.int32)
    p = None
    if pos is None:
        attr = nx.get_node_attributes(g, "pos") if nx is not None else {}
        if len(attr) == n:
            pos = attr
    if pos is not None:
        p = np.asarray([pos[nd] for nd in nodes], dtype=np.float64).reshape(n, 2)
    return GraphSpec(nodes=nodes, row_ptr=row_ptr, col_idx=col_idx, pop=popv, pos=p,
                     nx_graph=g, index=index)


def from_json(src, pop_attr: str = "population", pos_attrs: Optional[Sequence[str]] = None) -> GraphSpec:
    """A gerrychain / networkx JSON graph -> :class:`GraphSpec`.

    ``src`` is a path, a file object or an already-parsed dict in networkx's
    ``adjacency_data`` layout (what gerrychain ``Graph.to_json`` writes and ``Graph.from_json``
    reads [gc-0.2]; ``networkx.readwrite.json_graph`` is imported by the reference at
    ``grid_chain_sec11.py:12``) or its ``node_link_data`` layout.  List-valued node ids
    (tuples after a JSON round trip) become tuples again.  Positions for the planar ring
    builder come from ``pos_attrs`` (e.g. ``("C_X", "C_Y")``), else a ``pos`` attribute,
    else 2-tuple node ids."""
    import json
    from networkx.readwrite import json_graph
    if isinstance(src, dict):
        data = src
    elif hasattr(src, "read"):
        data = json.load(src)
    else:
        with open(src) as f:
            data = json.load(f)

    def tup(x):
        return tuple(tup(y) for y in x) if isinstance(x, list) else x

    data = dict(data)
    if "adjacency" in data:
        data["nodes"] = [dict(nd, id=tup(nd["id"])) for nd in data["nodes"]]
        data["adjacency"] = [[dict(e, id=tup(e["id"])) for e in row] for row in data["adjacency"]]
        g = json_graph.adjacency_graph(data)
    elif "links" in data or "edges" in data:
        key = "links" if "links" in data else "edges"
        data["nodes"] = [dict(nd, id=tup(nd["id"])) for nd in data["nodes"]]
        data[key] = [dict(e, source=tup(e["source"]), target=tup(e["target"])) for e in data[key]]
        g = json_graph.node_link_graph(data, edges=key)
    else:
        raise ValueError("from_json: neither an adjacency_data nor a node_link_data graph")
    pos = None
    if pos_attrs is not None:
        pos = {nd: (float(g.nodes[nd][pos_attrs[0]]), float(g.nodes[nd][pos_attrs[1]])) for nd in g.nodes}
    elif all("pos" in g.nodes[nd] for nd in g.nodes):
        pos = {nd: tuple(float(x) for x in g.nodes[nd]["pos"]) for nd in g.nodes}
    elif all(isinstance(nd, tuple) and len(nd) == 2 for nd in g.nodes):
        pos = {nd: (float(nd[0]), float(nd[1])) for nd in g.nodes}
    return from_networkx(g, pop_attr=pop_attr, pos=pos)


# --------------------------------------------------------------------------------------
# sec11 (grid_chain_sec11.py)
# --------------------------------------------------------------------------------------
SEC11_MU = 2.63815853  # grid_chain_sec11.py:33
SEC11_BASES = [.1, 1 / SEC11_MU ** 2, .2, 1 / SEC11_MU, .8, 1, SEC11_MU, 4, SEC11_MU ** 2, 10]  # :34
SEC11_POPS = [.01, .05, .1, .5, .9]  # :36
SEC11_DIAGONALS = [((0, 1), (1, 0)), ((0, 38), (1, 39)), ((38, 0), (39, 1)), ((38, 39), (39, 38))]  # :236
SEC11_CORNERS = [(0, 0), (0, 39), (39, 0), (39, 39)]  # :252


def sec11_nx(gn: int = 20, k: int = 2):
    """The sec11 lattice exactly as ``grid_chain_sec11.py:191,218,236,252`` builds it."""
    g = nx.grid_graph([k * gn, k * gn])
    for nd in g.nodes():
        g.nodes[nd]["population"] = 1  # :218
    g.add_edges_from(SEC11_DIAGONALS)
    g.remove_nodes_from(SEC11_CORNERS)
    return g


def sec11_graph() -> GraphSpec:
    g = sec11_nx()
    return from_networkx(g, pos={nd: (float(nd[0]), float(nd[1])) for nd in g.nodes()})


def sec11_plan(alignment: int, nodes: Optional[Sequence] = None) -> Dict:
    """±1 start plan, ``grid_chain_sec11.py:195-214`` (corners dropped as at :254-260)."""
    if nodes is None:
        nodes = [(x, y) for x in range(40) for y in range(40) if (x, y) not in SEC11_CORNERS]
    out = {}
    for n in nodes:
        if alignment == 0:
            out[n] = 1 if n[0] > 19 else -1
        elif alignment == 1:
            out[n] = 1 if n[1] > 19 else -1
        elif alignment == 2:
            if n[0] > n[1]:
                out[n] = 1
            elif n[0] == n[1] and n[0] > 19:
                out[n] = 1
            else:
                out[n] = -1
        else:
            raise ValueError("alignment must be 0, 1 or 2")
    return out


# --------------------------------------------------------------------------------------
# FRANK (Frankenstein_chain.py)
# --------------------------------------------------------------------------------------
FRANK_BASES = [.3, 1 / .3]  # Frankenstein_chain.py:34
FRANK_POPS = [.05, .1, .5, .9]  # :36


def frank_nx(m: int = 20):
    """``Frankenstein_chain.py:186-195``: grid (shifted to y <= 0) composed with a triangular lattice."""
    G = nx.grid_graph([m, m])
    relabel = {x: (x[0], x[1] - m + 1) for x in G.nodes()}
    G = nx.relabel_nodes(G, relabel)
    H = nx.triangular_lattice_graph(m, 2 * m - 2)
    F = nx.compose(G, H)
    for nd in F.nodes():
        F.nodes[nd]["population"] = 1
    return F


def frank_positions(F) -> Dict:
    pos = {}
    for nd in F.nodes():
        p = F.nodes[nd].get("pos")
        pos[nd] = (float(p[0]), float(p[1])) if p is not None else (float(nd[0]), float(nd[1]))
    return pos


def frank_graph(m: int = 20) -> GraphSpec:
    F = frank_nx(m)
    return from_networkx(F, pos=frank_positions(F))


def frank_plan(alignment: int, nodes: Sequence, m: int = 20) -> Dict:
    """``Frankenstein_chain.py:207-246``: start_plans = [diagonal, vertical, horizontal]."""
    if alignment == 0:
        inside = lambda x: 2 * x[0] - x[1] <= m - 3
    elif alignment == 1:
        inside = lambda x: x[0] < m / 2
    elif alignment == 2:
        inside = lambda x: x[1] < 0
    else:
        raise ValueError("alignment must be 0, 1 or 2")
    return {n: (1 if inside(n) else -1) for n in nodes}


# --------------------------------------------------------------------------------------
# Generic lattices used by the BASELINE configs
# --------------------------------------------------------------------------------------
def grid_graph(nx_: int, ny: int) -> GraphSpec:
    g = nx.grid_graph([nx_, ny])
    for nd in g.nodes():
        g.nodes[nd]["population"] = 1
    return from_networkx(g, pos={nd: (float(nd[0]), float(nd[1])) for nd in g.nodes()})


def threshold_plan(nodes: Sequence, axis: int, cut: float) -> Dict:
    """±1 plan by ``node[axis] >= cut`` (C1: 10x10 grid, ``x[0] >= 5``)."""
    return {n: (1 if n[axis] >= cut else -1) for n in nodes}


def triangular_graph(m: int, n: int) -> GraphSpec:
    H = nx.triangular_lattice_graph(m, n)
    for nd in H.nodes():
        H.nodes[nd]["population"] = 1
    return from_networkx(H)


def quadrant_plan(nodes: Sequence, half: float = 20) -> Dict:
    """C3's k=4 start plan on the sec11 lattice: district ``(x >= half) + 2 (y >= half)``
    (labels 0..3)."""
    return {n: int(n[0] >= half) + 2 * int(n[1] >= half) for n in nodes}


def strip_plan(spec: GraphSpec, k: int) -> Dict:
    """k vertical strips of (nearly) equal node count by x-coordinate, ties by y
    (C4's k=8 start plan on the triangular lattice; labels 0..k-1)."""
    if spec.pos is None:
        raise ValueError("strip_plan needs node positions")
    order = np.lexsort((spec.pos[:, 1], spec.pos[:, 0]))
    out = {}
    for rank, i in enumerate(order):
        out[spec.nodes[int(i)]] = int(rank * k // spec.n)
    return out


def delaunay_graph(n_points: int = 10000, seed: int = 0, sigma: float = 0.5) -> GraphSpec:
    """C5's synthetic precinct-like dual graph: the Delaunay triangulation of ``n_points``
    uniform points in the unit square (``scipy.spatial.Delaunay``, seed 0), irregular
    degree, node populations ``max(1, round(lognormal(0, sigma)))``."""
    from scipy.spatial import Delaunay
    rng = np.random.default_rng(seed)
    pts = rng.random((n_points, 2))
    pops = np.maximum(1, np.rint(rng.lognormal(0.0, sigma, n_points))).astype(np.int64)
    tri = Delaunay(pts)
    g = nx.Graph()
    for i in range(n_points):
        g.add_node(i, population=int(pops[i]))
    for s in tri.simplices:
        a, b, c = (int(x) for x in s)
        g.add_edges_from([(a, b), (b, c), (a, c)])
    return from_networkx(g, pos={i: (float(pts[i, 0]), float(pts[i, 1])) for i in range(n_points)})


def bisection_plan(spec: GraphSpec, k: int) -> Dict:
    """Recursive coordinate bisection into k districts (labels 0..k-1): split the node set
    along its longer coordinate extent at the population quantile k1/k (k1 = k // 2),
    recurse on both halves (C5's k=18 start plan).  Parts that come out disconnected
    have their stray components merged into the neighbouring district they touch most."""
    if spec.pos is None:
        raise ValueError("bisection_plan needs node positions")
    out = np.zeros(spec.n, dtype=np.int64)

    def split(idx: np.ndarray, kk: int, first: int):
        if kk == 1:
            out[idx] = first
            return
        k1 = kk // 2
        ext = spec.pos[idx].max(axis=0) - spec.pos[idx].min(axis=0)
        ax = int(np.argmax(ext))
        order = idx[np.argsort(spec.pos[idx, ax], kind="stable")]
        cum = np.cumsum(spec.pop[order].astype(np.int64))
        cut = int(np.searchsorted(cum, cum[-1] * k1 / kk))
        split(order[:cut], k1, first)
        split(order[cut:], kk - k1, first + k1)

    split(np.arange(spec.n), k, 0)
    # repair: keep the largest component of each district, hand the rest to a neighbour
    g = spec.nx_graph
    for _ in range(4):
        changed = False
        for d in range(k):
            nodes = [spec.nodes[i] for i in np.nonzero(out == d)[0]]
            comps = sorted(nx.connected_components(g.subgraph(nodes)), key=len, reverse=True)
            for comp in comps[1:]:
                for nd in comp:
                    i = spec.index[nd]
                    votes = np.bincount([out[spec.index[w]] for w in g.neighbors(nd) if out[spec.index[w]] != d],
                                        minlength=k)
                    if votes.sum():
                        out[i] = int(np.argmax(votes))
                        changed = True
        if not changed:
            break
    return {spec.nodes[i]: int(out[i]) for i in range(spec.n)}


# --------------------------------------------------------------------------------------
# Frame edges for the slope / angle diagnostic (boundary_slope)
# --------------------------------------------------------------------------------------
# boundary_slope keeps the cut edges whose two endpoints share one frame coordinate, plus
# (sec11 only) the four corner diagonals: grid_chain_sec11.py:55-78 (lines x=0, y=0,
# x=39, y=39) and Frankenstein_chain.py:55-78 (x=0, y=-19, x=19, y=20, diagonals
# commented out).  The angle is taken about (20, 20) in both drivers (:389-390, :417-418).
FRAME_RULES = {
    "sec11": {"lines": ((0, 0), (1, 0), (0, 39), (1, 39)), "diagonals": SEC11_DIAGONALS, "center": (20.0, 20.0)},
    "frank": {"lines": ((0, 0), (1, -19), (0, 19), (1, 20)), "diagonals": (), "center": (20.0, 20.0)},
}


@dataclass
class SlopeFrame:
    """Frame edges (canonical-edge order), their midpoints and the angle centre."""

    eu: np.ndarray    # int32 [F]
    ev: np.ndarray    # int32 [F]
    mid: np.ndarray   # float64 [F, 2]: ((u0+v0)/2, (u1+v1)/2) in node-label coordinates
    center: tuple


def slope_frame(spec: GraphSpec, kind: str = "sec11") -> SlopeFrame:
    """The edges ``boundary_slope`` can ever return: its filter applied to every edge.

    With both districts contiguous on a disc-like lattice exactly two frame edges are cut,
    so the result does not depend on which two the reference's set order picks first; for
    more, the device uses the first two in this (canonical edge) order."""
    rule = FRAME_RULES[kind]
    diag = {tuple(d) for d in rule["diagonals"]} | {(d[1], d[0]) for d in rule["diagonals"]}
    eu, ev, mid = [], [], []
    for u, v in spec.edges():
        a, b = spec.nodes[int(u)], spec.nodes[int(v)]
        on_line = any(a[axis] == val and b[axis] == val for axis, val in rule["lines"])
        if on_line or (a, b) in diag:
            eu.append(int(u))
            ev.append(int(v))
            mid.append(((a[0] + b[0]) / 2, (a[1] + b[1]) / 2))
    return SlopeFrame(eu=np.asarray(eu, dtype=np.int32), ev=np.asarray(ev, dtype=np.int32),
                      mid=np.asarray(mid, dtype=np.float64).reshape(-1, 2), center=rule["center"])


# --------------------------------------------------------------------------------------
# Known answers used by tests (host-side, networkx)
# --------------------------------------------------------------------------------------
def cut_and_boundary(spec: GraphSpec, assign: np.ndarray):
    """(|cut edges|, |boundary nodes|, district populations) of a district-id array."""
    e = spec.edges()
    cut = assign[e[:, 0]] != assign[e[:, 1]]
    bnodes = np.zeros(spec.n, dtype=bool)
    bnodes[e[cut, 0]] = True
    bnodes[e[cut, 1]] = True
    k = int(assign.max()) + 1
    pops = np.bincount(assign.astype(np.int64), weights=spec.pop, minlength=k).astype(np.int64)
    return int(cut.sum()), int(bnodes.sum()), pops


def population_bounds(total_pop: int, k: int, percent: float):
    """gerrychain ``within_percent_of_ideal_population`` bounds [gc-0.2], used at
    ``grid_chain_sec11.py:319``: ``((1-p)*ideal, (1+p)*ideal)`` with ``ideal = total/k``;
    returned as the float pair and the equivalent inclusive integer pair."""
    ideal = total_pop / k
    lo = (1 - percent) * ideal
    hi = (1 + percent) * ideal
    return (lo, hi), (int(math.ceil(lo)), int(math.floor(hi)))


def log1mp_table(n_nodes: int, k: int, width: Optional[int] = None) -> np.ndarray:
    """``log(1 - p)`` for ``p = |B| / (N**k - 1)``, |B| = 0..N (or 0..width-1: |b_nodes| counted
    as pairs, ``nb_width``) -- the exact float pipeline of ``geom_wait``
    (``grid_chain_sec11.py:147-148``: Python true division of ints, then numpy's legacy
    ``log(1.0 - p)``)."""
    denom = n_nodes ** k - 1
    return np.asarray([math.log(1.0 - (b / denom)) for b in range(width or n_nodes + 1)], dtype=np.float64)


def nb_width(spec: "GraphSpec", k: int, pairs: bool) -> int:
    """Entries of a |B| histogram row / log(1 - p) table (``fc_run_nb_width``): n + 1, or, with
    |b_nodes| counted as the (node, district) pairs of the pair updater ``b_nodes``
    (``grid_chain_sec11.py:151-153``; ``FC_FLAG_NB_PAIRS``, k > 2), the largest pair count
    sum_u min(deg u, k - 1), plus one."""
    if not pairs or k <= 2:
        return spec.n + 1
    deg = np.diff(np.asarray(spec.row_ptr, dtype=np.int64))
    return int(np.minimum(deg, k - 1).sum()) + 1
