"""gerrychain-shaped drop-in for the reference's chain construction and loop.

The reference builds its chain as (``grid_chain_sec11.py:299-342``)::

    updaters = {'population': Tally('population'), 'cut_edges': cut_edges,
                'b_nodes': b_nodes_bi, 'base': new_base, 'geom': geom_wait, ...}
    grid_partition = Partition(graph, assignment=cddict, updaters=updaters)
    popbound = within_percent_of_ideal_population(grid_partition, pop1)
    exp_chain = MarkovChain(slow_reversible_propose_bi,
                            Validator([single_flip_contiguous, popbound]),
                            accept=cut_accept, initial_state=grid_partition,
                            total_steps=100000)
    for part in exp_chain: ...

The same lines run unchanged against this module.  ``MarkovChain`` compiles the
recognised callables (by name: ``slow_reversible_propose_bi``, ``single_flip_contiguous``,
``Bounds`` over ``population``, ``cut_accept`` / ``always_accept``) into device parameters
and runs the chain on the GPU through the C-ABI.  Anything else raises
``NotImplementedError``: there is no CPU fallback for the chain itself.

Iterating a ``MarkovChain`` yields Partition-like views of every state (rejected steps
re-yield the same object, as gerrychain does), reconstructed on the host from the device's
per-proposal trace; ``MarkovChain.run()`` is the fast path that returns the driver's
diagnostics (``wait.txt`` sum, ``cut_times``, ``num_flips``, ``part_sum`` ...) computed on
the device.

The host-side helpers (``Tally``, ``cut_edges``, ``b_nodes_bi``, ``Bounds``,
``single_flip_contiguous``, ...) restate gerrychain 0.2 [gc-0.2] for direct calls on a
``Partition``; they are not on the hot path.
"""
from __future__ import annotations

import math
import random
from collections.abc import Mapping
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Hashable, Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from .graphs import GraphSpec, from_networkx, log1mp_table, slope_frame

# ----------------------------------------------------------------------------------------
# gerrychain updaters / constraints restated for host-side use  [gc-0.2]
# ----------------------------------------------------------------------------------------


class Tally:
    """``gerrychain.updaters.Tally``: per-part sum of a node attribute."""

    def __init__(self, fields, alias: Optional[str] = None):
        self.fields = [fields] if isinstance(fields, str) else list(fields)
        self.alias = alias

    def __call__(self, partition):
        out: Dict[Any, float] = {}
        g = partition.graph
        for nd, p in partition.assignment.items():
            out[p] = out.get(p, 0) + sum(g.nodes[nd][f] for f in self.fields)
        return out


def cut_edges(partition):
    """``gerrychain.updaters.cut_edges``: edges (sorted tuples) whose ends are in different parts."""
    a = partition.assignment
    return {tuple(sorted(e)) for e in partition.graph.edges if a[e[0]] != a[e[1]]}


def b_nodes_bi(partition):
    """``grid_chain_sec11.py:155-156``."""
    return {x[0] for x in partition["cut_edges"]}.union({x[1] for x in partition["cut_edges"]})


def b_nodes(partition):
    """``grid_chain_sec11.py:151-153`` (node, neighbouring part) pairs."""
    a = partition.assignment
    return {(x[0], a[x[1]]) for x in partition["cut_edges"]}.union(
        {(x[1], a[x[0]]) for x in partition["cut_edges"]})


def geom_wait(partition):
    """``grid_chain_sec11.py:147-148`` on numpy's global legacy stream (host use only; inside a
    device chain the wait comes from the canonical stream)."""
    p = len(list(partition["b_nodes"])) / (len(partition.graph.nodes) ** (len(partition.parts)) - 1)
    return int(np.random.geometric(p, 1)) - 1


class Bounds:
    """``gerrychain.constraints.Bounds``: ``lower <= min(func(p))`` and ``max(func(p)) <= upper``."""

    def __init__(self, func: Callable, bounds):
        self.func = func
        self.bounds = bounds

    def __call__(self, partition) -> bool:
        lower, upper = self.bounds
        values = self.func(partition)
        return lower <= min(values) and max(values) <= upper


def within_percent_of_ideal_population(initial_partition, percent: float = 0.01, pop_key: str = "population"):
    """[gc-0.2]: bounds ``((1-p)*ideal, (1+p)*ideal)`` fixed from the initial partition."""
    number_of_districts = len(initial_partition[pop_key].keys())
    total_population = sum(initial_partition[pop_key].values())
    ideal_population = total_population / number_of_districts
    bounds = ((1 - percent) * ideal_population, (1 + percent) * ideal_population)
    b = Bounds(lambda partition: partition[pop_key].values(), bounds=bounds)
    b.pop_key = pop_key
    return b


def contiguous(partition) -> bool:
    """Every part induces a connected subgraph."""
    import networkx as nx
    for nodes in partition.parts.values():
        if not nx.is_connected(partition.graph.subgraph(nodes)):
            return False
    return True


def single_flip_contiguous(partition) -> bool:
    """[gc-0.2] restated (BFS through the old district with the flipped node removed)."""
    parent = partition.parent
    if not parent:
        return contiguous(partition)
    graph, assignment = partition.graph, partition.assignment
    for changed, _ in partition.flips.items():
        old = parent.assignment[changed]
        old_nbrs = [n for n in graph.neighbors(changed) if assignment[n] == old]
        if not old_nbrs:
            return False
        seen, stack = {old_nbrs[0]}, [old_nbrs[0]]
        while stack:
            u = stack.pop()
            for w in graph.neighbors(u):
                if w not in seen and w != changed and assignment[w] == old:
                    seen.add(w)
                    stack.append(w)
        if any(n not in seen for n in old_nbrs):
            return False
    return True


class Validator:
    """``gerrychain.constraints.Validator``: ordered AND; a non-bool result is a TypeError."""

    def __init__(self, constraints):
        self.constraints = list(constraints)

    def __call__(self, partition) -> bool:
        for c in self.constraints:
            r = c(partition)
            if r is False:
                return False
            if r is not True:
                raise TypeError(f"Constraint {c!r} returned a non-boolean.")
        return True


def slow_reversible_propose(partition):
    """``grid_chain_sec11.py:117-130``: uniform over the (node, district) pairs of the pair
    updater ``b_nodes`` (``:151-153``) registered under ``"b_nodes"`` (host use; the device
    samples the same distribution, FC_PROPOSE_PAIR)."""
    flip = random.choice(list(partition["b_nodes"]))
    return partition.flip({flip[0]: flip[1]})


def slow_reversible_propose_bi(partition):
    """``grid_chain_sec11.py:132-145`` (host use; the device samples the same distribution)."""
    fnode = random.choice(list(partition["b_nodes"]))
    return partition.flip({fnode: -1 * partition.assignment[fnode]})


def cut_accept(partition) -> bool:
    """``grid_chain_sec11.py:171-179``."""
    bound = 1
    if partition.parent is not None:
        bound = partition["base"] ** (-len(partition["cut_edges"]) + len(partition.parent["cut_edges"]))
    return random.random() < bound


def always_accept(partition) -> bool:
    return True


# ---- accept / constraint variants the reference builds but does not run ----


def boundary_condition(partition) -> bool:
    """``grid_chain_sec11.py:43-52``: some node of ``partition["boundary"]`` (the
    ``boundary_node`` set, ``:228-234,292-297``) lies outside the district of the first."""
    blist = partition["boundary"]
    o_part = partition.assignment[blist[0]]
    for x in blist:
        if partition.assignment[x] != o_part:
            return True
    return False


class FixedCutEdges:
    """Constraint: the given edges stay cut.  ``fixed_endpoints`` (``:39-40``) is the
    instance with the sec11 edges (19,0)-(20,0) and (19,39)-(20,39)."""

    def __init__(self, pinned, name: str = "fixed_cut_edges"):
        self.pinned = [tuple(e) for e in pinned]
        self.__name__ = name

    def __call__(self, partition) -> bool:
        return all(partition.assignment[u] != partition.assignment[w] for u, w in self.pinned)


fixed_endpoints = FixedCutEdges([((19, 0), (20, 0)), ((19, 39), (20, 39))], name="fixed_endpoints")


class UniformAccept:
    """``uniform_accept`` (``:159-165``): ``random() < 1`` iff ``popbound``,
    ``single_flip_contiguous`` and ``boundary_condition`` hold, else ``< 0``.  The reference
    reads its module-level ``popbound``; here it is the constructor argument, or the
    Validator's population bound when the chain is compiled."""

    __name__ = "uniform_accept"

    def __init__(self, popbound=None):
        self.popbound = popbound

    def __call__(self, partition) -> bool:
        if self.popbound is None:
            raise ValueError("uniform_accept: no popbound given")
        bound = 0
        if self.popbound(partition) and single_flip_contiguous(partition) and boundary_condition(partition):
            bound = 1
        return random.random() < bound


class AnnealingCutAcceptBackwards:
    """``annealing_cut_accept_backwards`` (``:81-110``): ``random() < base ** (beta * (cut -
    cut')) * |B'| / |B|`` (B = endpoints of the cut edges), 0 unless ``popbound`` and
    ``single_flip_contiguous`` hold.  The reference fixes ``base = .1``, ``beta = 5``."""

    __name__ = "annealing_cut_accept_backwards"

    def __init__(self, popbound=None, base: float = .1, beta: float = 5):
        self.popbound, self.base, self.beta = popbound, base, beta

    def __call__(self, partition) -> bool:
        if self.popbound is None:
            raise ValueError("annealing_cut_accept_backwards: no popbound given")
        b1 = {x[0] for x in partition["cut_edges"]} | {x[1] for x in partition["cut_edges"]}
        b2 = {x[0] for x in partition.parent["cut_edges"]} | {x[1] for x in partition.parent["cut_edges"]}
        bound = 1
        if partition.parent is not None:
            bound = (self.base ** (self.beta * (-len(partition["cut_edges"]) + len(partition.parent["cut_edges"])))) \
                * (len(b1) / len(b2))
            if not self.popbound(partition):
                bound = 0
            if not single_flip_contiguous(partition):
                bound = 0
        return random.random() < bound


def recom(partition, pop_col, pop_target, epsilon, node_repeats=1):
    """gerrychain 0.2 ``recom`` [gc-0.2], the tree proposal the reference builds at
    ``grid_chain_sec11.py:328-335`` (host use; the device runs it from the compiled chain):
    merge the two districts of a random cut edge, draw a random spanning tree (maximum
    spanning tree of uniform edge weights), and split it at a random edge whose subtree
    population is within ``epsilon`` of ``pop_target`` (new root / tree while there is none)."""
    import networkx as nx
    edge = random.choice(tuple(partition["cut_edges"]))
    parts = (partition.assignment[edge[0]], partition.assignment[edge[1]])
    nodes = [n for n in partition.graph.nodes if partition.assignment[n] in parts]
    sub = partition.graph.subgraph(nodes)
    pops = {n: sub.nodes[n][pop_col] for n in sub.nodes}
    while True:
        h = nx.Graph()
        h.add_nodes_from(sub.nodes)
        h.add_weighted_edges_from((u, v, random.random()) for u, v in sub.edges)
        tree = nx.maximum_spanning_tree(h, algorithm="kruskal")
        for _ in range(node_repeats):
            root = random.choice([x for x in tree if tree.degree(x) > 1])
            pred = dict(nx.bfs_predecessors(tree, root))
            order = [root] + [v for _, v in nx.bfs_edges(tree, root)]
            sub_pop = dict(pops)
            for x in reversed(order[1:]):
                sub_pop[pred[x]] += sub_pop[x]
            cuts = [x for x in order[1:] if abs(sub_pop[x] - pop_target) < epsilon * pop_target]
            if cuts:
                child = random.choice(cuts)
                below = set(nx.dfs_preorder_nodes(tree.subgraph(set(tree) - {pred[child]}), child))
                flips = {n: (parts[0] if n in below else parts[1]) for n in nodes}
                return partition.flip(flips)


uniform_accept = UniformAccept()
annealing_cut_accept_backwards = AnnealingCutAcceptBackwards()


# ----------------------------------------------------------------------------------------
# Partition
# ----------------------------------------------------------------------------------------


class Partition:
    """``gerrychain.partition.Partition`` (host object: construction, ``flip``, lazy cached
    updaters).  The device chain takes its graph, assignment and updaters from it."""

    def __init__(self, graph=None, assignment=None, updaters=None, parent=None, flips=None):
        if parent is None:
            self.graph = graph
            self.assignment = dict(assignment) if not isinstance(assignment, str) else \
                {n: graph.nodes[n][assignment] for n in graph.nodes}
            self.updaters = dict(updaters or {})
            self.parent = None
            self.flips = None
        else:
            self.graph = parent.graph
            self.updaters = parent.updaters
            self.parent = parent
            self.flips = dict(flips)
            self.assignment = dict(parent.assignment)
            self.assignment.update(flips)
        self._cache: Dict[str, Any] = {}
        if "cut_edges" not in self.updaters:
            self.updaters.setdefault("cut_edges", cut_edges)

    @property
    def parts(self):
        out: Dict[Any, set] = {}
        for n, p in self.assignment.items():
            out.setdefault(p, set()).add(n)
        return {p: frozenset(s) for p, s in out.items()}

    def flip(self, flips):
        return Partition(parent=self, flips=flips)

    def __getitem__(self, key):
        if key not in self._cache:
            self._cache[key] = self.updaters[key](self)
        return self._cache[key]

    def __len__(self):
        return len(set(self.assignment.values()))

    def keys(self):
        return self.updaters.keys()


# ----------------------------------------------------------------------------------------
# compile the reference's callables into device parameters
# ----------------------------------------------------------------------------------------


def _name(f) -> str:
    return getattr(f, "__name__", type(f).__name__)


@dataclass
class ChainSpec:
    spec: GraphSpec
    labels: List[Any]
    init: np.ndarray
    base: float
    pop_lo: int
    pop_hi: int
    pop_bounds_float: tuple
    contig_first: bool = True
    pop_key: str = "population"
    accept: int = 0                 # FC_ACCEPT_*
    con_valid: int = 0              # FC_CON_* of the Validator
    con_accept: int = 0             # FC_CON_* of the accept callable
    beta: float = 0.0
    pinned: List[tuple] = field(default_factory=list)
    frozen: List[int] = field(default_factory=list)
    boundary_nodes: Optional[List[Hashable]] = None
    proposal: int = 0               # FC_PROPOSE_*
    recom: Optional[Dict[str, Any]] = None  # pop_target, epsilon, node_repeats
    # slow_reversible_propose: |b_nodes| counts the pairs of the registered pair updater
    # (FC_FLAG_NB_PAIRS), so geom_wait's p and the driver's rbn are what the reference computes
    nb_pairs: bool = False
    dev_labels: Optional[List[int]] = None  # int labels for the device's part_sum (None: indices)


def _bounds_of(b) -> tuple:
    lo_f, hi_f = b.bounds
    return (lo_f, hi_f), (int(math.ceil(lo_f)), int(math.floor(hi_f)))


def compile_chain(proposal, constraints, accept, initial_state: Partition) -> ChainSpec:
    """Map the reference's callables onto the device chain (NotImplementedError otherwise)."""
    import functools
    recom_kw = None
    pair = False
    if isinstance(proposal, functools.partial) and getattr(proposal.func, "__name__", "") == "recom":
        kw = dict(proposal.keywords)
        recom_kw = {"pop_col": kw.get("pop_col", "population"), "pop_target": float(kw["pop_target"]),
                    "epsilon": float(kw["epsilon"]), "node_repeats": int(kw.get("node_repeats", 1))}
    elif _name(proposal) == "slow_reversible_propose":
        # grid_chain_sec11.py:117-130: random.choice(list(partition["b_nodes"])) over the pair
        # updater b_nodes (:151-153) -> FC_PROPOSE_PAIR, any k
        pair = True
        bn = _name(initial_state.updaters.get("b_nodes"))
        if "b_nodes" not in initial_state.updaters:
            raise ValueError("slow_reversible_propose reads partition['b_nodes']: register the pair updater "
                             "b_nodes (grid_chain_sec11.py:151-153)")
        if bn != "b_nodes":
            raise NotImplementedError(f"slow_reversible_propose with the 'b_nodes' updater {bn!r}: it draws "
                                      "(node, district) pairs, so 'b_nodes' must be the pair updater b_nodes (:151-153)")
    elif _name(proposal) != "slow_reversible_propose_bi":
        raise NotImplementedError(f"proposal {_name(proposal)!r}: the device implements "
                                  "slow_reversible_propose_bi (grid_chain_sec11.py:132-145), "
                                  "slow_reversible_propose (:117-130) and partial(recom, ...) (:328-335)")
    cons = constraints.constraints if isinstance(constraints, Validator) else (
        list(constraints) if isinstance(constraints, (list, tuple)) else [constraints])
    contig_idx, bounds, pop_key = None, None, "population"
    con_valid, pinned = 0, []
    for i, c in enumerate(cons):
        nm = _name(c)
        if nm in ("single_flip_contiguous", "contiguous"):
            contig_idx = i
            con_valid |= _lib.FC_CON_CONTIG
        elif isinstance(c, Bounds):
            if bounds is not None:
                raise NotImplementedError("only one population Bounds constraint is supported")
            bounds = (i, c)
            pop_key = getattr(c, "pop_key", "population")
            con_valid |= _lib.FC_CON_POP
        elif nm == "boundary_condition":
            con_valid |= _lib.FC_CON_BOUNDARY
        elif isinstance(c, FixedCutEdges):
            con_valid |= _lib.FC_CON_FIXED
            pinned += c.pinned
        else:
            raise NotImplementedError(f"constraint {nm!r} is not implemented on the device")
    an = _name(accept)
    acc_kind, con_accept, beta, acc_bounds = _lib.FC_ACCEPT_CUT, 0, 0.0, None
    if an == "cut_accept":
        if "base" not in initial_state.updaters:
            raise ValueError("cut_accept reads partition['base']: add the 'base' updater")
        base = float(initial_state["base"])
    elif an == "always_accept":
        base = 1.0
    elif isinstance(accept, UniformAccept):
        acc_kind, base = _lib.FC_ACCEPT_UNIFORM, 1.0
        con_accept = _lib.FC_CON_CONTIG | _lib.FC_CON_POP | _lib.FC_CON_BOUNDARY
        acc_bounds = accept.popbound
    elif isinstance(accept, AnnealingCutAcceptBackwards):
        acc_kind, base, beta = _lib.FC_ACCEPT_ANNEAL, float(accept.base), float(accept.beta)
        con_accept = _lib.FC_CON_CONTIG | _lib.FC_CON_POP
        acc_bounds = accept.popbound
    else:
        raise NotImplementedError(f"accept {an!r}: the device implements cut_accept / always_accept / "
                                  "uniform_accept / annealing_cut_accept_backwards")
    if con_valid == 0:
        con_valid = _lib.FC_CON_EMPTY  # Validator([]): nothing re-draws
    if recom_kw is None and not ((con_valid | con_accept) & _lib.FC_CON_CONTIG):
        raise NotImplementedError("the device chain keeps districts connected: single_flip_contiguous must be "
                                  "in the Validator or the accept callable")
    # one population bound on the device: the Validator's, the accept's, or both equal
    if acc_bounds is None and (con_accept & _lib.FC_CON_POP):
        if bounds is None:
            raise NotImplementedError(f"{an}: give it a popbound (or a Bounds constraint in the Validator)")
        acc_bounds = bounds[1]
    if acc_bounds is not None and bounds is not None and tuple(acc_bounds.bounds) != tuple(bounds[1].bounds):
        raise NotImplementedError("the Validator's and the accept callable's population bounds differ")
    g = initial_state.graph
    labels = sorted(set(initial_state.assignment.values()))
    if pair and len(labels) > 2:
        if acc_kind != _lib.FC_ACCEPT_CUT or con_valid & ~(_lib.FC_CON_POP | _lib.FC_CON_CONTIG) or con_accept:
            raise NotImplementedError("k > 2: the device runs the Validator([single_flip_contiguous, popbound]) + "
                                      "cut_accept / always_accept chain (the accept / constraint variants are k = 2)")
        if bounds is not None and contig_idx is not None and bounds[0] < contig_idx:
            raise NotImplementedError("k > 2: the device's Validator tests single_flip_contiguous first")
    if pair and len(labels) > 32:
        raise NotImplementedError("the device holds at most 32 districts")
    if recom_kw is not None:
        if con_valid & ~(_lib.FC_CON_POP | _lib.FC_CON_CONTIG) or acc_kind != _lib.FC_ACCEPT_CUT:
            raise NotImplementedError("recom runs with the population Validator and cut_accept / always_accept")
        if recom_kw["pop_col"] != pop_key and bounds is not None:
            raise NotImplementedError("recom pop_col and the population bound must use the same column")
        pop_key = recom_kw["pop_col"]
    elif not pair and (len(labels) != 2 or sorted(labels) != [-1, 1]):
        raise NotImplementedError("slow_reversible_propose_bi flips -1 <-> 1: the plan must use labels -1 / 1")
    for n in g.nodes:
        g.nodes[n].setdefault(pop_key, 1)
    spec = from_networkx(g, pop_attr=pop_key,
                         pos={n: (g.nodes[n]["pos"] if "pos" in g.nodes[n] else n) for n in g.nodes}
                         if all(isinstance(n, tuple) and len(n) == 2 for n in g.nodes) else None)
    init = spec.assignment_array(initial_state.assignment, labels)
    pb = bounds[1] if bounds is not None else acc_bounds
    if pb is not None:
        (lo_f, hi_f), (lo, hi) = _bounds_of(pb)
        contig_first = bounds is None or contig_idx is None or contig_idx < bounds[0]
    else:
        lo_f, hi_f, lo, hi, contig_first = -math.inf, math.inf, -(2 ** 31), 2 ** 31 - 1, True
    frozen = sorted({spec.index[x] for e in pinned for x in e})
    bnodes = None
    if (con_valid | con_accept) & _lib.FC_CON_BOUNDARY:
        if "boundary" not in initial_state.updaters:
            raise ValueError("boundary_condition reads partition['boundary']: add the 'boundary' updater")
        bnodes = list(initial_state["boundary"])
    ints = all(isinstance(x, (int, np.integer)) and not isinstance(x, bool) and -2 ** 31 <= int(x) < 2 ** 31
               for x in labels)
    return ChainSpec(spec=spec, labels=labels, init=init, base=base, pop_lo=lo, pop_hi=hi,
                     pop_bounds_float=(lo_f, hi_f), contig_first=contig_first, pop_key=pop_key,
                     accept=acc_kind, con_valid=con_valid, con_accept=con_accept, beta=beta, pinned=pinned,
                     frozen=frozen, boundary_nodes=bnodes,
                     proposal=_lib.FC_PROPOSE_RECOM if recom_kw is not None else
                     _lib.FC_PROPOSE_PAIR if pair else _lib.FC_PROPOSE_BI_SIGN,
                     recom=recom_kw, nb_pairs=pair and len(labels) > 2,
                     dev_labels=[int(x) for x in labels] if ints else None)


def check_device_constraints(cs: ChainSpec, graph) -> None:
    """Preconditions of the device forms of the variant constraints: ``boundary_condition``
    is evaluated from the outer-face counts, so the boundary set must be the outer face;
    ``fixed_endpoints`` freezes the pinned edges' endpoints, exact when the start plan cuts
    every pinned edge (a k = 2 flip of an endpoint then always uncuts one)."""
    if cs.boundary_nodes is not None:
        _, meta = graph.rings()
        outer = {cs.spec.nodes[i] for i in np.nonzero(meta & np.uint64(1 << 9))[0]}
        if set(cs.boundary_nodes) != outer:
            raise NotImplementedError("boundary_condition: the 'boundary' set must be the graph's outer face")
    for u, w in cs.pinned:
        if cs.init[cs.spec.index[u]] == cs.init[cs.spec.index[w]]:
            raise NotImplementedError(f"fixed_endpoints: pinned edge {u}-{w} is not cut in the initial state")


# ----------------------------------------------------------------------------------------
# per-step views
# ----------------------------------------------------------------------------------------


class _AssignmentView(Mapping):
    __slots__ = ("_a", "_spec", "_labels")

    def __init__(self, a, spec, labels):
        self._a, self._spec, self._labels = a, spec, labels

    def __getitem__(self, node):
        return self._labels[self._a[self._spec.index[node]]]

    def __iter__(self):
        return iter(self._spec.nodes)

    def __len__(self):
        return self._spec.n


class StateView:
    """A yielded chain state: ``part[key]`` for the reference's updaters, ``part.assignment``,
    ``part.flips`` (stale on rejected steps, as in gerrychain), ``part.parent`` (None)."""

    def __init__(self, chain, a: np.ndarray, flips, wait: int, cut: int, nb: int, step: int):
        self._chain = chain
        self._a = a
        self.flips = flips
        self.parent = None
        self.graph = chain.initial_state.graph
        self.updaters = chain.initial_state.updaters
        self._cache: Dict[str, Any] = {"geom": wait}
        self._cut, self._nb, self.step = cut, nb, step
        self.assignment = _AssignmentView(a, chain.cspec.spec, chain.cspec.labels)

    @property
    def parts(self):
        sp, lab = self._chain.cspec.spec, self._chain.cspec.labels
        return {lab[d]: frozenset(sp.nodes[i] for i in np.nonzero(self._a == d)[0]) for d in range(len(lab))}

    def __len__(self):
        return len(self._chain.cspec.labels)

    def __getitem__(self, key):
        if key in self._cache:
            return self._cache[key]
        sp = self._chain.cspec.spec
        if key == "cut_edges":
            e = self._chain.edges
            m = self._a[e[:, 0]] != self._a[e[:, 1]]
            nodes = sp.nodes
            val = {tuple(sorted((nodes[u], nodes[v]))) for u, v in e[m]}
            assert len(val) == self._cut
        elif key == "b_nodes" and self.updaters.get("b_nodes") is b_nodes_bi:
            val = b_nodes_bi(self)
        elif key == "population":
            pops = np.bincount(self._a, weights=sp.pop, minlength=len(self._chain.cspec.labels))
            val = {self._chain.cspec.labels[d]: int(pops[d]) for d in range(len(pops))}
        else:
            val = self.updaters[key](self)
        self._cache[key] = val
        return val


class MarkovChain:
    """``gerrychain.MarkovChain`` backed by the device (one chain, ``fc_run`` of size 1)."""

    def __init__(self, proposal, constraints, accept, initial_state, total_steps: int, *,
                 seed: int = 0, chain_id: int = 0, device: int = 0, chunk: int = 4096):
        self.proposal, self.constraints, self.accept = proposal, constraints, accept
        self.initial_state = initial_state
        self.total_steps = int(total_steps)
        self.seed, self.chain_id, self.device, self.chunk = seed, chain_id, device, chunk
        self.cspec = compile_chain(proposal, constraints, accept, initial_state)
        self.edges = self.cspec.spec.edges()
        self._run = None
        self._graph = None
        # MarkovChain.__init__ validates the initial state [gc-0.2]
        cons = constraints.constraints if isinstance(constraints, Validator) else (
            list(constraints) if isinstance(constraints, (list, tuple)) else [constraints])
        failed = [_name(c) for c in cons if not c(initial_state)]
        if failed:
            raise ValueError("The given initial_state is not valid according is_valid. "
                             "The failed constraints were: " + ",".join(failed))
        if self.cspec.boundary_nodes is not None or self.cspec.pinned:
            from .engine import FlipGraph
            self._graph = FlipGraph(self.cspec.spec)
            check_device_constraints(self.cspec, self._graph)

    def __len__(self):
        return self.total_steps

    def _make_run(self, trace: bool, diag: int, event_cap: int = 0):
        from .engine import FlipGraph, FlipRun, RunConfig
        if self._graph is None:
            self._graph = FlipGraph(self.cspec.spec)
        cs = self.cspec
        if cs.proposal == _lib.FC_PROPOSE_RECOM:
            cfg = RunConfig(k=len(cs.labels), labels=tuple(cs.labels), proposal=cs.proposal, seed=self.seed,
                            chain_id_offset=self.chain_id, pop_lo=cs.pop_lo, pop_hi=cs.pop_hi, base=cs.base,
                            device=self.device, diag_mask=0, trace_chains=1 if trace else 0,
                            trace_cap=self.chunk + 16 if trace else 0, recom_pop_target=cs.recom["pop_target"],
                            recom_epsilon=cs.recom["epsilon"], recom_node_repeats=cs.recom["node_repeats"])
            return FlipRun(self._graph, cs.init[None, :], cfg)
        k = len(cs.labels)
        # k > 2: the reference's Validator([single_flip_contiguous, popbound]) (or without a bound:
        # the same with bounds nothing fails) is the kernels' default constraint set
        con_valid = 0 if k > 2 else cs.con_valid
        cfg = RunConfig(k=k, proposal=cs.proposal, seed=self.seed, chain_id_offset=self.chain_id,
                        pop_lo=cs.pop_lo, pop_hi=cs.pop_hi, base=cs.base, device=self.device, diag_mask=diag,
                        flags=_lib.FC_FLAG_NB_PAIRS if cs.nb_pairs else 0,
                        trace_chains=1 if trace else 0, trace_cap=64 * self.chunk + 4096 if trace else 0,
                        labels=tuple(cs.dev_labels if cs.dev_labels is not None else range(k)),
                        event_cap=event_cap, accept=cs.accept, con_valid=con_valid, con_accept=cs.con_accept,
                        beta=cs.beta, frozen=tuple(cs.frozen))
        return FlipRun(self._graph, self.cspec.init[None, :], cfg)

    # ---- per-step iteration (debugging path) -------------------------------------------
    def __iter__(self):
        if self.cspec.proposal == _lib.FC_PROPOSE_RECOM:
            yield from self._iter_recom()
            return
        run = self._make_run(trace=True, diag=_lib.FC_DIAG_WAIT)
        sp, lab = self.cspec.spec, self.cspec.labels
        a = self.cspec.init.copy()
        st = run.stats()
        view = StateView(self, a.copy(), None, int(st["wait_cur"][0]), int(st["cut"][0]), int(st["nb"][0]), 0)
        yield view
        done = 1
        while done < self.total_steps:
            n = min(self.chunk, self.total_steps - done)
            run.trace_reset()
            run.steps(n)
            for r in run.trace(0):
                if not (r["flags"] & 1):
                    continue
                done += 1
                if r["flags"] & 2:
                    v = int(r["v"])
                    a[v] = (int(r["flags"]) >> 8) & 0xff  # the target district (k = 2: 1 - a[v])
                    view = StateView(self, a.copy(), {sp.nodes[v]: lab[a[v]]}, int(r["wait"]), int(r["cut"]),
                                     int(r["nb"]), done - 1)
                yield view
        run.close()

    def _run_recom(self) -> "ChainResult":
        """ReCom on the device: the driver's sums (|cut|, |B| over yields), acceptance
        counts, spanning trees (``stats["bfs_levels"]``) and roots tried (``stats["bfs_calls"]``)."""
        if self._graph is None:
            from .engine import FlipGraph
            self._graph = FlipGraph(self.cspec.spec)
        run = self._make_run(trace=False, diag=0)
        if self.total_steps > 1:
            run.steps(self.total_steps - 1)
        res = _recom_result(self, run)
        run.close()
        return res

    def _iter_recom(self):
        """ReCom yields, one device step per yield (debugging path): the state is read back
        after every step; ``flips`` holds the nodes the last accepted proposal moved."""
        if self._graph is None:
            from .engine import FlipGraph
            self._graph = FlipGraph(self.cspec.spec)
        run = self._make_run(trace=False, diag=0)
        sp, lab = self.cspec.spec, self.cspec.labels
        a = self.cspec.init.copy()
        st = run.stats()
        view = StateView(self, a.copy(), None, 0, int(st["cut"][0]), int(st["nb"][0]), 0)
        yield view
        for t in range(1, self.total_steps):
            acc0 = int(st["accepted"][0])
            run.steps(1)
            st = run.stats()
            if int(st["accepted"][0]) > acc0:
                b = run.state()[0]
                moved = np.nonzero(b != a)[0]
                a = b
                view = StateView(self, a.copy(), {sp.nodes[i]: lab[a[i]] for i in moved}, 0, int(st["cut"][0]),
                                 int(st["nb"][0]), t)
            yield view
        run.close()

    # ---- fast path -------------------------------------------------------------------
    def run(self, series: bool = True, frame: Optional[str] = "auto", corrected: bool = True) -> "ChainResult":
        """All ``total_steps`` yields on the device; the reference driver's outputs
        (``grid_chain_sec11.py:366-419``) come back as a :class:`ChainResult`.

        ``series`` keeps the per-yield lists ``rce`` / ``rbn`` (``:367-369``) through the
        device event log; ``frame`` ("sec11", "frank", None or "auto": from the
        ``slope`` updater and the node labels) adds the ``slopes`` / ``angles`` lists
        (``:371-394``) computed by ``fc_run_frame_series``.  ``corrected`` adds the
        statistics the driver's quirky tallies aim at, beside them:
        ``flip_count`` / ``occupancy`` / ``last_accept`` (FC_DIAG_FLIPS_EXACT) and the
        Rao-Blackwellised ``waits_expected``."""
        if self.cspec.proposal == _lib.FC_PROPOSE_RECOM:
            return self._run_recom()
        diag = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS
        if frame == "auto":
            frame = None
            # (the frame-edge slope / angle of :371-394 is a two-district statistic; k = 2 only)
            if series and len(self.cspec.labels) == 2 and \
                    _name(self.initial_state.updaters.get("slope")) == "boundary_slope":
                neg = any(isinstance(nd, tuple) and nd[1] < 0 for nd in self.cspec.spec.nodes)
                frame = "frank" if neg else "sec11"
        if series:
            diag |= _lib.FC_DIAG_SERIES
        if corrected:
            diag |= _lib.FC_DIAG_FLIPS_EXACT
        run = self._make_run(trace=False, diag=diag, event_cap=max(self.total_steps, 1) if series else 0)
        if self.total_steps > 1:
            run.steps(self.total_steps - 1)
        res = ChainResult.from_run(self, run, 0)
        if corrected:
            sp = self.cspec.spec
            xf, xo, xl = run.flips_exact()
            res.flip_count = {sp.nodes[i]: int(xf[0, i]) for i in range(sp.n)}
            res.occupancy = {sp.nodes[i]: int(xo[0, i]) for i in range(sp.n)}
            res.last_accept = {sp.nodes[i]: int(xl[0, i]) for i in range(sp.n)}
            res.waits_expected = float(run.wait_expected()[0])
        if series:
            res.rce = run.yield_values("cut", 0)
            res.rbn = run.yield_values("nb", 0)
            if frame is not None:
                fs = run.frame_series(slope_frame(self.cspec.spec, frame), chains=[0])
                res.slopes = run.yield_series(fs["slope"][0], 0)
                res.angles = run.yield_series(fs["angle"][0], 0)
        run.close()
        return res


def _recom_result(chain: "MarkovChain", run) -> "ChainResult":
    sp, lab = chain.cspec.spec, chain.cspec.labels
    st = run.stats()
    fin = run.state()[0]
    return ChainResult(
        steps=int(st["steps"][0]), proposals=int(st["proposals"][0]), accepted=int(st["accepted"][0]),
        waits_sum=0, rce_sum=int(st["sum_cut"][0]), rbn_sum=int(st["sum_nb"][0]),
        cut_hist=np.zeros(0, dtype=np.int64), nb_hist=np.zeros(0, dtype=np.int64), cut_times={}, num_flips={},
        part_sum={}, last_flipped={}, lognum_flips={}, final_assignment={sp.nodes[i]: lab[fin[i]] for i in range(sp.n)},
        stats={k: int(v[0]) for k, v in st.items()})


@dataclass
class ChainResult:
    """What the reference's loop body + finalisation accumulate, for one chain."""

    steps: int
    proposals: int
    accepted: int
    waits_sum: int                      # wait.txt (:410-411)
    rce_sum: int                        # sum of len(cut_edges) over yields
    rbn_sum: int
    cut_hist: np.ndarray                # counts of len(cut_edges) over yields
    nb_hist: np.ndarray
    cut_times: Dict[tuple, int]         # graph[u][v]["cut_times"]
    num_flips: Dict[Hashable, int]      # graph.nodes[n]["num_flips"]
    part_sum: Dict[Hashable, int]       # graph.nodes[n]["part_sum"] (finalised, :416-418)
    last_flipped: Dict[Hashable, int]
    lognum_flips: Dict[Hashable, float]
    final_assignment: Dict[Hashable, Any]
    stats: Dict[str, int] = field(default_factory=dict)
    rce: Optional[np.ndarray] = None     # per-yield len(cut_edges)   (:367)
    rbn: Optional[np.ndarray] = None     # per-yield len(b_nodes)     (:369)
    slopes: Optional[np.ndarray] = None  # per-yield slope            (:371-382)
    angles: Optional[np.ndarray] = None  # per-yield angle            (:389-394)
    # corrected companions of the quirky tallies (run(corrected=True)):
    flip_count: Optional[Dict[Hashable, int]] = None   # accepted flips (num_flips counts re-yields)
    occupancy: Optional[Dict[Hashable, int]] = None    # sum_t label (part_sum lacks final segments)
    last_accept: Optional[Dict[Hashable, int]] = None  # yield of the last accepted flip
    waits_expected: Optional[float] = None             # sum_t E[geom | |B_t|] (cached-sample-free)

    def heatmaps(self, shape=(40, 40), offset=(0, 0)) -> Dict[str, np.ndarray]:
        """The driver's ``A2`` arrays (``grid_chain_sec11.py:431-528``): ``A2[n[0], n[1]]``
        (FRANK: ``shape=(20, 40), offset=(0, 19)``, ``Frankenstein_chain.py:468-549``) of the
        final assignment (``end2``), ``part_sum`` (``wca2``), ``num_flips`` (``flip2``) and
        ``lognum_flips`` (``logflip2``)."""
        out = {}
        for name, vals in (("end2", self.final_assignment), ("wca2", self.part_sum),
                           ("flip2", self.num_flips), ("logflip2", self.lognum_flips)):
            A2 = np.zeros(shape)
            for n, x in vals.items():
                A2[n[0] + offset[0], n[1] + offset[1]] = x
            out[name] = A2
        return out

    def write_outputs(self, directory: str, prefix: str, shape=(40, 40), offset=(0, 0)) -> List[str]:
        """Write what the reference's sweep leaves per configuration, as data: ``wait.txt``
        (``str(sum(waits))``, ``:410-411``), the heatmap arrays, per-edge ``cut_times`` and
        the per-yield series, as ``.npy`` beside it (the PNG plotting is out of scope).
        ``prefix`` is the reference's ``f"{alignment}B{int(100*base)}P{int(100*pop1)}"``."""
        import os
        os.makedirs(directory, exist_ok=True)
        paths = []
        p = os.path.join(directory, prefix + "wait.txt")
        with open(p, "w") as f:
            f.write(str(self.waits_sum))
        paths.append(p)
        arrays = dict(self.heatmaps(shape, offset))
        arrays["edges"] = np.asarray(list(self.cut_times.values()), dtype=np.int64)
        for name in ("rce", "rbn", "slopes", "angles"):
            if getattr(self, name) is not None:
                arrays[name] = getattr(self, name)
        for name, arr in arrays.items():
            p = os.path.join(directory, prefix + name + ".npy")
            np.save(p, arr)
            paths.append(p)
        return paths

    @classmethod
    def from_run(cls, chain: MarkovChain, run, c: int) -> "ChainResult":
        st = run.stats()
        ch, nh = run.hist()
        nf, ps, lf = run.flips()
        return cls.from_arrays(chain.cspec, chain.edges, st, ch, nh, run.cut_times(), nf, ps, lf, run.state(), c)

    @classmethod
    def from_arrays(cls, cspec, edges, st, ch, nh, ct, nf, ps, lf, fin, c: int) -> "ChainResult":
        """Chain ``c`` of a run's read-outs (``stats``, ``hist``, ``cut_times``, ``flips``,
        ``state``, each ``[chains, ...]``): the one place a ChainResult is assembled, for the
        single-chain ``MarkovChain.run`` and the batched ``sweep.Sweep`` alike."""
        sp, lab = cspec.spec, cspec.labels
        ctc, finc = ct[c], fin[c]
        return cls(
            steps=int(st["steps"][c]), proposals=int(st["proposals"][c]), accepted=int(st["accepted"][c]),
            waits_sum=int(st["sum_wait"][c]), rce_sum=int(st["sum_cut"][c]), rbn_sum=int(st["sum_nb"][c]),
            cut_hist=ch[c], nb_hist=nh[c],
            cut_times={(sp.nodes[u], sp.nodes[v]): int(ctc[i]) for i, (u, v) in enumerate(edges)},
            num_flips={sp.nodes[i]: int(nf[c, i]) for i in range(sp.n)},
            part_sum={sp.nodes[i]: int(ps[c, i]) for i in range(sp.n)},
            last_flipped={sp.nodes[i]: int(lf[c, i]) for i in range(sp.n)},
            lognum_flips={sp.nodes[i]: math.log(int(nf[c, i]) + 1) for i in range(sp.n)},
            final_assignment={sp.nodes[i]: lab[finc[i]] for i in range(sp.n)},
            stats={k: int(v[c]) for k, v in st.items()})
