"""TEST INFRASTRUCTURE ONLY -- the parity oracle for the flip-walk hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product
(``flipcomplexityempirical_amd``) never imports it.

Three pieces:

* :func:`philox4x32_10` -- numpy Philox4x32-10 (the canonical random stream).
* :class:`CRef` -- ctypes binding of ``oracle/flipref.c`` (plain-C restatement, fast
  enough for 1e5-1e6-step parity runs).
* :class:`GcFaithfulChain` -- pure-Python restatement with gerrychain-0.2 data structures
  (dict assignment copied per proposal, cut-edge sets of sorted tuples, ``b_nodes_bi``
  set, networkx ``multi_source_dijkstra`` contiguity).  This is the "reference Python CPU
  path" (``cpu_baseline.kind = "port"``) and the small-case cross-check of the C oracle.

Citations (``/root/reference``): proposal ``grid_chain_sec11.py:132-145``; boundary
``:155-156``; acceptance ``:171-179``; geometric wait ``:147-148``; chain/validator
``:319,340-342``; driver diagnostics ``:365-419``.  gerrychain internals are restated
from gerrychain 0.2.x (not vendored in the reference) and marked [gc-0.2].

Parity pinning of this oracle: ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from typing import Dict, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libflipref.so")

MASK32 = np.uint64(0xFFFFFFFF)
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)

FLAG_VALID, FLAG_ACCEPTED, FLAG_INV_CONTIG, FLAG_INV_POP = 1, 2, 4, 8


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10; inputs broadcast, returns 4 uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) & MASK32 for x in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint64) & MASK32
    k1 = np.asarray(k1, dtype=np.uint64) & MASK32
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & MASK32
            k1 = (k1 + _W1) & MASK32
        p0 = _M0 * c0
        p1 = _M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & MASK32,
                          (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & MASK32)
    return tuple(np.asarray(x, dtype=np.uint32) for x in (c0, c1, c2, c3))


def node_words_k2(seed: int, chain_id: int, d) -> np.ndarray:
    """k = 2 node stream (flipref.c draw_words): the node word of draw d is word d mod 4 of the
    purpose-3 Philox call at counter d // 4."""
    d = np.asarray(d, dtype=np.uint64)
    q = d >> np.uint64(2)
    w = philox4x32_10(q & MASK32, q >> np.uint64(32), chain_id, 3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return np.choose((d & np.uint64(3)).astype(np.int64), w).astype(np.uint32)


def draw_tape(seed: int, chain_id: int, n_draws: int, start: int = 0, *, k: int) -> np.ndarray:
    """The canonical stream as an explicit tape: 6 u32 per draw (4 proposal words, then the
    2 geometric-wait words of purpose 1); k = 2 takes word 0 from the four-per-call node stream,
    k > 2 from the draw's own purpose-0 call.  ``k`` is required: the two streams differ in word
    0, and a tape replayed on both sides would not show a wrong choice."""
    d = np.arange(start, start + n_draws, dtype=np.uint64)
    lo, hi = d & MASK32, d >> np.uint64(32)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    a = philox4x32_10(lo, hi, chain_id, 0, k0, k1)
    g = philox4x32_10(lo, hi, chain_id, 1, k0, k1)
    w0 = node_words_k2(seed, chain_id, d) if k == 2 else a[0]
    tape = np.stack([w0, a[1], a[2], a[3], g[0], g[1]], axis=1)
    return np.ascontiguousarray(tape.reshape(-1), dtype=np.uint32)


def u53(a: int, b: int) -> float:
    """CPython ``random.random()`` from two 32-bit words."""
    return ((a >> 5) * 67108864.0 + (b >> 6)) * (1.0 / 9007199254740992.0)


# --------------------------------------------------------------------------------------
# ctypes binding of flipref.c
# --------------------------------------------------------------------------------------
class FrRecord(ctypes.Structure):
    _fields_ = [("draw", ctypes.c_int64), ("v", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("cut", ctypes.c_int32), ("nb", ctypes.c_int32), ("wait", ctypes.c_int64)]


RECORD_DTYPE = np.dtype([("draw", "<i8"), ("v", "<i4"), ("flags", "<i4"), ("cut", "<i4"),
                         ("nb", "<i4"), ("wait", "<i8")])


class FrStats(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_int64), ("proposals", ctypes.c_int64), ("draws", ctypes.c_int64),
                ("accepted", ctypes.c_int64), ("inv_contig", ctypes.c_int64), ("inv_pop", ctypes.c_int64),
                ("sum_cut", ctypes.c_int64), ("sum_nb", ctypes.c_int64), ("sum_wait", ctypes.c_int64),
                ("sum_cut2", ctypes.c_double), ("sum_nb2", ctypes.c_double),
                ("cut", ctypes.c_int32), ("nb", ctypes.c_int32),
                ("wait0", ctypes.c_int64), ("wait_cur", ctypes.c_int64),
                ("last_flip", ctypes.c_int32), ("stuck", ctypes.c_int32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_P = ctypes.POINTER


class FrParams(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("row_ptr", _P(ctypes.c_int32)), ("col_idx", _P(ctypes.c_int32)),
                ("pop", _P(ctypes.c_int32)), ("k", ctypes.c_int32), ("labels", _P(ctypes.c_int32)),
                ("base", ctypes.c_double), ("pop_lo", ctypes.c_int64), ("pop_hi", ctypes.c_int64),
                ("seed", ctypes.c_uint64), ("chain_id", ctypes.c_uint32),
                ("tape", _P(ctypes.c_uint32)), ("tape_draws", ctypes.c_int64),
                ("n_steps", ctypes.c_int64), ("max_draws", ctypes.c_int64),
                ("log1mp", _P(ctypes.c_double)), ("proposal", ctypes.c_int32), ("wmax", ctypes.c_int32),
                ("accept", ctypes.c_int32), ("con_valid", ctypes.c_uint32), ("con_accept", ctypes.c_uint32),
                ("beta", ctypes.c_double), ("boundary", _P(ctypes.c_uint8)), ("pinned", _P(ctypes.c_int32)),
                ("n_pinned", ctypes.c_int32), ("wait0_words", _P(ctypes.c_uint32)),
                ("stream", ctypes.c_int32), ("nb_pairs", ctypes.c_int32)]


ACCEPT_CUT, ACCEPT_UNIFORM, ACCEPT_ANNEAL = 0, 1, 2
CON_CONTIG, CON_POP, CON_BOUNDARY, CON_FIXED, CON_EMPTY = 1, 2, 4, 8, 0x100


PROPOSE_BI_SIGN, PROPOSE_PAIR = 0, 1
STREAM_NODE, STREAM_BAND = 0, 1  # flipref.h FR_STREAM_*


class FrOutputs(ctypes.Structure):
    _fields_ = [("trace", _P(FrRecord)), ("trace_cap", ctypes.c_int64), ("trace_len", ctypes.c_int64),
                ("final_assign", _P(ctypes.c_int8)), ("cut_hist", _P(ctypes.c_int64)),
                ("nb_hist", _P(ctypes.c_int64)), ("cut_times", _P(ctypes.c_int64)),
                ("num_flips", _P(ctypes.c_int64)), ("part_sum", _P(ctypes.c_int64)),
                ("last_flipped", _P(ctypes.c_int64)),
                # corrected companions, flipref.h fr_outputs
                ("flip_count", _P(ctypes.c_int64)), ("occupancy", _P(ctypes.c_int64)),
                ("last_accept", _P(ctypes.c_int64))]


def build_lib(force: bool = False) -> str:
    def stale():
        return force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < max(os.path.getmtime(os.path.join(HERE, f))
                                             for f in ("flipref.c", "flipref.h", "recomref.c", "recomref.h"))
    if stale():
        import fcntl  # one build at a time (pytest-xdist workers share oracle/build)
        os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
        with open(os.path.join(os.path.dirname(LIB_PATH), ".lock"), "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                if stale():
                    subprocess.run(["make", "-C", HERE, "-s"], check=True)
            finally:
                fcntl.flock(lk, fcntl.LOCK_UN)
    return LIB_PATH


def _ptr(arr, ctype):
    if arr is None:
        return ctypes.POINTER(ctype)()
    return arr.ctypes.data_as(ctypes.POINTER(ctype))


def nb_width(spec, k: int, nb_pairs: bool) -> int:
    """Entries of the |B| histogram / log(1 - p) table: n + 1, or with ``nb_pairs`` (|b_nodes|
    counted as the pair updater's (node, district) pairs, grid_chain_sec11.py:151-153) one more
    than the largest pair count, sum_u min(deg u, k - 1)."""
    if not nb_pairs:
        return spec.n + 1
    deg = np.diff(np.asarray(spec.row_ptr, dtype=np.int64))
    return int(np.minimum(deg, k - 1).sum()) + 1


class CRef:
    """The plain-C oracle.  ``run`` restates one chain from its initial state."""

    def __init__(self, lib_path: Optional[str] = None):
        path = lib_path or LIB_PATH
        if not os.path.exists(path):
            build_lib()
        self.lib = ctypes.CDLL(path)
        self.lib.fr_run.argtypes = [_P(FrParams), _P(ctypes.c_int8), _P(FrStats), _P(FrOutputs)]
        self.lib.fr_run.restype = ctypes.c_int
        self.lib.fr_flip_contiguous.argtypes = [ctypes.c_int32, _P(ctypes.c_int32), _P(ctypes.c_int32),
                                                _P(ctypes.c_int8), ctypes.c_int32]
        self.lib.fr_districts_contiguous.argtypes = [ctypes.c_int32, _P(ctypes.c_int32), _P(ctypes.c_int32),
                                                     ctypes.c_int32, _P(ctypes.c_int8)]
        self.lib.fr_philox4x32_10.argtypes = [_P(ctypes.c_uint32), _P(ctypes.c_uint32), _P(ctypes.c_uint32)]

    def philox(self, ctr, key):
        c = (ctypes.c_uint32 * 4)(*ctr)
        k = (ctypes.c_uint32 * 2)(*key)
        o = (ctypes.c_uint32 * 4)()
        self.lib.fr_philox4x32_10(c, k, o)
        return list(o)

    def districts_contiguous(self, spec, assign: np.ndarray, k: int) -> bool:
        a = np.ascontiguousarray(assign, dtype=np.int8)
        return self.lib.fr_districts_contiguous(spec.n, _ptr(spec.row_ptr, ctypes.c_int32),
                                                _ptr(spec.col_idx, ctypes.c_int32), k,
                                                _ptr(a, ctypes.c_int8)) == 1

    def flip_contiguous(self, spec, assign: np.ndarray, v: int) -> bool:
        a = np.ascontiguousarray(assign, dtype=np.int8)
        return self.lib.fr_flip_contiguous(spec.n, _ptr(spec.row_ptr, ctypes.c_int32),
                                           _ptr(spec.col_idx, ctypes.c_int32), _ptr(a, ctypes.c_int8), v) == 1

    def run(self, spec, init_assign: np.ndarray, *, base: float, pop_lo: int, pop_hi: int,
            seed: int, chain_id: int, n_steps: int, k: int = 2, labels=(-1, 1),
            log1mp: Optional[np.ndarray] = None, tape: Optional[np.ndarray] = None,
            max_draws: int = 0, trace_cap: int = 0, want_hist: bool = False,
            want_edges: bool = False, want_flips: bool = False, proposal: int = 0, wmax: int = 0,
            accept: int = 0, con_valid: int = 0, con_accept: int = 0, beta: float = 0.0,
            boundary: Optional[np.ndarray] = None, pinned: Optional[np.ndarray] = None,
            wait0_words: Optional[np.ndarray] = None, want_exact_flips: bool = False,
            stream: int = STREAM_NODE, nb_pairs: bool = False) -> Dict:
        n, E = spec.n, spec.n_edges
        row_ptr = np.ascontiguousarray(spec.row_ptr, dtype=np.int32)
        col_idx = np.ascontiguousarray(spec.col_idx, dtype=np.int32)
        pop = np.ascontiguousarray(spec.pop, dtype=np.int32)
        if labels is None or len(labels) != k:
            labels = list(range(k))
        lab = np.ascontiguousarray(labels, dtype=np.int32)
        init = np.ascontiguousarray(init_assign, dtype=np.int8)
        l1 = None if log1mp is None else np.ascontiguousarray(log1mp, dtype=np.float64)
        tp = None if tape is None else np.ascontiguousarray(tape, dtype=np.uint32)
        bnd = None if boundary is None else np.ascontiguousarray(boundary, dtype=np.uint8)
        pin = None if pinned is None else np.ascontiguousarray(pinned, dtype=np.int32).reshape(-1)
        w0 = None if wait0_words is None else np.ascontiguousarray(wait0_words, dtype=np.uint32).reshape(2)
        p = FrParams(n=n, row_ptr=_ptr(row_ptr, ctypes.c_int32), col_idx=_ptr(col_idx, ctypes.c_int32),
                     pop=_ptr(pop, ctypes.c_int32), k=k, labels=_ptr(lab, ctypes.c_int32),
                     base=float(base), pop_lo=int(pop_lo), pop_hi=int(pop_hi), seed=int(seed),
                     chain_id=int(chain_id), tape=_ptr(tp, ctypes.c_uint32),
                     tape_draws=0 if tp is None else tp.shape[0] // 6,
                     n_steps=int(n_steps), max_draws=int(max_draws), log1mp=_ptr(l1, ctypes.c_double),
                     proposal=int(proposal), wmax=int(wmax), accept=int(accept), con_valid=int(con_valid),
                     con_accept=int(con_accept), beta=float(beta), boundary=_ptr(bnd, ctypes.c_uint8),
                     pinned=_ptr(pin, ctypes.c_int32), n_pinned=0 if pin is None else pin.size // 2,
                     wait0_words=_ptr(w0, ctypes.c_uint32), stream=int(stream), nb_pairs=int(bool(nb_pairs)))
        trace = np.zeros(trace_cap, dtype=RECORD_DTYPE) if trace_cap else None
        final = np.zeros(n, dtype=np.int8)
        cut_hist = np.zeros(E + 1, dtype=np.int64) if want_hist else None
        nb_w = nb_width(spec, k, nb_pairs)
        nb_hist = np.zeros(nb_w, dtype=np.int64) if want_hist else None
        cut_times = np.zeros(E, dtype=np.int64) if want_edges else None
        nf = np.zeros(n, dtype=np.int64) if want_flips else None
        ps = np.zeros(n, dtype=np.int64) if want_flips else None
        lf = np.zeros(n, dtype=np.int64) if want_flips else None
        xfc, xocc, xla = ((np.zeros(n, dtype=np.int64) for _ in range(3)) if want_exact_flips
                          else (None, None, None))
        o = FrOutputs(trace=ctypes.cast(trace.ctypes.data, _P(FrRecord)) if trace is not None else _P(FrRecord)(),
                      trace_cap=trace_cap, trace_len=0, final_assign=_ptr(final, ctypes.c_int8),
                      cut_hist=_ptr(cut_hist, ctypes.c_int64), nb_hist=_ptr(nb_hist, ctypes.c_int64),
                      cut_times=_ptr(cut_times, ctypes.c_int64), num_flips=_ptr(nf, ctypes.c_int64),
                      part_sum=_ptr(ps, ctypes.c_int64), last_flipped=_ptr(lf, ctypes.c_int64),
                      flip_count=_ptr(xfc, ctypes.c_int64), occupancy=_ptr(xocc, ctypes.c_int64),
                      last_accept=_ptr(xla, ctypes.c_int64))
        st = FrStats()
        rc = self.lib.fr_run(ctypes.byref(p), _ptr(init, ctypes.c_int8), ctypes.byref(st), ctypes.byref(o))
        if rc == -1:
            raise ValueError("The given initial_state is not valid according is_valid.")
        if rc == -2:
            raise RuntimeError("fr_run: bad arguments")
        out = {"rc": rc, "stats": st.as_dict(), "final": final}
        if trace is not None:
            out["trace"] = trace[:o.trace_len].copy()
        if want_hist:
            out["cut_hist"], out["nb_hist"] = cut_hist, nb_hist
        if want_edges:
            out["cut_times"] = cut_times
        if want_flips:
            out["num_flips"], out["part_sum"], out["last_flipped"] = nf, ps, lf
        if want_exact_flips:
            out["flip_count"], out["occupancy"], out["last_accept"] = xfc, xocc, xla
        return out


# --------------------------------------------------------------------------------------
# gerrychain-0.2-faithful pure-Python restatement ("reference Python CPU path")
# --------------------------------------------------------------------------------------
class _Partition:
    """Partition [gc-0.2]: ``flip`` builds a child that copies the node->part dict and
    rebuilds the affected part frozensets (O(N)); updaters are lazy and cached per object."""

    __slots__ = ("graph", "assignment", "parts", "parent", "flips", "_cache", "_ups")

    def __init__(self, graph, assignment=None, updaters=None, parent=None, flips=None):
        self.graph = graph
        self._cache = {}
        if parent is None:
            self.assignment = dict(assignment)
            parts = {}
            for nd, p in self.assignment.items():
                parts.setdefault(p, set()).add(nd)
            self.parts = {p: frozenset(s) for p, s in parts.items()}
            self._ups = dict(updaters)
            self.parent = None
            self.flips = None
        else:
            self._ups = parent._ups
            self.parent = parent
            self.flips = flips
            self.assignment = parent.assignment.copy()
            self.assignment.update(flips)
            parts = dict(parent.parts)
            touched = set(flips.values()) | {parent.assignment[nd] for nd in flips}
            for p in touched:
                parts[p] = frozenset(nd for nd, q in self.assignment.items() if q == p)
            self.parts = parts

    def flip(self, flips):
        return _Partition(self.graph, parent=self, flips=flips)

    def __getitem__(self, key):
        if key not in self._cache:
            self._cache[key] = self._ups[key](self)
        return self._cache[key]

    def __len__(self):
        return len(self.parts)


def _cut_edges(partition):  # gerrychain.updaters.cut_edges [gc-0.2]
    if partition.parent is None:
        a = partition.assignment
        return {tuple(sorted(e)) for e in partition.graph.edges if a[e[0]] != a[e[1]]}
    parent_cut = partition.parent["cut_edges"]
    a = partition.assignment
    new_cuts, obsolete = set(), set()
    for node in partition.flips:
        for nb in partition.graph.neighbors(node):
            e = tuple(sorted((node, nb)))
            if a[node] != a[nb]:
                new_cuts.add(e)
            else:
                obsolete.add(e)
    return (parent_cut | new_cuts) - obsolete


def _b_nodes_pairs(partition):  # b_nodes, grid_chain_sec11.py:151-153
    a = partition.assignment
    cut = partition["cut_edges"]
    return {(x[0], a[x[1]]) for x in cut}.union({(x[1], a[x[0]]) for x in cut})


def _pair_slot_bound(partition):
    """The canonical PAIR stream's slot bound: the state's largest number of foreign districts
    of one node (>= 1), i.e. the largest count of b_nodes pairs (:151-153) sharing a node."""
    cnt: Dict = {}
    for x, _ in partition["pairs"]:
        cnt[x] = cnt.get(x, 0) + 1
    return max(cnt.values(), default=1)


def _b_nodes_bi(partition):  # grid_chain_sec11.py:155-156
    return {x[0] for x in partition["cut_edges"]}.union({x[1] for x in partition["cut_edges"]})


def _population(partition):  # Tally('population') [gc-0.2], incremental from the parent
    if partition.parent is None:
        out = {}
        for nd, p in partition.assignment.items():
            out[p] = out.get(p, 0) + partition.graph.nodes[nd]["population"]
        return out
    out = dict(partition.parent["population"])
    for nd, new in partition.flips.items():
        pop = partition.graph.nodes[nd]["population"]
        out[partition.parent.assignment[nd]] -= pop
        out[new] = out.get(new, 0) + pop
    return out


def _single_flip_contiguous(partition):  # [gc-0.2] restated
    import networkx as nx
    graph, assignment = partition.graph, partition.assignment

    def avoid(start, end, attrs):
        return None if assignment[start] != assignment[end] else 1

    for changed, _ in partition.flips.items():
        old = partition.parent.assignment[changed]
        old_nbrs = [nd for nd in graph.neighbors(changed) if assignment[nd] == old]
        if not old_nbrs:
            return False
        start = old_nbrs[0]  # canonical stream: the choice does not change the outcome
        for nbr in old_nbrs:
            try:
                nx.multi_source_dijkstra(graph, [nbr], target=start, weight=avoid)
            except nx.NetworkXNoPath:
                return False
    return True


class GcFaithfulChain:
    """One k=2 chain restated with gerrychain 0.2 structures, driven by the canonical
    stream (Philox or a tape): node-tape replay of ``slow_reversible_propose_bi``."""

    def __init__(self, spec, plan: Dict, *, base: float, pop_bounds, seed: int, chain_id: int,
                 log1mp: Optional[np.ndarray] = None, tape: Optional[np.ndarray] = None,
                 pair: bool = False, wmax: int = 0, band: bool = False, nb_pairs: bool = False):
        self.spec = spec
        # |b_nodes| as len(partition["b_nodes"]) sees it: the nodes of b_nodes_bi (:155-156), or
        # with nb_pairs the (node, district) pairs of the pair updater b_nodes (:151-153), which a
        # k > 2 driver running slow_reversible_propose registers as "b_nodes"
        self.nb_key = "pairs" if nb_pairs else "b_nodes"
        self.g = spec.nx_graph
        self.base = base
        self.lo, self.hi = pop_bounds  # float bounds, exactly as Bounds compares
        self.seed, self.chain_id = seed, chain_id
        self.log1mp = log1mp
        self.tape = tape
        self.labels = sorted(set(plan.values()))
        ups = {"population": _population, "cut_edges": _cut_edges, "b_nodes": _b_nodes_bi, "pairs": _b_nodes_pairs,
               "pair_slots": _pair_slot_bound}
        self.state = _Partition(self.g, assignment=plan, updaters=ups)
        self.d = 0
        self.n = spec.n
        self.thresh = (1 << 32) % self.n
        self.pair = pair
        k = len(self.labels)
        # slot bound: fixed (wmax > 0) or the canonical dynamic one, the state's largest
        # foreign-district count (oracle/flipref.c)
        self.wmax = wmax if wmax > 0 else 0
        self.stats = dict(steps=0, proposals=0, draws=0, accepted=0, inv_contig=0, inv_pop=0,
                          sum_cut=0, sum_nb=0, sum_wait=0)
        self.trace = []
        # band stream (flipref.h FR_STREAM_BAND): nodes drawn over S = b_nodes + neighbours,
        # ascending, rebuilt only when a node enters b_nodes outside S
        self.band = band
        if band:
            self._band_build()
        self.wait = self._geom(0, 2)
        self._yield()

    def _band_build(self):
        idx = self.spec.index
        S = set()
        for x in self.state["b_nodes"]:
            S.add(idx[x])
            S.update(idx[y] for y in self.g.neighbors(x))
        self.band_set = S
        self.band_list = sorted(S)

    def _words(self, d, purpose):
        if self.tape is not None and purpose != 2:
            t = self.tape[6 * d: 6 * d + 6]
            return [int(x) for x in (t[:4] if purpose == 0 else t[4:6])]
        w = [int(x) for x in philox4x32_10(d & 0xFFFFFFFF, d >> 32, self.chain_id, purpose,
                                            self.seed & 0xFFFFFFFF, self.seed >> 32)]
        if purpose == 0 and len(self.labels) == 2 and not self.band:  # k = 2 node stream
            w[0] = int(node_words_k2(self.seed, self.chain_id, d))
        return w

    def _geom(self, d, purpose):
        if self.log1mp is None:
            return 0
        w = self._words(d, purpose)
        U = u53(w[0], w[1])
        nb = len(self.state[self.nb_key])
        l1 = self.log1mp[nb]
        q = math.log(1.0 - U) / l1 if l1 != 0.0 else -math.inf
        if not abs(q) < 2.0 ** 62:
            return 1 << 62  # saturated, as the C restatement
        return int(math.ceil(q)) - 1

    def _yield(self):
        s = self.state
        self.stats["sum_cut"] += len(s["cut_edges"])
        self.stats["sum_nb"] += len(s[self.nb_key])
        self.stats["sum_wait"] += self.wait

    def _valid(self, proposal):
        if not _single_flip_contiguous(proposal):
            return FLAG_INV_CONTIG
        vals = proposal["population"].values()
        if not (self.lo <= min(vals) and max(vals) <= self.hi):
            return FLAG_INV_POP
        return 0

    def step(self):
        """Advance one valid step (MarkovChain.__next__ [gc-0.2])."""
        while True:
            draw = self.d
            w = self._words(draw, 0)
            self.d += 1
            self.stats["draws"] += 1
            ns = len(self.band_list) if self.band else self.n
            m = w[0] * ns
            if (m & 0xFFFFFFFF) < (1 << 32) % ns:
                continue
            node = self.spec.nodes[self.band_list[m >> 32] if self.band else m >> 32]
            s = self.state
            if node not in s["b_nodes"]:
                continue
            if self.pair:
                # slow_reversible_propose (:117-130): uniform over the (node, district) pairs
                # of b_nodes (:151-153) -- canonical: slot r < wcap, r-th foreign district
                wcap = self.wmax or s["pair_slots"]
                mw = w[3] * wcap
                if (mw & 0xFFFFFFFF) < (1 << 32) % wcap:
                    continue
                foreign = sorted({d for (x, d) in s["pairs"] if x == node}, key=self.labels.index)
                r = mw >> 32
                if r >= len(foreign):
                    continue
                target = foreign[r]
            else:
                target = -1 * s.assignment[node]  # :145 (labels are ±1)
            tid = self.labels.index(target) << 8
            self.stats["proposals"] += 1
            proposal = s.flip({node: target})
            s.parent = None  # MarkovChain.__next__ erases the grandparent [gc-0.2]
            bad = self._valid(proposal)
            if bad:
                self.stats["inv_contig" if bad == FLAG_INV_CONTIG else "inv_pop"] += 1
                self.trace.append((draw, self.spec.index[node], bad | tid, len(s["cut_edges"]), len(s[self.nb_key]), 0))
                continue
            self.stats["steps"] += 1
            bound = self.base ** (-len(proposal["cut_edges"]) + len(s["cut_edges"]))  # :175
            acc = u53(w[1], w[2]) < bound
            if acc:
                self.state = proposal
                self.stats["accepted"] += 1
                if self.band and any(self.spec.index[x] not in self.band_set for x in proposal["b_nodes"]):
                    self._band_build()
                self.wait = self._geom(draw, 1)
            self._yield()
            cur = self.state
            self.trace.append((draw, self.spec.index[node], FLAG_VALID | (FLAG_ACCEPTED if acc else 0) | tid,
                               len(cur["cut_edges"]), len(cur[self.nb_key]), self.wait))
            return cur

    def run(self, n_steps: int):
        for _ in range(n_steps):
            self.step()
        return self

    def assignment_ids(self):
        lut = {lab: i for i, lab in enumerate(self.labels)}
        return np.asarray([lut[self.state.assignment[nd]] for nd in self.spec.nodes], dtype=np.int8)


class NativeRngChain(GcFaithfulChain):
    """The reference's flip step under its own (native) random streams, for the
    distributional checks: ``random.choice(list(partition["b_nodes"]))`` (:143),
    ``random.random()`` in cut_accept (:179), ``np.random.geometric`` in geom_wait (:148),
    and the ``random.choice`` that gerrychain's single_flip_contiguous makes among the old
    neighbours [gc-0.2] -- CPython's Mersenne Twister and numpy's legacy RandomState,
    seeded per chain instead of globally.

    ``record=True`` also writes the **node tape** of SURVEY App. A.4: per proposal, the six
    words the device / C oracle replay (``fc_run_set_tape``) -- word 0 maps to the drawn node
    under the exact Lemire map, words 1-2 carry the 53-bit ``random()`` value of a valid
    proposal, words 4-5 the 53-bit ``random_sample()`` numpy's geometric inverted for the
    state it created -- plus the initial state's wait words (``fc_run_set_initial_wait``)
    and the per-proposal trace in the device's record layout.  Every draw of this chain is a
    proposal (it samples B itself), so tape draw i is proposal i.

    ``pair=True`` runs ``slow_reversible_propose`` (:117-130) instead: one
    ``random.choice(list(pairs))`` over the (node, district) pairs of ``b_nodes`` (:151-153),
    then ``partition.flip({node: district})``.  The pair set is the proposal's own (the inline
    form commented at :125-126); the ``"b_nodes"`` updater stays ``b_nodes_bi`` as registered at
    :305, so ``geom_wait`` (:148) and the driver's ``rbn`` (:369) keep counting nodes; with
    ``nb_pairs=True`` they count the pairs instead, as in a driver that registers the pair updater
    ``b_nodes`` under ``"b_nodes"`` (which ``slow_reversible_propose`` reads, :128).  The node
    tape then also carries word 3: the Lemire word that sends the state's slot bound ``wcap``
    (its largest foreign-district count, the canonical PAIR stream's bound) to the drawn
    district's rank among the node's foreign districts, ascending."""

    def __init__(self, spec, plan: Dict, *, base: float, pop_bounds, seed: int,
                 log1mp: Optional[np.ndarray] = None, record: bool = False, pair: bool = False,
                 nb_pairs: bool = False):
        import random as _random
        self.rng = _random.Random(seed)
        self.nprng = np.random.RandomState(seed & 0xFFFFFFFF)
        self.record = record
        self.tape_words = []      # 6 u32 per proposal
        self.wait0_words = None
        self._geom_words = None   # words of the last geometric draw
        super().__init__(spec, plan, base=base, pop_bounds=pop_bounds, seed=seed, chain_id=0, log1mp=log1mp,
                         pair=pair, nb_pairs=nb_pairs)
        if record:
            self.wait0_words = self._geom_words

    @staticmethod
    def _u53_words(u: float):
        """(a, b) with ((a >> 5) * 2^26 + (b >> 6)) / 2^53 == u (CPython random(), numpy
        random_sample()): the exact inverse of u53 for any 53-bit double in [0, 1)."""
        x = int(u * 9007199254740992.0)
        assert x / 9007199254740992.0 == u
        return (x >> 26) << 5, (x & ((1 << 26) - 1)) << 6

    @staticmethod
    def _lemire_word(v: int, N: int) -> int:
        """x0 with (x0 * N) >> 32 == v and (x0 * N) mod 2^32 >= 2^32 mod N (never rejected)."""
        x0 = (((v + 1) << 32) - 1) // N
        m = x0 * N
        assert m >> 32 == v and (m & 0xFFFFFFFF) >= (1 << 32) % N
        return x0

    def _node_word(self, v: int) -> int:
        return self._lemire_word(v, self.n)

    def _slot_word(self, node, target) -> int:
        """Word 3 of a PAIR proposal: rank of ``target`` among ``node``'s foreign districts
        (ascending label order, as the canonical stream ranks them) under the slot bound."""
        s = self.state
        a = s.assignment
        foreign = sorted({a[y] for y in self.g.neighbors(node) if a[y] != a[node]}, key=self.labels.index)
        wcap = s["pair_slots"]
        return self._lemire_word(foreign.index(target), wcap)

    def _geom(self, d, purpose):
        if self.log1mp is None:
            return 0
        s = self.state
        p = len(list(s[self.nb_key])) / (len(self.g.nodes) ** len(self.labels) - 1)  # :148
        if self.record:
            clone = np.random.RandomState()
            clone.set_state(self.nprng.get_state())
            U = clone.random_sample()
            self._geom_words = self._u53_words(U)
        w = int(self.nprng.geometric(p, 1)[0]) - 1
        nb = len(s[self.nb_key])
        if float(self.log1mp[nb]) == 0.0:
            # 1 - p rounds to 1.0 (N^k beyond 2^53 |B|, e.g. k = 8 on 3,120 nodes): numpy's
            # inversion divides by log(1.0) = 0 and casts +inf to int64, which gives INT64_MIN;
            # the C restatement and the device saturate at 2^62 instead (flipref.c geom_wait).
            assert w == -(1 << 63) - 1, (p, w)
            return 1 << 62
        if self.record:  # the replayed inversion must give numpy's own answer
            q = math.log(1.0 - U) / float(self.log1mp[nb])
            assert int(math.ceil(q)) - 1 == w, (U, p, w)
        return w

    def step(self):
        while True:
            s = self.state
            if self.pair:
                node, target = self.rng.choice(list(s["pairs"]))  # :128 over the :151-153 pairs
            else:
                node = self.rng.choice(list(s["b_nodes"]))  # :143
                target = -1 * s.assignment[node]  # :145
            draw = self.stats["draws"]
            self.stats["draws"] += 1
            self.stats["proposals"] += 1
            tid = self.labels.index(target) << 8
            words = [self._node_word(self.spec.index[node]), 0, 0, 0, 0, 0] if self.record else None
            if self.record and self.pair:
                words[3] = self._slot_word(node, target)
            proposal = s.flip({node: target})
            s.parent = None
            old_nbrs = [nd for nd in self.g.neighbors(node) if proposal.assignment[nd] == s.assignment[node]]
            if old_nbrs:
                self.rng.choice(old_nbrs)  # single_flip_contiguous's start node [gc-0.2]
            bad = self._valid(proposal)
            if bad:
                self.stats["inv_contig" if bad == FLAG_INV_CONTIG else "inv_pop"] += 1
                if self.record:
                    self.tape_words.extend(words)
                    self.trace.append((draw, self.spec.index[node], bad | tid, len(s["cut_edges"]),
                                       len(s[self.nb_key]), 0))
                continue
            self.stats["steps"] += 1
            bound = self.base ** (-len(proposal["cut_edges"]) + len(s["cut_edges"]))  # :175
            u = self.rng.random()
            acc = u < bound  # :179
            if self.record:
                words[1], words[2] = self._u53_words(u)
            if acc:
                self.state = proposal
                self.stats["accepted"] += 1
                if self.band and any(self.spec.index[x] not in self.band_set for x in proposal["b_nodes"]):
                    self._band_build()
                self.wait = self._geom(0, 1)
                if self.record:
                    words[4], words[5] = self._geom_words
            self._yield()
            if self.record:
                self.tape_words.extend(words)
                cur = self.state
                self.trace.append((draw, self.spec.index[node], FLAG_VALID | (FLAG_ACCEPTED if acc else 0) | tid,
                                   len(cur["cut_edges"]), len(cur[self.nb_key]), self.wait))
            return self.state

    def node_tape(self) -> np.ndarray:
        """The recorded node tape, ``[proposals * 6]`` u32."""
        return np.asarray(self.tape_words, dtype=np.uint32)

    def trace_array(self) -> np.ndarray:
        return np.asarray(self.trace, dtype=[("draw", "<i8"), ("v", "<i4"), ("flags", "<i4"), ("cut", "<i4"),
                                             ("nb", "<i4"), ("wait", "<i8")])


# --------------------------------------------------------------------------------------
# Series diagnostics restated from a proposal trace (checker for FC_DIAG_SERIES).
# The reference driver keeps the per-yield lists rce / rbn (grid_chain_sec11.py:367-369);
# C4 asks for their autocorrelation and a hitting time of a target |cut|.
# --------------------------------------------------------------------------------------
def yield_series(trace: np.ndarray, x0: int, field: str = "cut") -> np.ndarray:
    """Per-yield values (yield 0 = the initial state with value ``x0``; one yield per
    valid proposal) from an oracle/device proposal trace."""
    valid = (trace["flags"] & FLAG_VALID) != 0
    return np.concatenate([[x0], trace[field][valid]]).astype(np.int64)


def events_from_trace(trace: np.ndarray) -> np.ndarray:
    """(t, v, cut, nb, target) of every accepted flip: t = yield index it creates."""
    valid = (trace["flags"] & FLAG_VALID) != 0
    t = np.cumsum(valid.astype(np.int64))
    acc = (trace["flags"] & FLAG_ACCEPTED) != 0
    return np.stack([t[acc], trace["v"][acc], trace["cut"][acc], trace["nb"][acc],
                     (trace["flags"][acc] >> 8) & 0xFF], axis=1).astype(np.int64)


def hitting_time(series: np.ndarray, lo: int, hi: int) -> int:
    hit = np.nonzero((series >= lo) & (series <= hi))[0]
    return int(hit[0]) if hit.size else -1


def acf_exact(x: np.ndarray, lags) -> tuple:
    """Biased sample ACF (statsmodels ``acf`` default) of an integer series, formed exactly
    as ``fc_run_autocorr`` does: integer lag sums, then one rounding of the exact rational
    T^2 sum (x_t - m)(x_{t+L} - m) / (T^2 sum (x_t - m)^2) to double.  Returns
    ``(lag_sums, acf)``."""
    xs = [int(v) for v in x]
    T = len(xs)
    Sx = sum(xs)
    Sxx = sum(v * v for v in xs)
    sums, out = [], []
    for L in lags:
        L = int(L)
        if L >= T:
            sums.append(0)
            out.append(0.0)
            continue
        P = sum(xs[t] * xs[t + L] for t in range(T - L))
        H = sum(xs[:T - L])
        G = sum(xs[L:])
        num = T * T * P - T * Sx * (H + G) + (T - L) * Sx * Sx
        den = T * (T * Sxx - Sx * Sx)
        sums.append(P)
        out.append(float(num) / float(den) if den else 0.0)
    return np.asarray(sums, dtype=np.int64), np.asarray(out, dtype=np.float64)


def acf_float(x: np.ndarray, lags) -> np.ndarray:
    """The same ACF in plain float64 numpy (tolerance cross-check)."""
    x = np.asarray(x, dtype=np.float64)
    d = x - x.mean()
    den = float(np.dot(d, d))
    return np.asarray([float(np.dot(d[:len(d) - L], d[L:])) / den if L < len(d) and den else 0.0
                       for L in lags])


# --------------------------------------------------------------------------------------
# boundary_slope + the driver's slope / angle lines (checker for fc_run_frame_series).
# grid_chain_sec11.py:55-78 (sec11 frame) and Frankenstein_chain.py:55-78 (FRANK frame),
# loop body grid_chain_sec11.py:371-394 / Frankenstein_chain.py:399-422.  Restated over
# node-label tuples exactly as the reference's updater sees partition["cut_edges"].
# --------------------------------------------------------------------------------------
_SEC11_E = [((0, 1), (1, 0)), ((0, 38), (1, 39)), ((38, 0), (39, 1)), ((38, 39), (39, 38))]
_SEC11_E_REV = [((1, 0), (0, 1)), ((1, 39), (0, 38)), ((39, 1), (38, 0)), ((39, 38), (38, 39))]


def boundary_slope(cut_edges, kind: str = "sec11") -> list:
    """``boundary_slope(partition)`` on a cut-edge collection of node-label pairs."""
    a, b, c, d, e = [], [], [], [], []
    if kind == "sec11":
        lim = (0, 0, 39, 39)
    else:  # Frankenstein_chain.py:59-66
        lim = (0, -19, 19, 20)
    for x in cut_edges:
        if x[0][0] == lim[0] and x[1][0] == lim[0]:
            a.append(x)
        elif x[0][1] == lim[1] and x[1][1] == lim[1]:
            b.append(x)
        elif x[0][0] == lim[2] and x[1][0] == lim[2]:
            c.append(x)
        elif x[0][1] == lim[3] and x[1][1] == lim[3]:
            d.append(x)
        elif kind == "sec11" and x in _SEC11_E:
            e.append(x)
        elif kind == "sec11" and x in _SEC11_E_REV:
            e.append(x)
    return list(set(a + b + c + d + e))


def slope_angle(temp) -> tuple:
    """The driver's per-yield lines on ``temp = part["slope"]`` (``:374-394``): raises
    IndexError for fewer than two frame edges, as the reference does."""
    enda = ((temp[0][0][0] + temp[0][1][0]) / 2, (temp[0][0][1] + temp[0][1][1]) / 2)
    endb = ((temp[1][0][0] + temp[1][1][0]) / 2, (temp[1][0][1] + temp[1][1][1]) / 2)
    if endb[0] != enda[0]:
        slope = (endb[1] - enda[1]) / (endb[0] - enda[0])
    else:
        slope = np.inf
    anga = (enda[0] - 20, enda[1] - 20)
    angb = (endb[0] - 20, endb[1] - 20)
    angle = np.arccos(np.clip(np.dot(anga / np.linalg.norm(anga), angb / np.linalg.norm(angb)), -1, 1))
    return float(slope), float(angle)


def cut_edge_labels(spec, assign: np.ndarray) -> set:
    """gerrychain ``cut_edges`` of a district-id array, as sorted node-label tuples [gc-0.2]."""
    e = spec.edges()
    m = assign[e[:, 0]] != assign[e[:, 1]]
    return {tuple(sorted((spec.nodes[u], spec.nodes[v]))) for u, v in e[m]}


# --------------------------------------------------------------------------------------
# ReCom (oracle/recomref.c): gerrychain 0.2 recom + bipartition_tree restated
# (grid_chain_sec11.py:328-335 builds it), checker of the HIP ReCom kernel.
# --------------------------------------------------------------------------------------
class RrParams(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("row_ptr", _P(ctypes.c_int32)), ("col_idx", _P(ctypes.c_int32)),
                ("pop", _P(ctypes.c_int32)), ("k", ctypes.c_int32), ("pop_target", ctypes.c_double),
                ("epsilon", ctypes.c_double), ("node_repeats", ctypes.c_int32), ("max_attempts", ctypes.c_int32),
                ("pop_lo", ctypes.c_int64), ("pop_hi", ctypes.c_int64), ("base", ctypes.c_double),
                ("seed", ctypes.c_uint64), ("chain_id", ctypes.c_uint32), ("n_steps", ctypes.c_int64),
                ("max_draws", ctypes.c_int64)]


class RrStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int64) for f in ("steps", "proposals", "accepted", "inv_pop", "attempts", "trees",
                                             "sum_cut", "sum_nb")] + \
               [(f, ctypes.c_int32) for f in ("cut", "nb", "stuck", "pad")]


RR_RECORD_DTYPE = np.dtype([("draw", "<i8"), ("edge", "<i4"), ("root", "<i4"), ("child", "<i4"),
                            ("attempts", "<i4"), ("flags", "<i4"), ("cut", "<i4")])


def recom_run(spec, init_assign: np.ndarray, *, k: int, pop_target: float, epsilon: float, pop_lo: int,
              pop_hi: int, seed: int, chain_id: int, n_steps: int, node_repeats: int = 1, base: float = 1.0,
              max_attempts: int = 100000, max_draws: int = 0, trace_cap: int = 0) -> Dict:
    """One ReCom chain on the CPU (``rr_run``): stats, final assignment, per-proposal trace."""
    L = ctypes.CDLL(build_lib())
    L.rr_run.argtypes = [ctypes.POINTER(RrParams), _P(ctypes.c_int8), ctypes.POINTER(RrStats), _P(ctypes.c_int8),
                         ctypes.c_void_p, ctypes.c_int64, _P(ctypes.c_int64)]
    row_ptr = np.ascontiguousarray(spec.row_ptr, dtype=np.int32)
    col_idx = np.ascontiguousarray(spec.col_idx, dtype=np.int32)
    pop = np.ascontiguousarray(spec.pop, dtype=np.int32)
    init = np.ascontiguousarray(init_assign, dtype=np.int8)
    p = RrParams(n=spec.n, row_ptr=_ptr(row_ptr, ctypes.c_int32), col_idx=_ptr(col_idx, ctypes.c_int32),
                 pop=_ptr(pop, ctypes.c_int32), k=k, pop_target=float(pop_target), epsilon=float(epsilon),
                 node_repeats=int(node_repeats), max_attempts=int(max_attempts), pop_lo=int(pop_lo),
                 pop_hi=int(pop_hi), base=float(base), seed=int(seed), chain_id=int(chain_id),
                 n_steps=int(n_steps), max_draws=int(max_draws))
    st = RrStats()
    final = np.zeros(spec.n, dtype=np.int8)
    trace = np.zeros(max(trace_cap, 1), dtype=RR_RECORD_DTYPE)
    tl = ctypes.c_int64(0)
    rc = L.rr_run(ctypes.byref(p), _ptr(init, ctypes.c_int8), ctypes.byref(st), _ptr(final, ctypes.c_int8),
                  ctypes.c_void_p(trace.ctypes.data), int(trace_cap), ctypes.byref(tl))
    if rc == -1:
        raise ValueError("The given initial_state is not valid according is_valid.")
    if rc == -2:
        raise RuntimeError("rr_run: bad arguments")
    return {"rc": rc, "stats": {f: int(getattr(st, f)) for f, _ in RrStats._fields_}, "final": final,
            "trace": trace[:tl.value].copy()}
