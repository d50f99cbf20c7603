"""Batched multi-chain engine over the C-ABI: the MI355X replacement of the reference's
``Partition`` + ``MarkovChain`` hot loop (``grid_chain_sec11.py:316-408``).

``FlipGraph`` owns an ``fc_graph`` (CSR + link rings, built natively from a
:class:`~flipcomplexityempirical_amd.graphs.GraphSpec`); ``FlipRun`` owns an ``fc_run``
(``n_chains`` independent k=2 chains, one per wavefront on the device).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check
from .graphs import GraphSpec, log1mp_table, nb_width

_P = ctypes.POINTER

STAT_FIELDS = [f for f, _ in _lib.ChainStats._fields_]
RECORD_DTYPE = np.dtype([("draw", "<i8"), ("v", "<i4"), ("flags", "<i4"), ("cut", "<i4"),
                         ("nb", "<i4"), ("wait", "<i8")])
RECOM_RECORD_DTYPE = np.dtype([("draw", "<i8"), ("edge", "<i4"), ("root", "<i4"), ("child", "<i4"),
                               ("attempts", "<i4"), ("flags", "<i4"), ("cut", "<i4")])
EVENT_DTYPE = np.dtype([("t", "<i8"), ("v", "<u2"), ("cut", "<u2"), ("nb", "<u2"), ("target", "u1"),
                        ("reserved", "u1")])


def _p(arr, ct):
    return arr.ctypes.data_as(_P(ct)) if arr is not None else _P(ct)()


def _set_fields(struct, **fields):
    for name, val in fields.items():
        setattr(struct, name, val)


def pin_host(arr: np.ndarray) -> np.ndarray:
    """Page-lock a numpy buffer for the device-to-host copies of the readers
    (``fc_host_register``); :func:`unpin_host` before it is freed."""
    check(_lib.load().fc_host_register(ctypes.c_void_p(arr.ctypes.data), int(arr.nbytes)), "fc_host_register")
    return arr


def unpin_host(arr: np.ndarray) -> None:
    check(_lib.load().fc_host_unregister(ctypes.c_void_p(arr.ctypes.data)), "fc_host_unregister")


class FlipGraph:
    """Native graph handle (``fc_graph_create``)."""

    def __init__(self, spec: GraphSpec, use_positions: bool = True, exact: bool = True):
        self.spec = spec
        L = _lib.load()
        self._row = np.ascontiguousarray(spec.row_ptr, dtype=np.int32)
        self._col = np.ascontiguousarray(spec.col_idx, dtype=np.int32)
        self._pop = np.ascontiguousarray(spec.pop, dtype=np.int32)
        pos = None
        if use_positions and spec.pos is not None:
            pos = np.ascontiguousarray(spec.pos, dtype=np.float64).reshape(-1)
        h = ctypes.c_void_p()
        flags = 0 if exact else _lib.FC_GRAPH_NO_EXACT
        check(L.fc_graph_create(spec.n, _p(self._row, ctypes.c_int32), _p(self._col, ctypes.c_int32),
                                _p(self._pop, ctypes.c_int32), _p(pos, ctypes.c_double), flags,
                                ctypes.byref(h)), "fc_graph_create")
        self.handle = h
        info = _lib.GraphInfo()
        check(L.fc_graph_get_info(h, ctypes.byref(info)), "fc_graph_get_info")
        self.info = {f: getattr(info, f) for f, _ in _lib.GraphInfo._fields_}

    @property
    def n(self) -> int:
        return self.info["n_nodes"]

    @property
    def n_edges(self) -> int:
        return self.info["n_edges"]

    def edges(self) -> np.ndarray:
        eu = np.zeros(self.n_edges, dtype=np.int32)
        ev = np.zeros(self.n_edges, dtype=np.int32)
        check(_lib.load().fc_graph_edges(self.handle, _p(eu, ctypes.c_int32), _p(ev, ctypes.c_int32)))
        return np.stack([eu, ev], axis=1)

    def rings(self):
        R = self.info["ring_max"]
        ring = np.zeros(self.n * R, dtype=np.int32)
        meta = np.zeros(self.n, dtype=np.uint64)
        check(_lib.load().fc_graph_rings(self.handle, _p(ring, ctypes.c_int32), _p(meta, ctypes.c_uint64)))
        return ring.reshape(self.n, R), meta

    def close(self):
        if getattr(self, "handle", None):
            _lib.load().fc_graph_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass


@dataclass
class RunConfig:
    k: int = 2
    base: float = 1.0
    pop_lo: int = 0
    pop_hi: int = 2 ** 31 - 1
    seed: int = 0
    chain_id_offset: int = 0
    diag_mask: int = _lib.FC_DIAG_WAIT
    flags: int = 0
    device: int = 0
    trace_chains: int = 0
    trace_cap: int = 0
    labels: Sequence[int] = (-1, 1)
    proposal: int = _lib.FC_PROPOSE_BI_SIGN
    wmax: int = 0
    hit_lo: int = 1          # hitting-time window on |cut| (hit_lo > hit_hi: off)
    hit_hi: int = 0
    event_cap: int = 0       # FC_DIAG_SERIES events kept per chain per window
    # accept / constraint variants (k = 2; defaults: Validator([contiguous, popbound]) + cut_accept)
    accept: int = _lib.FC_ACCEPT_CUT
    con_valid: int = 0       # FC_CON_* of the Validator (0: CONTIG | POP)
    con_accept: int = 0      # FC_CON_* tested by the accept callable
    beta: float = 0.0        # FC_ACCEPT_ANNEAL exponent factor
    frozen: Sequence[int] = ()  # FC_CON_FIXED: endpoints of the pinned edges
    # FC_PROPOSE_RECOM: recom(pop_target, epsilon, node_repeats) (grid_chain_sec11.py:328-335)
    recom_pop_target: float = 0.0
    recom_epsilon: float = 0.05
    recom_node_repeats: int = 1
    recom_max_attempts: int = 0
    # launch tuning (fc_params.tune_*): scheduling only, never the trajectory; 0 = default.
    # Keys: nsub, hit_stop, par_min, wait_queue, chains_per_block, prio_div (3), prio_th (3),
    # search_waves, deal, multi_flip.
    tune: Optional[Dict[str, object]] = None
    # k = 2 node stream (fc_params.stream): "node" draws over all n nodes, "band" over the band
    # S = b_nodes + neighbours; the chain's law is the same, the trajectory not
    stream: str = "node"


TUNE_KEYS = ("nsub", "hit_stop", "par_min", "wait_queue", "chains_per_block", "prio_div", "prio_th",
             "search_waves", "deal", "multi_flip")


def parse_tune(text: str) -> Dict[str, object]:
    """``"nsub=2,hit_stop=24,prio_div=2:5:10"`` -> RunConfig.tune (tools / bench.py --tune)."""
    out: Dict[str, object] = {}
    for item in filter(None, (t.strip() for t in (text or "").split(","))):
        key, _, val = item.partition("=")
        if key not in TUNE_KEYS:
            raise ValueError(f"unknown tuning key {key!r} (known: {', '.join(TUNE_KEYS)})")
        if key in ("prio_div", "prio_th"):
            conv = int if key == "prio_div" else float
            vals = [conv(x) for x in val.split(":")]
            out[key] = tuple(vals) + (vals[-1],) * (3 - len(vals)) if len(vals) < 3 else tuple(vals[:3])
        else:
            out[key] = int(val)
    return out


class FlipRun:
    """``n_chains`` chains on one GPU (``fc_run_create``).  ``init_assign`` is
    ``[n_chains, n]`` (or ``[n]``, broadcast) district ids; ``bases`` optional per chain."""

    def __init__(self, graph: FlipGraph, init_assign: np.ndarray, cfg: RunConfig,
                 bases: Optional[Sequence[float]] = None, n_chains: Optional[int] = None,
                 log1mp: Optional[np.ndarray] = None, pop_bounds: Optional[np.ndarray] = None):
        """``pop_bounds`` (optional): ``[n_chains, 2]`` inclusive population bounds per chain
        (``fc_params.chain_pop_bounds``), so that configurations of different tolerance share a
        run; default ``cfg.pop_lo`` / ``cfg.pop_hi`` for every chain."""
        L = _lib.load()
        self.graph = graph
        self.cfg = cfg
        a = np.asarray(init_assign, dtype=np.int8)
        if a.ndim == 1:
            a = np.broadcast_to(a, (n_chains or 1, a.shape[0]))
        self.n_chains = int(a.shape[0])
        self._init = np.ascontiguousarray(a)
        if self._init.shape[1] != graph.n:
            raise ValueError("init_assign must have one entry per node")
        labels = list(cfg.labels) if len(cfg.labels) == cfg.k else list(range(cfg.k))
        self._labels = np.ascontiguousarray(labels, dtype=np.int32)
        pairs = bool(cfg.flags & _lib.FC_FLAG_NB_PAIRS) and cfg.k > 2
        width = nb_width(graph.spec, cfg.k, True) if pairs else graph.n + 1
        self._log1mp = np.ascontiguousarray(log1mp if log1mp is not None else log1mp_table(graph.n, cfg.k, width),
                                            dtype=np.float64)
        if self._log1mp.size < width:
            raise ValueError(f"log1mp needs {width} entries (|b_nodes| 0 .. {width - 1})")
        self._bases = None if bases is None else np.ascontiguousarray(bases, dtype=np.float64)
        if self._bases is not None and self._bases.shape[0] != self.n_chains:
            raise ValueError("bases must have one entry per chain")
        self._pop_bounds = None
        if pop_bounds is not None:
            self._pop_bounds = np.ascontiguousarray(pop_bounds, dtype=np.int64).reshape(-1)
            if self._pop_bounds.size != 2 * self.n_chains:
                raise ValueError("pop_bounds must be [n_chains, 2]")
        prm = _lib.Params()
        check(L.fc_params_init(ctypes.byref(prm), ctypes.sizeof(_lib.Params)), "fc_params_init")
        _set_fields(prm, k=cfg.k, proposal=int(cfg.proposal), base=float(cfg.base), wmax=int(cfg.wmax),
                    pop_lo=int(cfg.pop_lo), pop_hi=int(cfg.pop_hi), seed=int(cfg.seed),
                    chain_id_offset=int(cfg.chain_id_offset), diag_mask=int(cfg.diag_mask),
                    flags=int(cfg.flags), device=int(cfg.device), trace_chains=int(cfg.trace_chains),
                    trace_cap=int(cfg.trace_cap), labels=_p(self._labels, ctypes.c_int32),
                    log1mp=_p(self._log1mp, ctypes.c_double), hit_lo=int(cfg.hit_lo),
                    hit_hi=int(cfg.hit_hi), event_cap=int(cfg.event_cap), accept=int(cfg.accept),
                    con_valid=int(cfg.con_valid), con_accept=int(cfg.con_accept), beta=float(cfg.beta))
        prm.chain_pop_bounds = _p(self._pop_bounds, ctypes.c_int64)
        if cfg.stream not in ("node", "band"):
            raise ValueError(f"stream must be 'node' or 'band', not {cfg.stream!r}")
        prm.stream = _lib.STREAM_BAND if cfg.stream == "band" else _lib.STREAM_NODE
        self._frozen = np.ascontiguousarray(list(cfg.frozen), dtype=np.int32)
        prm.frozen = _p(self._frozen, ctypes.c_int32)
        prm.n_frozen = int(self._frozen.size)
        prm.recom_pop_target = float(cfg.recom_pop_target)
        prm.recom_epsilon = float(cfg.recom_epsilon)
        prm.recom_node_repeats = int(cfg.recom_node_repeats)
        prm.recom_max_attempts = int(cfg.recom_max_attempts)
        for key, val in (cfg.tune or {}).items():
            if key not in TUNE_KEYS:
                raise ValueError(f"unknown tuning key {key!r}")
            if key in ("prio_div", "prio_th"):
                arr = getattr(prm, "tune_" + key)
                for i, x in enumerate(val):
                    arr[i] = x
            else:
                setattr(prm, "tune_" + key, int(val))
        h = ctypes.c_void_p()
        check(L.fc_run_create(graph.handle, ctypes.byref(prm), self.n_chains, _p(self._init, ctypes.c_int8),
                              _p(self._bases, ctypes.c_double), ctypes.byref(h)), "fc_run_create")
        self.handle = h
        self._tape = None

    # ---- stepping ---------------------------------------------------------------------
    def steps(self, n_steps: int, max_draws: int = 0, stream: Optional[int] = None) -> "FlipRun":
        check(_lib.load().fc_run_steps(self.handle, int(n_steps), int(max_draws),
                                       ctypes.c_void_p(stream) if stream else None), "fc_run_steps")
        return self

    def set_tape(self, tape: Optional[np.ndarray], n_draws: int = 0):
        """Replay: ``tape`` is ``[n_chains, n_draws * 6]`` u32."""
        if tape is None:
            check(_lib.load().fc_run_set_tape(self.handle, _P(ctypes.c_uint32)(), 0))
            self._tape = None
            return
        t = np.ascontiguousarray(tape, dtype=np.uint32).reshape(self.n_chains, -1)
        n_draws = t.shape[1] // 6
        self._tape = t
        check(_lib.load().fc_run_set_tape(self.handle, _p(t, ctypes.c_uint32), n_draws), "fc_run_set_tape")

    def set_initial_wait(self, words: np.ndarray):
        """Replay the initial states' geometric waits: ``words`` is ``[n_chains, 2]`` u32 (the
        53-bit uniform numpy's geometric inverted; ``fc_run_set_initial_wait``)."""
        w = np.ascontiguousarray(words, dtype=np.uint32).reshape(self.n_chains, 2)
        check(_lib.load().fc_run_set_initial_wait(self.handle, _p(w, ctypes.c_uint32)), "fc_run_set_initial_wait")

    def checkpoint(self) -> bytes:
        """The run's resumable state as bytes (``fc_run_checkpoint``)."""
        L = _lib.load()
        n = ctypes.c_int64(0)
        check(L.fc_run_checkpoint(self.handle, None, 0, ctypes.byref(n)), "fc_run_checkpoint")
        buf = ctypes.create_string_buffer(int(n.value))
        check(L.fc_run_checkpoint(self.handle, buf, n.value, ctypes.byref(n)), "fc_run_checkpoint")
        return buf.raw

    def restore(self, blob: bytes):
        """Load a ``checkpoint()`` of a run with the same graph and configuration."""
        buf = ctypes.create_string_buffer(bytes(blob), len(blob))
        check(_lib.load().fc_run_restore(self.handle, buf, len(blob)), "fc_run_restore")

    def sync(self):
        check(_lib.load().fc_run_sync(self.handle))

    def last_ms(self) -> float:
        ms = ctypes.c_float(0)
        check(_lib.load().fc_run_last_ms(self.handle, ctypes.byref(ms)))
        return float(ms.value)

    def timings(self, cap: int = 4096) -> np.ndarray:
        """Device ms of every launch since the previous call (HIP events on the run's stream)."""
        out = np.zeros(cap, dtype=np.float32)
        n = ctypes.c_int32(0)
        check(_lib.load().fc_run_timings(self.handle, _p(out, ctypes.c_float), cap, ctypes.byref(n)))
        return out[:min(n.value, cap)].astype(np.float64)

    # ---- readouts ---------------------------------------------------------------------
    def stats(self) -> Dict[str, np.ndarray]:
        arr = (_lib.ChainStats * self.n_chains)()
        check(_lib.load().fc_run_read_stats(self.handle, arr), "fc_run_read_stats")
        raw = np.ctypeslib.as_array(arr)
        return {f: np.array(raw[f]) for f in STAT_FIELDS}

    def state(self) -> np.ndarray:
        out = np.zeros((self.n_chains, self.graph.n), dtype=np.int8)
        check(_lib.load().fc_run_read_state(self.handle, _p(out, ctypes.c_int8)), "fc_run_read_state")
        return out

    def pops(self) -> np.ndarray:
        out = np.zeros((self.n_chains, self.cfg.k), dtype=np.int64)
        check(_lib.load().fc_run_read_pops(self.handle, _p(out, ctypes.c_int64)), "fc_run_read_pops")
        return out

    def trace(self, chain: int = 0) -> np.ndarray:
        cap = self.cfg.trace_cap
        out = np.zeros(cap, dtype=RECORD_DTYPE)
        n = ctypes.c_int64(0)
        check(_lib.load().fc_run_read_trace(self.handle, chain, ctypes.cast(out.ctypes.data, _P(_lib.Record)),
                                            cap, ctypes.byref(n)), "fc_run_read_trace")
        if n.value > cap:
            raise OverflowError(f"trace capacity {cap} exceeded ({n.value} records)")
        return out[:n.value]

    def recom_trace(self, chain: int = 0) -> np.ndarray:
        """Per-proposal records of a traced ReCom chain (``fc_recom_record``)."""
        cap = self.cfg.trace_cap
        out = np.zeros(cap, dtype=RECOM_RECORD_DTYPE)
        n = ctypes.c_int64(0)
        check(_lib.load().fc_run_read_recom_trace(self.handle, chain,
                                                  ctypes.cast(out.ctypes.data, _P(_lib.RecomRecord)), cap,
                                                  ctypes.byref(n)), "fc_run_read_recom_trace")
        if n.value > cap:
            raise OverflowError(f"trace capacity {cap} exceeded ({n.value} records)")
        return out[:n.value]

    def trace_reset(self):
        check(_lib.load().fc_run_trace_reset(self.handle), "fc_run_trace_reset")

    def hist(self):
        E, n = self.graph.n_edges, self.graph.n
        ch = np.zeros((self.n_chains, E + 1), dtype=np.int64)
        nh = np.zeros((self.n_chains, self.nb_width()), dtype=np.int64)
        check(_lib.load().fc_run_read_hist(self.handle, _p(ch, ctypes.c_int64), _p(nh, ctypes.c_int64)))
        return ch, nh

    def cut_times(self) -> np.ndarray:
        out = np.zeros((self.n_chains, self.graph.n_edges), dtype=np.int64)
        check(_lib.load().fc_run_read_edges(self.handle, _p(out, ctypes.c_int64)))
        return out

    def flips(self):
        n = self.graph.n
        nf = np.zeros((self.n_chains, n), dtype=np.int64)
        ps = np.zeros((self.n_chains, n), dtype=np.int64)
        lf = np.zeros((self.n_chains, n), dtype=np.int64)
        check(_lib.load().fc_run_read_flips(self.handle, _p(nf, ctypes.c_int64), _p(ps, ctypes.c_int64),
                                            _p(lf, ctypes.c_int64)))
        return nf, ps, lf

    def flips_exact(self):
        """FC_DIAG_FLIPS_EXACT: (flip_count, occupancy, last_accept) [chains, n] -- the corrected
        companions of :meth:`flips` (include/flipchain.h)."""
        n = self.graph.n
        fc_ = np.zeros((self.n_chains, n), dtype=np.int64)
        occ = np.zeros((self.n_chains, n), dtype=np.int64)
        la = np.zeros((self.n_chains, n), dtype=np.int64)
        check(_lib.load().fc_run_read_flips_exact(self.handle, _p(fc_, ctypes.c_int64), _p(occ, ctypes.c_int64),
                                                  _p(la, ctypes.c_int64)))
        return fc_, occ, la

    def wait_expected(self) -> np.ndarray:
        """Rao-Blackwellised wait.txt companion (App. A.6 quirk 3): per chain, the sum over yields
        of E[geom_wait | |B|] = (N^k - 1)/|B| - 1 (:147-148), from the |B| histogram."""
        out = np.zeros(self.n_chains, dtype=np.float64)
        check(_lib.load().fc_run_read_wait_expected(self.handle, _p(out, ctypes.c_double)))
        return out

    # ---- series diagnostics (FC_DIAG_SERIES) ------------------------------------------
    def events(self, chain: int = 0) -> np.ndarray:
        """Accepted flips of ``chain`` in the current series window (``fc_event``)."""
        cap = int(self.cfg.event_cap)
        out = np.zeros(cap, dtype=EVENT_DTYPE)
        n = ctypes.c_int64(0)
        check(_lib.load().fc_run_read_events(self.handle, chain, ctypes.cast(out.ctypes.data, _P(_lib.Event)),
                                             cap, ctypes.byref(n)), "fc_run_read_events")
        if n.value > cap:
            raise OverflowError(f"event capacity {cap} exceeded ({n.value} events)")
        return out[:n.value]

    def series_reset(self):
        check(_lib.load().fc_run_series_reset(self.handle), "fc_run_series_reset")

    def cut_series(self, chain: int = 0) -> np.ndarray:
        """|cut| at every yield of the window -- the reference's ``rce`` list
        (``grid_chain_sec11.py:367``) -- expanded on the host from the event log."""
        st = self.stats()
        t0, x0, T = int(st["series_t0"][chain]), int(st["series_cut0"][chain]), int(st["steps"][chain])
        ev = self.events(chain)
        bounds = np.concatenate([[t0], ev["t"], [T + 1]]).astype(np.int64)
        vals = np.concatenate([[x0], ev["cut"].astype(np.int64)])
        return np.repeat(vals, np.diff(bounds))

    def yield_values(self, field: str = "cut", chain: int = 0) -> np.ndarray:
        """Per-yield ``|cut|`` ("cut") or ``|B|`` ("nb") over the window: the reference's
        ``rce`` / ``rbn`` lists (``grid_chain_sec11.py:367,369``)."""
        st = self.stats()
        x0 = int(st["series_cut0" if field == "cut" else "series_nb0"][chain])
        ev = self.events(chain)
        return self.yield_series(np.concatenate([[x0], ev[field].astype(np.int64)]), chain)

    def autocorr(self, lags: Sequence[int]):
        """Device autocorrelation of the |cut| series over the window: ``(lag_sums, acf)``,
        each ``[n_chains, len(lags)]`` (``fc_run_autocorr``)."""
        lg = np.ascontiguousarray(lags, dtype=np.int32)
        sums = np.zeros((self.n_chains, lg.size), dtype=np.int64)
        acf = np.zeros((self.n_chains, lg.size), dtype=np.float64)
        check(_lib.load().fc_run_autocorr(self.handle, _p(lg, ctypes.c_int32), int(lg.size),
                                          _p(sums, ctypes.c_int64), _p(acf, ctypes.c_double)), "fc_run_autocorr")
        return sums, acf

    def autocorr_pairs(self, lags: Sequence[int]) -> np.ndarray:
        """``[n_chains, len(lags)]``: the (t, t + lag) pairs each lag's sum runs over in the
        current window, max(0, yields - lag) -- a lag at or beyond the window has none."""
        st = self.stats()
        n = (st["steps"] - st["series_t0"] + 1).astype(np.int64)
        return np.maximum(0, n[:, None] - np.asarray(lags, dtype=np.int64)[None, :])

    def frame_series(self, frame, chains: Optional[Sequence[int]] = None,
                     out: Optional[Dict[str, np.ndarray]] = None) -> Dict[str, np.ndarray]:
        """Slope / angle of the frame cut edges after every accepted flip of the window, on
        the device (``fc_run_frame_series``; ``grid_chain_sec11.py:55-78,371-394``).

        ``frame`` is a :class:`~flipcomplexityempirical_amd.graphs.SlopeFrame`.  Returns
        ``slope``, ``angle``, ``n_cut`` as ``[len(chains), max_events + 1]`` (entry 0: window
        start) and ``len`` per chain; use :meth:`yield_series` for the per-yield lists.
        ``out`` (optional): C-contiguous host buffers ``slope`` / ``angle`` (float64) and
        ``n_cut`` (int32) to fill instead of new arrays (a caller that reads many chunks keeps its
        pages mapped); the result then holds views of their leading ``nc * cap`` entries.  A
        buffer of another dtype or layout raises ``ValueError`` (the native call writes through
        raw pointers); buffers too small for this call's ``nc * cap`` entries are not used (fresh
        arrays are returned).  Entries past a chain's ``len`` are padding with undefined values."""
        ch = np.arange(self.n_chains) if chains is None else np.asarray(chains, dtype=np.int64)
        if ch.size == 0:
            raise ValueError("frame_series: no chains")
        c0, nc = int(ch.min()), int(ch.max() - ch.min() + 1)
        st = self.stats()
        cap = int(st["events"][c0:c0 + nc].max()) + 1
        # every entry is copied from the device (entries past a chain's ``len`` are padding)
        if out is not None:
            for key, dt in (("slope", np.float64), ("angle", np.float64), ("n_cut", np.int32)):
                buf = out.get(key)
                if not isinstance(buf, np.ndarray) or buf.dtype != dt or not buf.flags.c_contiguous \
                        or not buf.flags.writeable:
                    raise ValueError(f"frame_series: out[{key!r}] must be a writeable C-contiguous {np.dtype(dt)} array")
        if out is not None and min(out[key].size for key in ("slope", "angle", "n_cut")) >= nc * cap:
            # the buffers' leading nc * cap entries, viewed as [nc, cap]
            slope = out["slope"].reshape(-1)[:nc * cap].reshape(nc, cap)
            angle = out["angle"].reshape(-1)[:nc * cap].reshape(nc, cap)
            ncut = out["n_cut"].reshape(-1)[:nc * cap].reshape(nc, cap)
        else:
            slope = np.empty((nc, cap), dtype=np.float64)
            angle = np.empty((nc, cap), dtype=np.float64)
            ncut = np.empty((nc, cap), dtype=np.int32)
        ln = np.zeros(nc, dtype=np.int64)
        eu = np.ascontiguousarray(frame.eu, dtype=np.int32)
        ev = np.ascontiguousarray(frame.ev, dtype=np.int32)
        mid = np.ascontiguousarray(frame.mid, dtype=np.float64)
        check(_lib.load().fc_run_frame_series(self.handle, c0, nc, int(eu.size), _p(eu, ctypes.c_int32),
                                              _p(ev, ctypes.c_int32), _p(mid, ctypes.c_double),
                                              float(frame.center[0]), float(frame.center[1]), cap,
                                              _p(slope, ctypes.c_double), _p(angle, ctypes.c_double),
                                              _p(ncut, ctypes.c_int32), _p(ln, ctypes.c_int64)),
              "fc_run_frame_series")
        sel = ch - c0
        if sel.size == nc and np.array_equal(sel, np.arange(nc)):  # a contiguous range: no copies
            return {"slope": slope, "angle": angle, "n_cut": ncut, "len": ln}
        return {"slope": slope[sel], "angle": angle[sel], "n_cut": ncut[sel], "len": ln[sel]}

    def frame_series_changes(self, frame, c0: int = 0, nc: Optional[int] = None,
                             out: Optional[Dict[str, np.ndarray]] = None, query: bool = False) -> Dict[str, np.ndarray]:
        """Change points of the slope / angle series of chains ``c0 .. c0 + nc - 1``
        (``fc_run_frame_series_changes``): ``offsets`` [nc + 1] and flat ``t`` (int64), ``slope``,
        ``angle`` (float64); chain ``c0 + i`` owns entries ``offsets[i]:offsets[i + 1]``, each
        value holding from its ``t`` to the next entry's -- what the reference's slope / angle
        plots draw (``grid_chain_sec11.py:476-484``); :meth:`changes_to_yields` expands one chain
        to its per-yield lists (``:382,394``).  ``out`` (optional): C-contiguous int64 / float64 /
        float64 buffers ``t`` / ``slope`` / ``angle`` to fill (e.g. pinned with
        :func:`pin_host`); used when large enough, the result then holds views of them.
        ``query``: only the offsets (sizing buffers)."""
        nc = self.n_chains - c0 if nc is None else int(nc)
        L = _lib.load()
        eu = np.ascontiguousarray(frame.eu, dtype=np.int32)
        ev = np.ascontiguousarray(frame.ev, dtype=np.int32)
        mid = np.ascontiguousarray(frame.mid, dtype=np.float64)
        off = np.zeros(nc + 1, dtype=np.int64)
        args = (self.handle, int(c0), nc, int(eu.size), _p(eu, ctypes.c_int32), _p(ev, ctypes.c_int32),
                _p(mid, ctypes.c_double), float(frame.center[0]), float(frame.center[1]))
        if out is not None and not query:
            for key, dt in (("t", np.int64), ("slope", np.float64), ("angle", np.float64)):
                b = out.get(key)
                if not isinstance(b, np.ndarray) or b.dtype != dt or not b.flags.c_contiguous or not b.flags.writeable:
                    raise ValueError(f"frame_series_changes: out[{key!r}] must be a writeable C-contiguous "
                                     f"{np.dtype(dt)} array")
            # one call: count, offsets, write and copy into the caller's buffers when they hold
            # every change point (the offsets come back either way)
            cap = min(out[key].size for key in ("t", "slope", "angle"))
            flat = {key: out[key].reshape(-1) for key in ("t", "slope", "angle")}
            rc = L.fc_run_frame_series_changes(*args, cap, _p(off, ctypes.c_int64), _p(flat["t"], ctypes.c_int64),
                                               _p(flat["slope"], ctypes.c_double), _p(flat["angle"], ctypes.c_double))
            total = int(off[-1])
            if rc == 0:
                return {"offsets": off, **{key: b[:total] for key, b in flat.items()}}
            if total <= cap:
                check(rc, "fc_run_frame_series_changes")
        else:
            check(L.fc_run_frame_series_changes(*args, 0, _p(off, ctypes.c_int64), _P(ctypes.c_int64)(),
                                                _P(ctypes.c_double)(), _P(ctypes.c_double)()),
                  "fc_run_frame_series_changes")
            total = int(off[-1])
            if query:
                return {"offsets": off}
        bufs = {"t": np.empty(total, dtype=np.int64), "slope": np.empty(total), "angle": np.empty(total)}
        check(L.fc_run_frame_series_changes(*args, total, _p(off, ctypes.c_int64), _p(bufs["t"], ctypes.c_int64),
                                            _p(bufs["slope"], ctypes.c_double), _p(bufs["angle"], ctypes.c_double)),
              "fc_run_frame_series_changes")
        return {"offsets": off, **bufs}

    def changes_to_yields(self, ch: Dict[str, np.ndarray], i: int, chain: int, key: str = "slope") -> np.ndarray:
        """Per-yield list (the reference's ``slopes`` / ``angles``, :382,394) of ``chain`` from
        entry ``i`` of a :meth:`frame_series_changes` result."""
        lo, hi = int(ch["offsets"][i]), int(ch["offsets"][i + 1])
        T = int(self.stats()["steps"][chain])
        bounds = np.concatenate([ch["t"][lo:hi], [T + 1]]).astype(np.int64)
        return np.repeat(ch[key][lo:hi], np.diff(bounds))

    def yield_series(self, values: np.ndarray, chain: int = 0) -> np.ndarray:
        """Expand a per-event series (entry 0 = window start, as ``frame_series`` returns it)
        to one value per yield of the window, as the reference's ``slopes`` / ``angles``
        lists hold them (``grid_chain_sec11.py:382,394``)."""
        st = self.stats()
        t0, T = int(st["series_t0"][chain]), int(st["steps"][chain])
        ev = self.events(chain)
        bounds = np.concatenate([[t0], ev["t"], [T + 1]]).astype(np.int64)
        return np.repeat(np.asarray(values)[:ev.size + 1], np.diff(bounds))

    def diag_paths(self) -> Dict[str, int]:
        """The paths the memory-dependent diagnostics took (``fc_run_diag_paths``): tally-log
        entries per chain granted / asked for, and whether the last change-point call was staged."""
        cap, want, staged = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
        check(_lib.load().fc_run_diag_paths(self.handle, ctypes.byref(cap), ctypes.byref(want), ctypes.byref(staged)),
              "fc_run_diag_paths")
        return {"tally_log_cap": int(cap.value), "tally_log_wanted": int(want.value),
                "series_staged": int(staged.value)}

    def nb_width(self) -> int:
        """Entries of a chain's |B| histogram row (``fc_run_nb_width``): n + 1, or the largest
        pair count + 1 with ``FC_FLAG_NB_PAIRS``."""
        return int(_lib.load().fc_run_nb_width(self.handle))

    def chain_lds_bytes(self) -> int:
        """LDS bytes of one chain's device state (``fc_run_chain_lds_bytes``)."""
        return int(_lib.load().fc_run_chain_lds_bytes(self.handle))

    def kernel_name(self) -> str:
        """The flip-kernel instance the last ``steps`` call launched (rocprofv3 spelling)."""
        buf = ctypes.create_string_buffer(128)
        check(_lib.load().fc_run_kernel_name(self.handle, buf, 128), "fc_run_kernel_name")
        return buf.value.decode()

    def close(self):
        if getattr(self, "handle", None):
            _lib.load().fc_run_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
