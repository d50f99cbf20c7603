"""ctypes binding of ``libflipchain.so`` (the C-ABI declared in ``include/flipchain.h``).

The library is required: there is no CPU fallback.  Importing this module builds the
in-tree library if it is missing and the toolchain is present, and raises otherwise.
"""
from __future__ import annotations

import ctypes
import os

from . import build as _build

_P = ctypes.POINTER

STREAM_NODE, STREAM_BAND = 0, 1  # include/flipchain.h FC_STREAM_*
FC_ABI_VERSION = 5  # include/flipchain.h: fc_params layout version

FC_OK = 0
FC_ERR_ARG = -1
FC_ERR_INVALID_STATE = -2
FC_ERR_HIP = -3
FC_ERR_UNSUPPORTED = -4
FC_ERR_NOMEM = -5

FC_GRAPH_NO_EXACT = 0x1
FC_PROPOSE_BI_SIGN, FC_PROPOSE_PAIR, FC_PROPOSE_RECOM = 0, 1, 2
FC_DIAG_WAIT, FC_DIAG_HIST, FC_DIAG_EDGES, FC_DIAG_FLIPS, FC_DIAG_SERIES = 0x1, 0x2, 0x4, 0x8, 0x10
FC_DIAG_FLIPS_EXACT = 0x20
FC_FLAG_FORCE_BFS = 0x1
FC_FLAG_SERIES_TWO_PASS = 0x2  # fc_run_frame_series_changes' two-pass form (cross-check)
FC_FLAG_TALLY_LOG_SMALL = 0x4  # a 64-entry tally log: the overflow path's atomics (cross-check)
FC_FLAG_NB_PAIRS = 0x8  # k > 2: |b_nodes| counts the pair updater's (node, district) pairs (:151-153)
FC_ACCEPT_CUT, FC_ACCEPT_UNIFORM, FC_ACCEPT_ANNEAL = 0, 1, 2
FC_CON_CONTIG, FC_CON_POP, FC_CON_BOUNDARY, FC_CON_FIXED, FC_CON_EMPTY = 0x1, 0x2, 0x4, 0x8, 0x100

EXPORTED = [
    "fc_graph_create", "fc_graph_get_info", "fc_graph_edges", "fc_graph_rings", "fc_graph_destroy",
    "fc_params_init", "fc_run_create", "fc_run_steps", "fc_run_set_tape", "fc_run_set_initial_wait", "fc_run_sync", "fc_run_last_ms", "fc_run_timings",
    "fc_run_read_stats", "fc_run_read_state", "fc_run_read_pops", "fc_run_read_trace", "fc_run_read_recom_trace",
    "fc_run_trace_reset", "fc_run_read_hist", "fc_run_checkpoint", "fc_run_restore",
    "fc_run_read_edges", "fc_run_read_flips", "fc_run_read_flips_exact", "fc_run_read_wait_expected",
    "fc_run_read_events", "fc_run_series_reset", "fc_run_autocorr",
    "fc_run_frame_series", "fc_run_frame_series_changes", "fc_host_register", "fc_host_unregister",
    "fc_run_kernel_name", "fc_run_n_chains", "fc_run_chain_lds_bytes", "fc_run_nb_width", "fc_run_diag_paths",
    "fc_run_destroy",
    "fc_device_count", "fc_device_pci_id", "fc_last_error", "fc_build_flags", "fc_build_id",
]

FC_BUILD_PHASE_PROF, FC_BUILD_PHASE_SYNC, FC_BUILD_VARIANT = 0x1, 0x2, 0x4  # include/flipchain.h
# environment variables that select a non-product library (build.py / load below)
VARIANT_ENV = ("FC_LIB_PATH", "FC_LIB_VARIANT", "FC_HIPCC_FLAGS", "FC_LIB_OUT")


class GraphInfo(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32), ("n_edges", ctypes.c_int32), ("ring_max", ctypes.c_int32),
                ("max_degree", ctypes.c_int32), ("n_exact", ctypes.c_int32), ("n_gamma", ctypes.c_int32),
                ("planar", ctypes.c_int32), ("outer_simple", ctypes.c_int32)]


class Params(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("abi_version", ctypes.c_uint32), ("k", ctypes.c_int32), ("proposal", ctypes.c_int32), ("base", ctypes.c_double),
                ("pop_lo", ctypes.c_int64), ("pop_hi", ctypes.c_int64), ("seed", ctypes.c_uint64),
                ("chain_id_offset", ctypes.c_uint32), ("diag_mask", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("device", ctypes.c_int32), ("trace_chains", ctypes.c_int32),
                ("trace_cap", ctypes.c_int64), ("labels", _P(ctypes.c_int32)), ("log1mp", _P(ctypes.c_double)),
                ("wmax", ctypes.c_int32), ("hit_lo", ctypes.c_int32), ("hit_hi", ctypes.c_int32),
                ("event_cap", ctypes.c_int64), ("accept", ctypes.c_int32), ("con_valid", ctypes.c_uint32),
                ("con_accept", ctypes.c_uint32), ("beta", ctypes.c_double), ("frozen", _P(ctypes.c_int32)),
                ("n_frozen", ctypes.c_int32), ("recom_pop_target", ctypes.c_double),
                ("recom_epsilon", ctypes.c_double), ("recom_node_repeats", ctypes.c_int32),
                ("recom_max_attempts", ctypes.c_int32),
                # launch tuning (scheduling only; 0 = default)
                ("tune_nsub", ctypes.c_int32), ("tune_hit_stop", ctypes.c_int32),
                ("tune_par_min", ctypes.c_int32), ("tune_wait_queue", ctypes.c_int32),
                ("tune_chains_per_block", ctypes.c_int32), ("tune_prio_div", ctypes.c_int32 * 3),
                ("tune_prio_th", ctypes.c_float * 3), ("tune_search_waves", ctypes.c_int32),
                ("tune_deal", ctypes.c_int32),
                # per-chain configuration
                ("chain_pop_bounds", _P(ctypes.c_int64)),
                # k = 2 node stream: FC_STREAM_NODE / FC_STREAM_BAND
                ("stream", ctypes.c_int32), ("tune_multi_flip", ctypes.c_int32)]


class ChainStats(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_int64), ("proposals", ctypes.c_int64), ("draws", ctypes.c_int64),
                ("accepted", ctypes.c_int64), ("inv_contig", ctypes.c_int64), ("inv_pop", ctypes.c_int64),
                ("sum_cut", ctypes.c_int64), ("sum_nb", ctypes.c_int64), ("sum_wait", ctypes.c_int64),
                ("sum_cut2", ctypes.c_int64), ("sum_nb2", ctypes.c_int64), ("wait_cur", ctypes.c_int64),
                ("bfs_calls", ctypes.c_int64), ("bfs_levels", ctypes.c_int64),
                ("cut", ctypes.c_int32), ("nb", ctypes.c_int32), ("last_flip", ctypes.c_int32),
                ("stuck", ctypes.c_int32), ("hit_time", ctypes.c_int64), ("events", ctypes.c_int64),
                ("series_t0", ctypes.c_int64), ("series_cut0", ctypes.c_int32), ("series_nb0", ctypes.c_int32)]


class Event(ctypes.Structure):
    _fields_ = [("t", ctypes.c_int64), ("v", ctypes.c_uint16), ("cut", ctypes.c_uint16), ("nb", ctypes.c_uint16),
                ("target", ctypes.c_uint8), ("reserved", ctypes.c_uint8)]


class Record(ctypes.Structure):
    _fields_ = [("draw", ctypes.c_int64), ("v", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("cut", ctypes.c_int32), ("nb", ctypes.c_int32), ("wait", ctypes.c_int64)]


class RecomRecord(ctypes.Structure):
    _fields_ = [("draw", ctypes.c_int64), ("edge", ctypes.c_int32), ("root", ctypes.c_int32),
                ("child", ctypes.c_int32), ("attempts", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("cut", ctypes.c_int32)]


class FlipChainError(RuntimeError):
    pass


_lib = None
_allow_variant = False


def lib_path() -> str:
    return _build.LIB


def build_flags() -> int:
    """``fc_build_flags()`` of the loaded library (FC_BUILD_*; 0 = the product build)."""
    return int(load().fc_build_flags())


def hip_runtime_path() -> str:
    """The HIP runtime this process mapped (``/proc/self/maps``): /opt/rocm's when the library is
    loaded first, torch's bundled copy when torch initialised its runtime first (same soname, so
    the library binds to it) -- one runtime per process either way."""
    seen = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.strip() else ""
                if "libamdhip64" in p and p not in seen:
                    seen.append(p)
    except OSError:
        pass
    return ";".join(seen)


def build_id() -> str:
    """``fc_build_id()`` of the loaded library: the content hash of the sources it was built from."""
    return load().fc_build_id().decode()


def load(build_if_missing: bool = True, allow_variant: bool = False):
    """Load (building if needed) the native library; raises when it cannot be had.

    A profiling / experiment library -- selected by FC_LIB_PATH, FC_LIB_VARIANT, FC_HIPCC_FLAGS
    or FC_LIB_OUT, or reporting FC_BUILD_* bits from ``fc_build_flags()`` -- is refused unless
    ``allow_variant`` (the A/B and profiling tools pass it; tests, ``bench.py`` and
    ``smoke()`` do not), so a stray environment variable cannot put a non-product library
    under the product's loader.  Once allowed, later calls return the same library."""
    global _lib, _allow_variant
    if allow_variant:
        _allow_variant = True
    if _lib is not None:
        return _lib
    env = [k for k in VARIANT_ENV if os.environ.get(k)]
    if env and not _allow_variant:
        raise ImportError(f"libflipchain: {', '.join(env)} set: a variant library is loaded only with "
                          "_lib.load(allow_variant=True) (A/B and profiling tools)")
    # FC_LIB_PATH: load this prebuilt library as is (A/B timing of two builds on one box)
    path = os.environ.get("FC_LIB_PATH") or _build.LIB
    if build_if_missing and "FC_LIB_PATH" not in os.environ and (not os.path.exists(path) or _build._stale()):
        if os.path.exists(_build.HIPCC):
            _build.build()
    if not os.path.exists(path):
        raise ImportError(f"libflipchain.so not found at {path}: run `python -m flipcomplexityempirical_amd.build` "
                          "(the HIP path is required; there is no CPU fallback)")
    L = ctypes.CDLL(path)
    i32, i64, u32, dbl = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_double
    vp = ctypes.c_void_p
    L.fc_graph_create.argtypes = [i32, _P(i32), _P(i32), _P(i32), _P(dbl), u32, _P(vp)]
    L.fc_graph_get_info.argtypes = [vp, _P(GraphInfo)]
    L.fc_graph_edges.argtypes = [vp, _P(i32), _P(i32)]
    L.fc_graph_rings.argtypes = [vp, _P(i32), _P(ctypes.c_uint64)]
    L.fc_graph_destroy.argtypes = [vp]
    L.fc_graph_destroy.restype = None
    L.fc_params_init.argtypes = [_P(Params), u32]
    L.fc_run_create.argtypes = [vp, _P(Params), i32, _P(ctypes.c_int8), _P(dbl), _P(vp)]
    L.fc_run_steps.argtypes = [vp, i64, i64, vp]
    L.fc_run_set_tape.argtypes = [vp, _P(ctypes.c_uint32), i64]
    L.fc_run_set_initial_wait.argtypes = [vp, _P(ctypes.c_uint32)]
    L.fc_run_sync.argtypes = [vp]
    L.fc_run_last_ms.argtypes = [vp, _P(ctypes.c_float)]
    L.fc_run_timings.argtypes = [vp, _P(ctypes.c_float), i32, _P(i32)]
    L.fc_run_read_stats.argtypes = [vp, _P(ChainStats)]
    L.fc_run_read_state.argtypes = [vp, _P(ctypes.c_int8)]
    L.fc_run_read_pops.argtypes = [vp, _P(i64)]
    L.fc_run_read_trace.argtypes = [vp, i32, _P(Record), i64, _P(i64)]
    L.fc_run_read_recom_trace.argtypes = [vp, i32, _P(RecomRecord), i64, _P(i64)]
    L.fc_run_trace_reset.argtypes = [vp]
    L.fc_run_checkpoint.argtypes = [vp, ctypes.c_void_p, i64, _P(i64)]
    L.fc_run_restore.argtypes = [vp, ctypes.c_void_p, i64]
    L.fc_run_read_hist.argtypes = [vp, _P(i64), _P(i64)]
    L.fc_run_read_edges.argtypes = [vp, _P(i64)]
    L.fc_run_read_flips.argtypes = [vp, _P(i64), _P(i64), _P(i64)]
    L.fc_run_read_flips_exact.argtypes = [vp, _P(i64), _P(i64), _P(i64)]
    L.fc_run_read_wait_expected.argtypes = [vp, _P(dbl)]
    L.fc_run_read_events.argtypes = [vp, i32, _P(Event), i64, _P(i64)]
    L.fc_run_series_reset.argtypes = [vp]
    L.fc_run_autocorr.argtypes = [vp, _P(i32), i32, _P(i64), _P(dbl)]
    L.fc_run_frame_series.argtypes = [vp, i32, i32, i32, _P(i32), _P(i32), _P(dbl), dbl, dbl, i64, _P(dbl),
                                      _P(dbl), _P(i32), _P(i64)]
    L.fc_run_frame_series_changes.argtypes = [vp, i32, i32, i32, _P(i32), _P(i32), _P(dbl), dbl, dbl, i64,
                                              _P(i64), _P(i64), _P(dbl), _P(dbl)]
    L.fc_host_register.argtypes = [vp, i64]
    L.fc_host_unregister.argtypes = [vp]
    L.fc_run_kernel_name.argtypes = [vp, ctypes.c_char_p, i32]
    L.fc_run_n_chains.argtypes = [vp]
    L.fc_run_n_chains.restype = i32
    L.fc_run_chain_lds_bytes.argtypes = [vp]
    L.fc_run_chain_lds_bytes.restype = i32
    L.fc_run_diag_paths.argtypes = [vp, _P(i64), _P(i64), _P(i32)]
    L.fc_run_nb_width.argtypes = [vp]
    L.fc_run_nb_width.restype = i32
    L.fc_device_pci_id.argtypes = [i32, ctypes.c_char_p, i32]
    L.fc_run_destroy.argtypes = [vp]
    L.fc_run_destroy.restype = None
    L.fc_device_count.argtypes = [_P(i32)]
    L.fc_last_error.argtypes = []
    L.fc_last_error.restype = ctypes.c_char_p
    L.fc_build_flags.argtypes = []
    L.fc_build_flags.restype = ctypes.c_uint32
    L.fc_build_id.argtypes = []
    L.fc_build_id.restype = ctypes.c_char_p
    for name in EXPORTED:
        if name not in ("fc_graph_destroy", "fc_run_destroy", "fc_last_error", "fc_run_n_chains",
                        "fc_run_chain_lds_bytes", "fc_run_nb_width", "fc_build_flags", "fc_build_id"):
            getattr(L, name).restype = ctypes.c_int
    bf = int(L.fc_build_flags())
    if bf and not _allow_variant:
        raise ImportError(f"{path}: a variant build (fc_build_flags() = {bf:#x}); loaded only with "
                          "_lib.load(allow_variant=True)")
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc == FC_OK:
        return
    msg = (load().fc_last_error() or b"").decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == FC_ERR_INVALID_STATE:
        raise ValueError(text)
    if rc == FC_ERR_ARG:
        raise ValueError(text)
    if rc == FC_ERR_UNSUPPORTED:
        raise NotImplementedError(text)
    if rc == FC_ERR_NOMEM:
        raise MemoryError(text)
    raise FlipChainError(text)


def device_count() -> int:
    n = ctypes.c_int32(0)
    rc = load().fc_device_count(ctypes.byref(n))
    return int(n.value) if rc == FC_OK else 0
