"""Where the full-diagnostics leg's per-launch frame-series time goes (bench.py's loop, C2 full
diagnostics + event log, 4096 chains x 100,000 steps): python tools/archive/probe_series.py [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from flipcomplexityempirical_amd import graphs as G, _lib
_lib.load(allow_variant=True)  # profiling tool: FC_LIB_PATH libraries allowed
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig, pin_host, unpin_host

IT = int(sys.argv[1]) if len(sys.argv) > 1 else 4
C, S = 4096, 100000
spec = G.sec11_graph()
fg = FlipGraph(spec)
plans = [spec.assignment_array(G.sec11_plan(al, spec.nodes), [-1, 1]) for al in range(3)]
inits = np.stack([plans[(c // 10) % 3] for c in range(C)])
bases = np.asarray([G.SEC11_BASES[c % 10] for c in range(C)])
(_, _), (lo, hi) = G.population_bounds(1596, 2, 0.1)
full = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS | _lib.FC_DIAG_SERIES
rf = FlipRun(fg, inits, RunConfig(seed=0x5EED0002, pop_lo=lo, pop_hi=hi, diag_mask=full, event_cap=S + 1), bases=bases)
frame = G.slope_frame(spec, "sec11")
rf.steps(S)
n_cp = int(rf.frame_series_changes(frame, query=True)["offsets"][-1])
n_cp = n_cp + n_cp // 2 + 4 * C
buf = {"t": np.empty(n_cp, dtype=np.int64), "slope": np.empty(n_cp), "angle": np.empty(n_cp)}
for b in buf.values():
    pin_host(b)
rf.series_reset()
rows = []
for it in range(IT):
    t0 = time.perf_counter()
    rf.steps(S)
    rf.sync()
    t1 = time.perf_counter()
    ch = rf.frame_series_changes(frame, out=buf)
    t2 = time.perf_counter()
    ev = int(rf.stats()["events"].sum())
    t3 = time.perf_counter()
    nn = int(np.isnan(ch["angle"]).sum())
    t4 = time.perf_counter()
    rf.series_reset()
    t5 = time.perf_counter()
    rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, int(ch["offsets"][-1]), ev, nn))
    print(f"it {it}: launch+sync {1e3*(t1-t0):7.2f} ms  changes {1e3*(t2-t1):6.2f}  stats {1e3*(t3-t2):6.2f}  "
          f"isnan {1e3*(t4-t3):6.2f}  reset {1e3*(t5-t4):6.2f}  change points {rows[-1][5]}  events {ev}  nan {nn}",
          flush=True)
for b in buf.values():
    unpin_host(b)
