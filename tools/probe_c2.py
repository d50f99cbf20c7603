"""Quick C2 throughput probe (4096 chains, sec11, base sweep)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from flipcomplexityempirical_amd import graphs as G, _lib
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
spec = G.sec11_graph(); fg = FlipGraph(spec)
C = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
plans = [spec.assignment_array(G.sec11_plan(al, spec.nodes), [-1, 1]) for al in range(3)]
inits = np.stack([plans[(c // 10) % 3] for c in range(C)])
bases = np.asarray([G.SEC11_BASES[c % 10] for c in range(C)])
(_, _), (lo, hi) = G.population_bounds(1596, 2, 0.1)
run = FlipRun(fg, inits, RunConfig(seed=0x5EED0002, pop_lo=lo, pop_hi=hi), bases=bases)
for it in range(6):
    s0 = run.stats()
    t = time.time(); run.steps(S); run.sync(); dt = time.time() - t
    s1 = run.stats()
    props = (s1['proposals'] - s0['proposals']).sum()
    print(f"iter {it}: {dt*1e3:8.1f} ms wall, kernel {run.last_ms():8.1f} ms, proposals {props:.3e} -> {props/dt:.3e}/s, steps/s {C*S/dt:.3e}", flush=True)
st = run.stats()
for b in range(10):
    m = np.arange(C) % 10 == b
    print(f"base {G.SEC11_BASES[b]:6.3f}: prop/step {st['proposals'][m].sum()/st['steps'][m].sum():5.2f} draws/prop {st['draws'][m].sum()/st['proposals'][m].sum():5.2f} acc/step {st['accepted'][m].sum()/st['steps'][m].sum():5.3f} cut {st['cut'][m].mean():7.1f} bfs {st['bfs_calls'][m].sum()}")
