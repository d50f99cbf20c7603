"""C2 throughput probe: python tools/probe_c2.py [chains] [steps/launch] [base_index|-1] [iters]"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from flipcomplexityempirical_amd import graphs as G, _lib
_lib.load(allow_variant=True)  # A/B and profiling tool: FC_LIB_PATH / FC_LIB_VARIANT libraries allowed
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig, parse_tune
spec = G.sec11_graph(); fg = FlipGraph(spec)
C = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
B = int(sys.argv[3]) if len(sys.argv) > 3 else -1
IT = int(sys.argv[4]) if len(sys.argv) > 4 else 6
plans = [spec.assignment_array(G.sec11_plan(al, spec.nodes), [-1, 1]) for al in range(3)]
inits = np.stack([plans[(c // 10) % 3] for c in range(C)])
bases = np.asarray([G.SEC11_BASES[c % 10 if B < 0 else B] for c in range(C)])
(_, _), (lo, hi) = G.population_bounds(1596, 2, 0.1)
# FC_PROBE_DIAG=<mask> overrides the diagnostics mask (0: no geometric waits)
cfg = RunConfig(seed=0x5EED0002, pop_lo=lo, pop_hi=hi, tune=parse_tune(os.environ.get('FC_TUNE', '')),
                stream=os.environ.get('FC_STREAM', 'node'))
if 'FC_PROBE_DIAG' in os.environ: cfg.diag_mask = int(os.environ['FC_PROBE_DIAG'])
if 'FC_PROBE_EVCAP' in os.environ: cfg.event_cap = int(os.environ['FC_PROBE_EVCAP'])  # FC_DIAG_SERIES event log
run = FlipRun(fg, inits, cfg, bases=bases)
for it in range(IT):
    s0 = run.stats()
    t = time.time(); run.steps(S); run.sync(); dt = time.time() - t
    s1 = run.stats()
    props = (s1['proposals'] - s0['proposals']).sum()
    if it >= IT - 2:
        print(f"base_idx {B} iter {it}: kernel {run.last_ms():8.2f} ms, proposals/s {props/dt:.3e}, steps/s {C*S/dt:.3e}, acc/prop {(s1['accepted']-s0['accepted']).sum()/props:.3f}, draws/prop {(s1['draws']-s0['draws']).sum()/props:.2f}", flush=True)
