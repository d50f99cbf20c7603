"""ReCom side measurement: python tools/recom_bench.py [chains] [steps/launch] [launches]

sec11 40x40, k=2, the reference's tree_proposal parameters (grid_chain_sec11.py:328-335:
pop_target = ideal, epsilon 0.05, node_repeats 1), Validator = population bound 0.1,
always_accept.  Prints one JSON line: ReCom steps/s on one GPU (HIP-event kernel time),
spanning trees per step, and the single-core rate of the C oracle (oracle/recomref.c) on
the same chains beside it."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

C = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 20
IT = int(sys.argv[3]) if len(sys.argv) > 3 else 3
spec = G.sec11_graph()
plans = [spec.assignment_array(G.sec11_plan(al, spec.nodes), [-1, 1]) for al in range(3)]
inits = np.stack([plans[c % 3] for c in range(C)])
_, (lo, hi) = G.population_bounds(spec.n, 2, 0.1)
cfg = RunConfig(proposal=_lib.FC_PROPOSE_RECOM, seed=0x5EED0010, pop_lo=lo, pop_hi=hi, base=1.0,
                recom_pop_target=spec.n / 2, recom_epsilon=0.05, recom_node_repeats=1, diag_mask=0)
run = FlipRun(FlipGraph(spec), inits, cfg)
run.steps(S)  # warmup
run.sync()
run.timings()
s0 = run.stats()
t0 = time.perf_counter()
for _ in range(IT):
    run.steps(S)
run.sync()
dt = time.perf_counter() - t0
ms = run.timings()
s1 = run.stats()
steps = float((s1["steps"] - s0["steps"]).sum())
trees = float((s1["bfs_levels"] - s0["bfs_levels"]).sum())
props = float((s1["proposals"] - s0["proposals"]).sum())
out = {"metric": "recom steps/sec, sec11 40x40 k=2 (tree_proposal of grid_chain_sec11.py:328-335)",
       "value": steps / dt, "unit": "steps/s", "n_gpus": 1, "chains": C, "steps_per_launch": S, "launches": IT,
       "kernel": run.kernel_name(), "kernel_ms": float(ms.mean()), "steps_per_s_kernel": steps / (ms.sum() * 1e-3),
       "trees_per_step": trees / steps, "proposals_per_step": props / steps}
from oracle.flipref import recom_run
t0, n, c = time.perf_counter(), 0, 0
while time.perf_counter() - t0 < 5.0:
    r = recom_run(spec, plans[c % 3], k=2, pop_target=spec.n / 2, epsilon=0.05, pop_lo=lo, pop_hi=hi,
                  seed=0x5EED0010, chain_id=c, n_steps=50)
    n += r["stats"]["steps"]
    c += 1
out["cpu_baseline"] = {"value": n / (time.perf_counter() - t0), "unit": "steps/s", "cores": 1, "kind": "port",
                       "sample": f"oracle/recomref.c, {c} chains x 50 steps from the start plans"}
print(json.dumps(out), flush=True)
