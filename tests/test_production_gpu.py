"""The kernels the bench times, at production shape (VERDICT r05
item 1).

* C2 (the headline, BASELINE config 2): bench.py's own workload object -- 4096 chains, base
  ``bases[g % 10]``, alignment ``(g // 10) % 3``, pop 0.1, seed 0x5EED0002 -- one 100,000-step
  launch of the lean instance bench.py times, 48 chains sampled over the id range (every (base,
  alignment) configuration of the two short-boundary bases 6.96 / 10 among them) against the C
  oracle: final state and every counter (``grid_chain_sec11.py:340-342,366-411``).
* C3 (BASELINE config 3: sec11 lattice, k = 4 quadrant plan, pair proposals, population
  tolerance 0.05, base mu, 8192 chains per GPU, the multi-flip commit on by default): the lean
  instance the bench times, 8192 chains in one launch, against the C oracle on 64 chains sampled
  over the whole id range (final state, populations, every counter); the same chains split over
  two ``chain_id_offset`` runs (two ranks' shards) are state-identical to the one run; and a
  traced run of the same launch shape compared with the oracle proposal by proposal.
* Long launches with the multi-flip commit on and off (C4 and C5 graphs, base-1 chains among
  them, three 100,000-step launches): byte-identical checkpoints -- assignment, foreign-district
  counts and their histogram, district tables, every per-chain scalar.
"""
import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

pytestmark = pytest.mark.gpu

STAT_KEYS = ["steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb",
             "sum_wait", "sum_cut2", "sum_nb2", "wait_cur", "cut", "nb"]
C3_SEED = 0x5EED0003  # bench.py's C3 seed


def _c3(sec11, chains, *, offset=0, trace=0):
    k = 4
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    _, (lo, hi) = G.population_bounds(sec11.n, k, 0.05)
    cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=C3_SEED, pop_lo=lo, pop_hi=hi,
                    chain_id_offset=offset, trace_chains=trace, trace_cap=200000 if trace else 0)
    run = FlipRun(FlipGraph(sec11), np.broadcast_to(a0, (chains, sec11.n)), cfg,
                  bases=np.full(chains, G.SEC11_MU))
    return run, a0, (lo, hi)


def test_c2_production_shape_against_oracle(gpu, cref):
    """The headline launch exactly as bench.py issues it (its Workload("c2"), its seed, one
    100,000-step launch of 4096 chains), the kernel name asserted, 48 sampled chains against the
    C oracle.  The oracle chains run on a thread pool (ctypes releases the GIL; fr_run keeps no
    global state)."""
    from concurrent.futures import ThreadPoolExecutor
    import bench
    W = bench.Workload("c2")
    assert W.chains == 4096 and W.seed == 0x5EED0002 and W.k == 2 and W.pct == 0.1
    C, steps = W.chains, 100000
    spec = W.spec
    inits = np.stack([W.init_of(g) for g in range(C)])
    bases = np.asarray([W.base_of(g) for g in range(C)])
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), W.k, W.pct)
    cfg = RunConfig(k=2, labels=(-1, 1), proposal=W.proposal, seed=W.seed, pop_lo=lo, pop_hi=hi, stream="node")
    run = FlipRun(FlipGraph(spec), inits, cfg, bases=bases)
    run.steps(steps)
    name = run.kernel_name()
    assert "flip2_kernel<8, 4, false, false, false, false>" in name, name
    st, state = run.stats(), run.state()
    assert (st["steps"] == steps).all() and not st["stuck"].any()
    # 32 chains spread over the ids + one chain of each (base 6.96 / 10) x alignment configuration,
    # placed in the upper half of the id range
    spread = set(np.linspace(0, C - 1, 32).astype(np.int64).tolist())
    slow = {2040 + 30 * j + 10 * al + b for j, (al, b) in enumerate((al, b) for al in range(3) for b in (8, 9))}
    slow |= {C - 1 - ((C - 1 - g) % 30) for g in (8, 9, 18, 19, 28, 29)}   # the same six near the top
    sample = sorted(spread | slow)[:48]
    assert {(W.base_of(g), W.plan_of(g)) for g in sample} >= {(W.bases[b], al) for b in (8, 9) for al in range(3)}
    l1 = G.log1mp_table(spec.n, 2)

    def ref(g):
        return g, cref.run(spec, inits[g], base=bases[g], pop_lo=lo, pop_hi=hi, seed=W.seed, chain_id=g,
                           n_steps=steps, log1mp=l1)

    with ThreadPoolExecutor(max_workers=8) as ex:
        refs = dict(ex.map(ref, sample))
    for g in sample:
        r = refs[g]
        assert np.array_equal(state[g], r["final"]), g
        for key in STAT_KEYS:
            assert int(st[key][g]) == int(r["stats"][key]), (g, key, W.base_of(g))
    run.close()


def test_c3_production_shape_against_oracle(gpu, cref, sec11):
    C, steps = 8192, 400
    run, a0, (lo, hi) = _c3(sec11, C)
    run.steps(steps)
    name = run.kernel_name()
    # lean, multi-flip with the exact marks (a byte per node costs C3 no residency)
    assert name.startswith("fc::flip_kernel<8,") and name.endswith(", 3, false, 2>"), name
    st, state, pops = run.stats(), run.state(), run.pops()
    assert (st["steps"] == steps).all() and not st["stuck"].any()
    sample = np.unique(np.linspace(0, C - 1, 64).astype(np.int64))
    for g in sample:
        ref = cref.run(sec11, a0, base=G.SEC11_MU, pop_lo=lo, pop_hi=hi, seed=C3_SEED, chain_id=int(g),
                       n_steps=steps, k=4, labels=[0, 1, 2, 3], log1mp=G.log1mp_table(sec11.n, 4), proposal=1)
        assert np.array_equal(state[g], ref["final"]), g
        for key in ("steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb",
                    "sum_wait", "cut", "nb"):
            assert int(st[key][g]) == int(ref["stats"][key]), (g, key)
        _, _, p_ref = G.cut_and_boundary(sec11, ref["final"])
        assert np.array_equal(pops[g], p_ref), g
    # two shards (two ranks' chain_id_offset) reproduce the one run chain for chain
    for off, cnt in ((0, C // 2), (C // 2, C // 2)):
        part, _, _ = _c3(sec11, cnt, offset=off)
        part.steps(steps // 2)
        part.steps(steps - steps // 2)
        ps = part.stats()
        assert np.array_equal(part.state(), state[off:off + cnt])
        for key in STAT_KEYS:
            assert np.array_equal(ps[key], st[key][off:off + cnt]), key
        part.close()
    run.close()


def test_c3_production_launch_traced(gpu, cref, sec11):
    """8192 chains per launch (the production grid), the first 64 traced per proposal."""
    C, steps, T = 8192, 300, 64
    run, a0, (lo, hi) = _c3(sec11, C, trace=T)
    run.steps(steps)
    for c in range(T):
        ref = cref.run(sec11, a0, base=G.SEC11_MU, pop_lo=lo, pop_hi=hi, seed=C3_SEED, chain_id=c, n_steps=steps,
                       k=4, labels=[0, 1, 2, 3], log1mp=G.log1mp_table(sec11.n, 4), trace_cap=200000, proposal=1)
        tr, rt = run.trace(c), ref["trace"]
        assert len(tr) == len(rt), c
        for f in ("draw", "v", "flags", "cut", "nb", "wait"):
            assert np.array_equal(tr[f], rt[f]), (c, f)
    run.close()


@pytest.mark.parametrize("case", ["c3", "c4", "c5"])
def test_multi_flip_long_launches_checkpoint_identical(gpu, case):
    """three 100,000-step launches of a few chains (base 1 among them, where most
    passes commit several flips) with the multi-flip commit on and off leave byte-identical
    checkpoints (C3: the exact-mark instance; C4 / C5: the hashed one)."""
    pct = 0.1
    if case == "c3":
        spec, k, pct = G.sec11_graph(), 4, 0.05
        a0 = spec.assignment_array(G.quadrant_plan(spec.nodes), list(range(k)))
    elif case == "c4":
        spec, k = G.triangular_graph(100, 198), 8
        a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    else:
        spec, k = G.delaunay_graph(10000, seed=0), 18
        a0 = spec.assignment_array(G.bisection_plan(spec, k), list(range(k)))
    fg = FlipGraph(spec)
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    inits = np.stack([a0] * 8)
    bases = np.asarray([1.0, 0.5, 2.0, 1.0] * 2)
    blobs, names = [], []
    for mf in (1, -1):
        cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=77, pop_lo=lo, pop_hi=hi,
                        tune={"multi_flip": mf})
        r = FlipRun(fg, inits, cfg, bases=bases)
        for _ in range(3):
            r.steps(100000)
        names.append(r.kernel_name())
        assert (r.stats()["steps"] == 300000).all()
        blobs.append(r.checkpoint())
        r.close()
    # C4 / C5 keep the hashed marks (exact ones would cost them residency), off: MF = 0
    assert names[0].endswith(", 2>" if case == "c3" else ", 1>") and names[1].endswith(", 0>"), names
    assert len(blobs[0]) == len(blobs[1])
    a, b = np.frombuffer(blobs[0], np.uint8), np.frombuffer(blobs[1], np.uint8)
    diff = np.nonzero(a != b)[0]
    assert diff.size == 0, f"checkpoints differ at {diff.size} bytes, first at {diff[:4]}"
