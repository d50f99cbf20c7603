"""GPU parity for PAIR proposals (k >= 2; slow_reversible_propose, grid_chain_sec11.py:117-130,
b_nodes pairs :151-153): the general-k kernel against the C oracle, bit-exact per proposal.

Covers BASELINE configs C3 (sec11 lattice, k=4 quadrant plan, pop tolerance 0.05, base mu)
and C4 (triangular lattice, k=8 vertical strips) at test sizes, plus PAIR == BI_SIGN at k=2.
"""
import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig

pytestmark = pytest.mark.gpu

STAT_KEYS = ["steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb",
             "sum_wait", "cut", "nb"]
ALL_DIAG = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS


def _run_pair(spec, inits, bases, k, *, steps, pct, seed=21, flags=0, chunks=1, exact=True, proposal=None,
              use_positions=True, tune=None):
    fg = FlipGraph(spec, exact=exact, use_positions=use_positions)
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR if proposal is None else proposal,
                    seed=seed, pop_lo=lo, pop_hi=hi, diag_mask=ALL_DIAG, flags=flags,
                    trace_chains=inits.shape[0], trace_cap=400000, tune=tune)
    run = FlipRun(fg, inits, cfg, bases=bases)
    per = steps // chunks
    for i in range(chunks):
        run.steps(per if i < chunks - 1 else steps - per * (chunks - 1))
    return run


def _check(cref, spec, run, k, inits, bases, *, steps, pct, seed=21):
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    st = run.stats()
    pops = run.pops()
    ch, nh = run.hist()
    ct = run.cut_times()
    nf, ps, lf = run.flips()
    state = run.state()
    for c in range(inits.shape[0]):
        ref = cref.run(spec, inits[c], base=float(bases[c]), pop_lo=lo, pop_hi=hi, seed=seed, chain_id=c,
                       n_steps=steps, k=k, labels=list(range(k)), log1mp=G.log1mp_table(spec.n, k),
                       trace_cap=500000, want_hist=True, want_edges=True, want_flips=True, proposal=1)
        tr, rt = run.trace(c), ref["trace"]
        assert len(tr) == len(rt), f"chain {c}: {len(tr)} vs {len(rt)} proposals"
        for f in ("draw", "v", "flags", "cut", "nb", "wait"):
            bad = np.nonzero(tr[f] != rt[f])[0]
            assert bad.size == 0, f"chain {c} field {f} first mismatch at {bad[:1]}: {tr[bad[:3]]} vs {rt[bad[:3]]}"
        for key in STAT_KEYS:
            assert int(st[key][c]) == int(ref["stats"][key]), f"chain {c} stat {key}"
        assert np.array_equal(state[c], ref["final"])
        _, _, p_ref = G.cut_and_boundary(spec, ref["final"])
        assert np.array_equal(pops[c], np.resize(p_ref, k))
        assert np.array_equal(ch[c], ref["cut_hist"]) and np.array_equal(nh[c], ref["nb_hist"])
        assert np.array_equal(ct[c], ref["cut_times"])
        assert np.array_equal(nf[c], ref["num_flips"]) and np.array_equal(lf[c], ref["last_flipped"])
        assert np.array_equal(ps[c], ref["part_sum"])


@pytest.mark.parametrize("chunks", [1, 3])
def test_c3_sec11_k4_pair_parity(gpu, cref, sec11, chunks):
    k, n_chains, steps = 4, 16, 2500
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    inits = np.stack([a0] * n_chains)
    bases = np.asarray([[G.SEC11_MU, 1.0, 0.5, 4.0][c % 4] for c in range(n_chains)])
    run = _run_pair(sec11, inits, bases, k, steps=steps, pct=0.05, chunks=chunks)
    _check(cref, sec11, run, k, inits, bases, steps=steps, pct=0.05)


def test_c3_force_bfs(gpu, cref, sec11):
    k = 4
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    inits = np.stack([a0] * 8)
    bases = np.asarray([0.3, 1.0, G.SEC11_MU, 8.0] * 2)
    run = _run_pair(sec11, inits, bases, k, steps=1500, pct=0.05, flags=_lib.FC_FLAG_FORCE_BFS)
    assert run.stats()["bfs_calls"].sum() > 0
    _check(cref, sec11, run, k, inits, bases, steps=1500, pct=0.05)


@pytest.mark.parametrize("m,n", [(20, 38), (40, 78)])
def test_c4_triangular_k8_pair_parity(gpu, cref, m, n):
    spec = G.triangular_graph(m, n)
    k = 8
    a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    inits = np.stack([a0] * 8)
    bases = np.asarray([1 / 2.0, 1.0, 2.0, 4.0] * 2)
    run = _run_pair(spec, inits, bases, k, steps=2000, pct=0.1)
    _check(cref, spec, run, k, inits, bases, steps=2000, pct=0.1)


def test_pair_k2_equals_bi_sign_gpu(gpu, sec11):
    k = 2
    inits = np.stack([sec11.assignment_array(G.sec11_plan(c % 3, sec11.nodes), [-1, 1]) for c in range(12)])
    bases = np.asarray(G.SEC11_BASES[:6] * 2)
    r0 = _run_pair(sec11, inits, bases, k, steps=2000, pct=0.1, proposal=_lib.FC_PROPOSE_BI_SIGN)
    r1 = _run_pair(sec11, inits, bases, k, steps=2000, pct=0.1)
    for c in range(12):
        assert np.array_equal(r0.trace(c), r1.trace(c))
    assert np.array_equal(r0.state(), r1.state())


def test_pair_rejects_bad_config(gpu, sec11):
    fg = FlipGraph(sec11)
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), [0, 1, 2, 3])[None, :]
    with pytest.raises(ValueError):  # BI_SIGN only flips between two districts
        FlipRun(fg, a0, RunConfig(k=4, labels=(0, 1, 2, 3), proposal=_lib.FC_PROPOSE_BI_SIGN,
                                  pop_lo=0, pop_hi=10 ** 6))
    with pytest.raises(NotImplementedError):
        FlipRun(fg, a0, RunConfig(k=40, labels=tuple(range(40)), proposal=_lib.FC_PROPOSE_PAIR,
                                  pop_lo=0, pop_hi=10 ** 6))


@pytest.mark.parametrize("n_points,steps", [(2000, 3000), (10000, 1500)])
def test_c5_delaunay_k18_pair_parity(gpu, cref, n_points, steps):
    """C5: Delaunay dual of uniform points (irregular degree up to 16), lognormal
    populations, k = 18 recursive-bisection plan, pop tolerance 0.1."""
    spec = G.delaunay_graph(n_points, seed=0)
    k = 18
    a0 = spec.assignment_array(G.bisection_plan(spec, k), list(range(k)))
    inits = np.stack([a0] * 8)
    bases = np.asarray([0.5, 1.0, 2.0, 4.0] * 2)
    run = _run_pair(spec, inits, bases, k, steps=steps, pct=0.1)
    _check(cref, spec, run, k, inits, bases, steps=steps, pct=0.1)


@pytest.mark.parametrize("graph", ["delaunay", "triangular"])
def test_k2_irregular_graphs_parity(gpu, cref, graph):
    """The k = 2 kernel off the square lattice: ring length 16 (Delaunay) or 6 (triangular),
    nodes the planar rule leaves to the wave search, labels (0, 1), every per-yield tally on,
    and stale slot views re-evaluated in place -- bit-exact against the oracle."""
    if graph == "delaunay":
        spec = G.delaunay_graph(1500, seed=0)
        a0 = spec.assignment_array(G.bisection_plan(spec, 2), [0, 1])
    else:
        spec = G.triangular_graph(30, 58)
        a0 = spec.assignment_array(G.strip_plan(spec, 2), [0, 1])
    inits = np.stack([a0] * 8)
    bases = np.asarray([0.5, 1.0, 2.0, 4.0] * 2)
    run = _run_pair(spec, inits, bases, 2, steps=3000, pct=0.1, chunks=2, proposal=_lib.FC_PROPOSE_BI_SIGN)
    assert "flip2_kernel" in run.kernel_name(), run.kernel_name()
    _check(cref, spec, run, 2, inits, bases, steps=3000, pct=0.1)


@pytest.mark.parametrize("launches", [[4] * 10 + [45] * 6, [2500]])
def test_c3_lean_wait_queue(gpu, cref, sec11, launches):
    """Without a trace or tape the general-k kernel queues accepted states (32 entries) and
    draws their geometric waits later (fc_kernels.hip wait_flush); batches accepting more than
    the queue holds draw them at once.  Short launches and one long launch give the oracle's
    sum of waits and current wait bit for bit."""
    k, n_chains = 4, 12
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    inits = np.stack([a0] * n_chains)
    bases = np.asarray([[0.5, 1.0, G.SEC11_MU, 3.0][c % 4] for c in range(n_chains)])
    fg = FlipGraph(sec11)
    _, (lo, hi) = G.population_bounds(int(sec11.pop.sum()), k, 0.05)
    cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=23, pop_lo=lo, pop_hi=hi)
    run = FlipRun(fg, inits, cfg, bases=bases)
    for n in launches:
        run.steps(n)
    st = run.stats()
    total = sum(launches)
    for c in range(n_chains):
        ref = cref.run(sec11, inits[c], base=float(bases[c]), pop_lo=lo, pop_hi=hi, seed=23, chain_id=c,
                       n_steps=total, k=k, labels=list(range(k)), log1mp=G.log1mp_table(sec11.n, k),
                       trace_cap=0, proposal=1)
        for key in ("steps", "accepted", "sum_wait", "wait_cur", "cut", "nb"):
            assert int(st[key][c]) == int(ref["stats"][key]), (launches[0], c, key)


@pytest.mark.parametrize("wait_queue", [1, 2, 7, 32])
def test_k4_wait_queue_lengths(gpu, cref, sec11, wait_queue):
    """The deferred-wait queue of the general-k kernel at every length (fc_params
    tune_wait_queue): a short queue makes batches that accept more states than it holds --
    the direct-draw path -- the common case, including right after a drain (empty queue) with
    rejected steps of the batch's start state still to charge (that order once
    lost wait_cur * r0).  Small bases and a loose population bound make most proposals
    accepted.  sum_wait and wait_cur are bit-exact against the oracle."""
    k, n_chains = 4, 16
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    inits = np.stack([a0] * n_chains)
    bases = np.asarray([[0.1, 0.3, 1.0, G.SEC11_MU][c % 4] for c in range(n_chains)])
    fg = FlipGraph(sec11)
    _, (lo, hi) = G.population_bounds(int(sec11.pop.sum()), k, 0.5)
    cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=29, pop_lo=lo, pop_hi=hi,
                    tune={"wait_queue": wait_queue})
    run = FlipRun(fg, inits, cfg, bases=bases)
    for n in (3, 40, 700, 1257):
        run.steps(n)
    st = run.stats()
    total = 3 + 40 + 700 + 1257
    assert int(st["accepted"].sum()) > 0.4 * n_chains * total  # most steps accept: multi-accept batches
    for c in range(n_chains):
        ref = cref.run(sec11, inits[c], base=float(bases[c]), pop_lo=lo, pop_hi=hi, seed=29, chain_id=c,
                       n_steps=total, k=k, labels=list(range(k)), log1mp=G.log1mp_table(sec11.n, k),
                       trace_cap=0, proposal=1)
        for key in ("steps", "accepted", "sum_wait", "wait_cur", "sum_cut", "sum_nb", "cut", "nb"):
            assert int(st[key][c]) == int(ref["stats"][key]), (wait_queue, c, key)


def test_tuning_fields_checked(gpu, sec11):
    """Out-of-range launch tuning is an FC_ERR_ARG (ValueError) naming the field and the kernel,
    never a generic HIP launch failure (an out-of-range FC_NSUB used to break every k > 2
    launch)."""
    fg = FlipGraph(sec11)
    a4 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(4)))
    _, (lo, hi) = G.population_bounds(int(sec11.pop.sum()), 4, 0.05)
    base = RunConfig(k=4, labels=tuple(range(4)), proposal=_lib.FC_PROPOSE_PAIR, seed=1, pop_lo=lo, pop_hi=hi)
    for bad, what in (({"nsub": 3}, "k > 2"), ({"wait_queue": 33}, "tune_wait_queue"),
                      ({"chains_per_block": 3}, "tune_chains_per_block"), ({"deal": 2}, "tune_deal")):
        cfg = RunConfig(**{**base.__dict__, "tune": bad})
        with pytest.raises(ValueError, match=what):
            FlipRun(fg, a4[None, :], cfg)


@pytest.mark.parametrize("waves", [4, 1])
@pytest.mark.parametrize("graph", ["delaunay10k", "triangular100"])
def test_large_graph_search_workgroup_and_wave(gpu, cref, graph, waves):
    """Large graphs given without positions (no planar rings, so neither the run rule's
    exactness nor the district-graph rule): every multi-run proposal goes to the device search
    -- by the whole 256-thread workgroup of the chain (tune_search_waves = 4) or by its one
    wave (1, the default).  Both are bit-exact against the oracle's
    BFS, per proposal, on C5's Delaunay graph (k = 18) and C4's triangular lattice (k = 8)."""
    if graph == "delaunay10k":
        spec = G.delaunay_graph(10000, seed=0)
        k = 18
        a0 = spec.assignment_array(G.bisection_plan(spec, k), list(range(k)))
    else:
        spec = G.triangular_graph(100, 198)
        k = 8
        a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    inits = np.stack([a0] * 6)
    bases = np.asarray([0.5, 1.0, 2.0] * 2)
    run = _run_pair(spec, inits, bases, k, steps=400, pct=0.1, chunks=2, use_positions=False,
                    tune={"search_waves": waves})
    st = run.stats()
    assert int(st["bfs_calls"].sum()) > 0
    _check(cref, spec, run, k, inits, bases, steps=400, pct=0.1)


def test_instance_selection_and_agreement(gpu, sec11):
    """The district-graph rule decides every C3 proposal, so the launch takes the instance without
    search code (KM = 3); FC_FLAG_FORCE_BFS takes the searching one (KM = 0).  Both are exact, so
    their chains agree state for state; likewise k = 2 without (SEARCH = false) and with forced
    search."""
    k, n_chains, steps = 4, 16, 1200
    a0 = sec11.assignment_array(G.quadrant_plan(sec11.nodes), list(range(k)))
    inits = np.stack([a0] * n_chains)
    bases = np.asarray([[0.5, 1.0, G.SEC11_MU, 3.0][c % 4] for c in range(n_chains)])
    runs = [_run_pair(sec11, inits, bases, k, steps=steps, pct=0.05, flags=f) for f in (0, _lib.FC_FLAG_FORCE_BFS)]
    assert runs[0].kernel_name().startswith("fc::flip_kernel<8, 2, 3, "), runs[0].kernel_name()
    assert runs[1].kernel_name().startswith("fc::flip_kernel<8, 2, 0, "), runs[1].kernel_name()
    assert runs[0].stats()["bfs_calls"].sum() == 0 and runs[1].stats()["bfs_calls"].sum() > 0
    for key in ("steps", "proposals", "accepted", "sum_cut", "sum_nb", "sum_wait", "cut", "nb"):
        assert np.array_equal(runs[0].stats()[key], runs[1].stats()[key]), key
    assert np.array_equal(runs[0].state(), runs[1].state())
    i2 = np.stack([sec11.assignment_array(G.sec11_plan(c % 3, sec11.nodes), [-1, 1]) for c in range(n_chains)])
    b2 = np.asarray([G.SEC11_BASES[c % 10] for c in range(n_chains)])
    r2 = [_run_pair(sec11, i2, b2, 2, steps=steps, pct=0.1, flags=f, proposal=_lib.FC_PROPOSE_BI_SIGN)
          for f in (0, _lib.FC_FLAG_FORCE_BFS)]
    # (every chain traced: the XTRA diagnostics instance, SEARCH the fourth parameter)
    assert r2[0].kernel_name().endswith(", true, false, true, false>"), r2[0].kernel_name()
    assert r2[1].kernel_name().endswith(", true, true, true, false>"), r2[1].kernel_name()
    for key in ("steps", "proposals", "accepted", "sum_cut", "sum_nb", "sum_wait", "cut", "nb"):
        assert np.array_equal(r2[0].stats()[key], r2[1].stats()[key]), key
    assert np.array_equal(r2[0].state(), r2[1].state())


@pytest.mark.parametrize("flags", [0, _lib.FC_FLAG_FORCE_BFS])
def test_enclave_states_district_rule(gpu, cref, flags):
    """k = 3 grids whose district 2 starts as an enclave inside district 1, some of them one row
    or column from the outer face (tests/test_district_rule.py ENCLAVES): outer nodes there have
    their old-district neighbours on two ring runs separated by the enclave and the outer-face
    wedge, and flipping them keeps district 1 connected around the enclave.  The district-graph
    instance (KM = 3) rejected exactly those flips before the wedge fix; it and the
    forced-search instance must match the oracle's BFS per proposal."""
    from test_district_rule import ENCLAVES, enclave_plan
    spec = G.grid_graph(16, 16)
    k = 3
    inits = np.stack([enclave_plan(spec, ex, ey) for ex, ey in ENCLAVES] * 2)
    bases = np.asarray([4.0] * len(ENCLAVES) + [1.0] * len(ENCLAVES))
    run = _run_pair(spec, inits, bases, k, steps=600, pct=0.95, flags=flags)
    want = "fc::flip_kernel<8, 2, 0, " if flags else "fc::flip_kernel<8, 2, 3, "
    assert run.kernel_name().startswith(want), run.kernel_name()
    _check(cref, spec, run, k, inits, bases, steps=600, pct=0.95)


@pytest.mark.parametrize("chunks", [1, 3])
def test_pair_slot_bound_long_chain_across_launches(gpu, cref, chunks):
    """The canonical PAIR slot bound (the state's largest foreign-district count,
    kept per chain as a histogram) over 9,000 steps, in one launch and in three: flips move the
    bound and end their batch when they do, and every proposal matches the oracle (base 1:
    every valid proposal accepted)."""
    spec = G.triangular_graph(20, 38)
    k = 6
    a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    inits = np.stack([a0] * 6)
    bases = np.asarray([1.0, 0.5, 1.0, 3.0, 1.0, 0.25])
    run = _run_pair(spec, inits, bases, k, steps=9000, pct=0.3, chunks=chunks)
    _check(cref, spec, run, k, inits, bases, steps=9000, pct=0.3)


@pytest.mark.parametrize("chunks", [1, 3])
def test_packed_node_bytes_saturated_counts(gpu, cref, chunks):
    """The district-rule instance packs a node into one byte (district | foreign districts
    saturated at 7).  A wheel whose hub, alone in district 0, touches eight rim districts has a
    saturated count from the start: the slot filter passes it to the exact recount, the nf
    histogram (the canonical slot bound) follows exact counts, and the write-back restores the
    exact count between launches.  Per proposal against the oracle, in one and three launches."""
    import math
    import networkx as nx
    m, k = 15, 9
    g = nx.wheel_graph(m + 1)  # hub 0, rim 1..m
    pos = {0: (0.0, 0.0)}
    pos.update({i: (math.cos(2 * math.pi * i / m), math.sin(2 * math.pi * i / m)) for i in range(1, m + 1)})
    spec = G.from_networkx(g, pos=pos)
    a0 = np.zeros(spec.n, dtype=np.int8)
    for i in range(1, m + 1):  # districts 1..7 two rim nodes each, district 8 the last one
        a0[spec.index[i]] = min((i - 1) // 2 + 1, k - 1)
    inits = np.stack([a0] * 12)
    bases = np.asarray([[0.5, 1.0, 3.0][c % 3] for c in range(12)])
    run = _run_pair(spec, inits, bases, k, steps=3000, pct=0.9, chunks=chunks)
    assert run.kernel_name().startswith("fc::flip_kernel<16, "), run.kernel_name()
    assert ", 3, " in run.kernel_name()  # the district-rule (packed) instance
    _check(cref, spec, run, k, inits, bases, steps=3000, pct=0.9)


@pytest.mark.parametrize("case", ["c3_tight", "c4", "c5", "grid_small"])
def test_multi_flip_commit_equals_one_at_a_time(gpu, cref, sec11, case):
    """The district-rule instance commits several independent accepted flips per pass
    (fc_params.tune_multi_flip; auto = on, forced on here): traced
    per proposal against the oracle, and its
    lean instance state for state against one flip at a time.  c3_tight: sec11 k = 4 with a 1 %
    population tolerance (population verdicts change under the flips taken before them); c4 /
    c5: the triangular lattice and the Delaunay graph, always-accept base 1 among the bases;
    grid_small: nine districts of 16 cells, whose adjacencies and slot bound move often, so the
    pass's all-at-once district-table update falls back to one flip at a time (tools/mf_cover.py
    counts those passes with the FC_PHASE_PROF build)."""
    if case == "c3_tight":
        spec, k, pct, steps = sec11, 4, 0.01, 2000
        a0 = spec.assignment_array(G.quadrant_plan(spec.nodes), list(range(k)))
    elif case == "c4":
        spec, k, pct, steps = G.triangular_graph(40, 78), 8, 0.1, 2000
        a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    elif case == "c5":
        spec, k, pct, steps = G.delaunay_graph(2000, seed=0), 18, 0.1, 2000
        a0 = spec.assignment_array(G.bisection_plan(spec, k), list(range(k)))
    else:
        spec, k, pct, steps = G.grid_graph(12, 12), 9, 0.9, 3000
        a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    inits = np.stack([a0] * 12)
    bases = np.asarray([1.0, 0.5, 2.0, 1.0] * 3)
    run = _run_pair(spec, inits, bases, k, steps=steps, pct=pct, chunks=2, tune={"multi_flip": 1})
    name = run.kernel_name()
    assert ", 3, " in name, name
    assert name.endswith((", true, 1>", ", true, 2>")), name  # FULL (traced), multi-flip (hashed / exact marks)
    _check(cref, spec, run, k, inits, bases, steps=steps, pct=pct)
    fg = FlipGraph(spec)
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    outs = []
    # on (auto marks), off, and both mark forms forced (2: hashed, 3: exact)
    for tune in ({"multi_flip": 1}, {"multi_flip": -1}, {"multi_flip": 2}, {"multi_flip": 3}):
        cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=21, pop_lo=lo, pop_hi=hi,
                        tune=tune)
        r = FlipRun(fg, inits, cfg, bases=bases)
        r.steps(steps // 2)
        r.steps(steps - steps // 2)
        outs.append((r.stats(), r.state()))
    for o in outs[1:]:
        for key in STAT_KEYS + ["wait_cur"]:
            assert np.array_equal(outs[0][0][key], o[0][key]), key
        assert np.array_equal(outs[0][1], o[1])
