"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit-exact.

Every comparison is per proposal -- (draw, node, valid/accepted/invalid-reason, |cut|,
|B|, geometric wait) -- plus final assignments, counters and all per-yield diagnostics.
Both sides consume the same canonical random stream (DESIGN.md "Random stream").
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


def _configs(spec, plan_fn, bases, n_chains):
    inits, bs = [], []
    for c in range(n_chains):
        al = c % 3
        inits.append(spec.assignment_array(plan_fn(al, spec.nodes), [-1, 1]))
        bs.append(bases[(c // 3) % len(bases)])
    return np.stack(inits), np.asarray(bs)


def _run_gpu(spec, inits, bases, *, steps, chunks=1, seed=11, pct=0.1, flags=0, diag=ALL_DIAG,
             trace_cap=200000, exact=True, tape=None):
    fg = FlipGraph(spec, exact=exact)
    (_, _), (lo, hi) = G.population_bounds(int(spec.pop.sum()), 2, pct)
    cfg = RunConfig(seed=seed, pop_lo=lo, pop_hi=hi, diag_mask=diag, flags=flags,
                    trace_chains=inits.shape[0], trace_cap=trace_cap)
    run = FlipRun(fg, inits, cfg, bases=bases)
    if tape is not None:
        run.set_tape(tape)
    per = steps // chunks
    for i in range(chunks):
        run.steps(per if i < chunks - 1 else steps - per * (chunks - 1))
    return fg, run


def _check_chain(cref, spec, run, c, init, base, *, steps, seed=11, pct=0.1, tape=None, diag=True,
                 trace_cap=500000):
    (_, _), (lo, hi) = G.population_bounds(int(spec.pop.sum()), 2, pct)
    ref = cref.run(spec, init, base=base, pop_lo=lo, pop_hi=hi, seed=seed, chain_id=c, n_steps=steps,
                   log1mp=G.log1mp_table(spec.n, 2), trace_cap=trace_cap, want_hist=diag, want_edges=diag,
                   want_flips=diag, tape=tape)
    assert len(ref["trace"]) < trace_cap
    st = run.stats()
    tr = run.trace(c)
    rt = ref["trace"]
    assert len(tr) == len(rt), f"chain {c}: {len(tr)} vs {len(rt)} proposals"
    for f in ("draw", "v", "flags", "cut", "nb", "wait"):
        bad = np.nonzero(tr[f] != rt[f])[0]
        assert bad.size == 0, f"chain {c} field {f} first mismatch at proposal {bad[:1]}: {tr[bad[:3]]} vs {rt[bad[:3]]}"
    for k in STAT_KEYS:
        assert int(st[k][c]) == int(ref["stats"][k]), f"chain {c} stat {k}: {st[k][c]} vs {ref['stats'][k]}"
    assert np.array_equal(run.state()[c], ref["final"])
    return ref


@pytest.mark.parametrize("chunks", [1, 4])
def test_sec11_trace_parity(gpu, cref, sec11, chunks):
    inits, bases = _configs(sec11, G.sec11_plan, G.SEC11_BASES, 30)
    _, run = _run_gpu(sec11, inits, bases, steps=3000, chunks=chunks)
    ch, nh = run.hist()
    ct = run.cut_times()
    nf, ps, lf = run.flips()
    for c in range(inits.shape[0]):
        ref = _check_chain(cref, sec11, run, c, inits[c], bases[c], steps=3000)
        assert np.array_equal(ch[c], ref["cut_hist"])
        assert np.array_equal(nh[c], ref["nb_hist"])
        assert np.array_equal(ct[c], ref["cut_times"])
        assert np.array_equal(nf[c], ref["num_flips"])
        assert np.array_equal(lf[c], ref["last_flipped"])
        assert np.array_equal(ps[c], ref["part_sum"])


def test_sec11_force_bfs_parity(gpu, cref, sec11):
    """Device BFS instead of the exact planar rule: identical trajectories."""
    inits, bases = _configs(sec11, G.sec11_plan, [0.1, 1.0, G.SEC11_MU], 9)
    _, run = _run_gpu(sec11, inits, bases, steps=1500, flags=_lib.FC_FLAG_FORCE_BFS)
    st = run.stats()
    assert st["bfs_calls"].sum() > 0
    for c in range(inits.shape[0]):
        _check_chain(cref, sec11, run, c, inits[c], bases[c], steps=1500)


def test_sec11_no_positions_bfs_parity(gpu, cref, sec11):
    """Rings without an embedding (no exactness): local rule + BFS fallback."""
    inits, bases = _configs(sec11, G.sec11_plan, [0.2, 1.0, 4.0], 6)
    _, run = _run_gpu(sec11, inits, bases, steps=1000, exact=False)
    for c in range(inits.shape[0]):
        _check_chain(cref, sec11, run, c, inits[c], bases[c], steps=1000)


def test_frank_trace_parity(gpu, cref, frank):
    inits, bases = _configs(frank, G.frank_plan, G.FRANK_BASES, 12)
    _, run = _run_gpu(frank, inits, bases, steps=3000, pct=0.05)
    ct = run.cut_times()
    for c in range(inits.shape[0]):
        ref = _check_chain(cref, frank, run, c, inits[c], bases[c], steps=3000, pct=0.05)
        assert np.array_equal(ct[c], ref["cut_times"])


def test_tape_replay_matches_philox(gpu, cref, sec11):
    """Replay mode: a tape holding the Philox words reproduces the native run, and an
    arbitrary tape is replayed identically by the oracle."""
    from oracle.flipref import draw_tape
    inits, bases = _configs(sec11, G.sec11_plan, [1.0, 10.0], 4)
    n_draws = 60000
    tapes = np.stack([draw_tape(11, c, n_draws, k=2) for c in range(4)])
    _, run_t = _run_gpu(sec11, inits, bases, steps=1000, tape=tapes)
    _, run_p = _run_gpu(sec11, inits, bases, steps=1000)
    for c in range(4):
        assert np.array_equal(run_t.trace(c), run_p.trace(c))
    rng = np.random.default_rng(5)
    wild = rng.integers(0, 2 ** 32, size=(4, n_draws * 6), dtype=np.uint64).astype(np.uint32)
    _, run_w = _run_gpu(sec11, inits, bases, steps=800, tape=wild)
    for c in range(4):
        _check_chain(cref, sec11, run_w, c, inits[c], bases[c], steps=800, tape=wild[c])


@pytest.mark.parametrize("cap", [1, 255, 1001, 4099])
def test_k2_node_stream_draw_cap(gpu, cref, sec11, cap):
    """The four-per-call node stream when the launch's draw cap falls inside a
    batch window (and at 1 draw): the device stops at the cap exactly where the oracle does --
    every proposal, every counter (draws included), the final state and the stuck flag."""
    inits, bases = _configs(sec11, G.sec11_plan, [0.5, 10.0], 6)
    (_, _), (lo, hi) = G.population_bounds(int(sec11.pop.sum()), 2, 0.1)
    fg = FlipGraph(sec11)
    cfg = RunConfig(seed=11, pop_lo=lo, pop_hi=hi, diag_mask=ALL_DIAG, trace_chains=6, trace_cap=200000)
    run = FlipRun(fg, inits, cfg, bases=bases)
    run.steps(10 ** 6, max_draws=cap)
    st = run.stats()
    for c in range(6):
        ref = cref.run(sec11, inits[c], base=bases[c], pop_lo=lo, pop_hi=hi, seed=11, chain_id=c, n_steps=10 ** 6,
                       log1mp=G.log1mp_table(sec11.n, 2), trace_cap=200000, max_draws=cap)
        tr, rt = run.trace(c), ref["trace"]
        assert len(tr) == len(rt), (c, len(tr), len(rt))
        for f in ("draw", "v", "flags", "cut", "nb", "wait"):
            assert np.array_equal(tr[f], rt[f]), (c, f)
        for k in STAT_KEYS:
            assert int(st[k][c]) == int(ref["stats"][k]), (c, k)
        assert int(st["stuck"][c]) == 1 and int(ref["stats"]["stuck"]) == 1, c
        assert np.array_equal(run.state()[c], ref["final"]), c
    run.close()


def test_c1_grid10(gpu, cref):
    """BASELINE config C1 at its configured length: 10x10 grid, plan x[0] >= 5, base 1
    (lambda = 1), pop tolerance 0.1, one chain of 1e5 yields (99,999 steps after S0), plus the
    same chain at bases mu and 1/mu.  Every proposal, every per-yield tally (histograms,
    cut_times, num_flips / part_sum / last_flipped) and the final state are bit-exact."""
    spec = G.grid_graph(10, 10)
    a0 = spec.assignment_array(G.threshold_plan(spec.nodes, 0, 5), [-1, 1])
    inits = np.stack([a0] * 3)
    bases = np.asarray([1.0, G.SEC11_MU, 1 / G.SEC11_MU])
    steps = 99999
    _, run = _run_gpu(spec, inits, bases, steps=steps, chunks=3, trace_cap=1500000)
    ct = run.cut_times()
    nf, ps, lf = run.flips()
    ch, nh = run.hist()
    for c in range(3):
        ref = _check_chain(cref, spec, run, c, inits[c], bases[c], steps=steps, trace_cap=1500000)
        assert np.array_equal(ct[c], ref["cut_times"])
        assert np.array_equal(nf[c], ref["num_flips"]) and np.array_equal(ps[c], ref["part_sum"])
        assert np.array_equal(lf[c], ref["last_flipped"])
        assert np.array_equal(ch[c], ref["cut_hist"]) and np.array_equal(nh[c], ref["nb_hist"])
        assert int(ch[c].sum()) == steps + 1


def test_invalid_initial_state_raises(gpu, sec11):
    fg = FlipGraph(sec11)
    a = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1]).copy()
    a[sec11.index[(0, 5)]] = 1  # island of +1 inside -1: not contiguous
    with pytest.raises(ValueError):
        FlipRun(fg, a[None, :], RunConfig(pop_lo=0, pop_hi=10 ** 6))
    with pytest.raises(ValueError):
        FlipRun(fg, sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])[None, :],
                RunConfig(pop_lo=799, pop_hi=10 ** 6))


def test_sharded_equals_unsharded(gpu, sec11):
    """Chain g gives the same trajectory whichever GPU/shard runs it (global chain ids)."""
    from flipcomplexityempirical_amd import distributed as D
    n_total, world = 96, 3
    inits, bases = _configs(sec11, G.sec11_plan, G.SEC11_BASES, n_total)
    fg = FlipGraph(sec11)
    _, (lo, hi) = G.population_bounds(sec11.n, 2, 0.1)
    full = FlipRun(fg, inits, RunConfig(seed=5, pop_lo=lo, pop_hi=hi), bases=bases).steps(2000)
    fs, fa = full.stats(), full.state()
    for r in range(world):
        off, cnt = D.shard(n_total, world, r)
        part = FlipRun(fg, inits[off:off + cnt], RunConfig(seed=5, pop_lo=lo, pop_hi=hi, chain_id_offset=off),
                       bases=bases[off:off + cnt]).steps(2000)
        ps = part.stats()
        for k in ("steps", "proposals", "draws", "accepted", "sum_cut", "sum_wait", "cut", "nb"):
            assert np.array_equal(ps[k], fs[k][off:off + cnt]), k
        assert np.array_equal(part.state(), fa[off:off + cnt])


def test_hit_stop_refused_on_k2_node_stream(gpu, sec11):
    """The k = 2 node stream's batch window is 64 * nsub draws closed by the 64th hit: a round
    cut-off would change nothing, so a nonzero tune_hit_stop is an argument error there (ADVICE
    r04), not a silent no-op."""
    (_, _), (lo, hi) = G.population_bounds(int(sec11.pop.sum()), 2, 0.1)
    a0 = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])[None, :]
    with pytest.raises(ValueError, match="tune_hit_stop"):
        FlipRun(FlipGraph(sec11), a0, RunConfig(seed=1, pop_lo=lo, pop_hi=hi, tune={"hit_stop": 24}))
    FlipRun(FlipGraph(sec11), a0, RunConfig(seed=1, pop_lo=lo, pop_hi=hi, stream="band", tune={"hit_stop": 24}))


# (k = 2 node stream: no round cut-off -- tune_hit_stop is refused there; the band stream's
# shapes with it are in tests/test_band_gpu.py)
@pytest.mark.parametrize("nsub,hit_stop,extra", [(1, 0, {}), (2, 0, {}), (4, 0, {}),
                                               (4, 0, {"wait_queue": 1}), (4, 0, {"wait_queue": 3}),
                                               (4, 0, {"par_min": 65}), (4, 0, {"par_min": 1}),
                                               (4, 0, {"chains_per_block": 4}), (4, 0, {"deal": 1}),
                                               (4, 0, {"prio_div": (-1, 0, 0)}),
                                               (2, 0, {"prio_th": (-1.0, 0.0, 0.0)})])
@pytest.mark.parametrize("lean", [True, False])
def test_sec11_batch_shapes(gpu, cref, sec11, nsub, hit_stop, extra, lean):
    """Every launch-tuning field of fc_params the k = 2 node stream takes (draw rounds per batch
    ``tune_nsub``, the deferred-wait queue length, the segment-parallel threshold,
    chains per workgroup, issue priorities, chain dealing) is a scheduling choice only: the lean instance
    (waits only) and the full instance (trace + histograms) stay bit-exact against the oracle
    under each of them (the guarantee include/flipchain.h states for fc_params.tune_*)."""
    inits, bases = _configs(sec11, G.sec11_plan, G.SEC11_BASES, 30)
    # full: trace + histograms, without the per-edge / per-node tallies, so that stale slot
    # views are re-evaluated in place (the ALL_DIAG tests above cover the batch-ending form)
    diag = _lib.FC_DIAG_WAIT if lean else (_lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST)
    fg = FlipGraph(sec11)
    (_, _), (lo, hi) = G.population_bounds(int(sec11.pop.sum()), 2, 0.1)
    cfg = RunConfig(seed=11, pop_lo=lo, pop_hi=hi, diag_mask=diag, trace_chains=0 if lean else 30,
                    trace_cap=0 if lean else 200000, tune=dict(nsub=nsub, hit_stop=hit_stop, **extra))
    run = FlipRun(fg, inits, cfg, bases=bases)
    run.steps(1500)
    run.steps(1500)
    name = run.kernel_name()
    # sec11: every node exact, so the instance without search code (fourth parameter false)
    assert f"flip2_kernel<8, {nsub}, {'false' if lean else 'true'}, false, " in name, name
    st = run.stats()
    fin = run.state()
    if not lean:
        ch, nh = run.hist()
    for c in range(30):
        ref = cref.run(sec11, inits[c], base=bases[c], pop_lo=lo, pop_hi=hi, seed=11, chain_id=c, n_steps=3000,
                       log1mp=G.log1mp_table(sec11.n, 2), trace_cap=500000, want_hist=not lean)
        for k in STAT_KEYS:
            assert int(st[k][c]) == int(ref["stats"][k]), (nsub, hit_stop, lean, c, k)
        assert np.array_equal(fin[c], ref["final"]), (nsub, hit_stop, lean, c)
        if not lean:
            tr, rt = run.trace(c), ref["trace"]
            assert len(tr) == len(rt) and all((tr[f] == rt[f]).all() for f in ("draw", "v", "flags", "cut", "nb", "wait"))
            assert np.array_equal(ch[c], ref["cut_hist"]) and np.array_equal(nh[c], ref["nb_hist"])


@pytest.mark.parametrize("lean", [True, False])
@pytest.mark.parametrize("launches", [[5] * 12 + [37] * 8, [3000]])
def test_sec11_lean_wait_queue(gpu, cref, sec11, launches, lean):
    """Without a trace or tape the k = 2 kernel (lean, or full with every tally but the trace)
    queues accepted states and draws their geometric waits later (fc_flip2.hip wait_flush: on
    queue overflow and at the end of each launch).  Launches of a few steps (the queue drained
    with the current state still running on) and one long launch (many overflows) give the
    oracle's sum of waits and current wait bit for bit."""
    inits, bases = _configs(sec11, G.sec11_plan, G.SEC11_BASES, 20)
    fg = FlipGraph(sec11)
    (_, _), (lo, hi) = G.population_bounds(int(sec11.pop.sum()), 2, 0.1)
    cfg = RunConfig(seed=13, pop_lo=lo, pop_hi=hi, diag_mask=_lib.FC_DIAG_WAIT if lean else ALL_DIAG)
    run = FlipRun(fg, inits, cfg, bases=bases)
    for n in launches:
        run.steps(n)
    assert f"flip2_kernel<8, 4, {'false' if lean else 'true'}, false, " in run.kernel_name()
    st = run.stats()
    total = sum(launches)
    for c in range(20):
        ref = cref.run(sec11, inits[c], base=bases[c], pop_lo=lo, pop_hi=hi, seed=13, chain_id=c, n_steps=total,
                       log1mp=G.log1mp_table(sec11.n, 2), trace_cap=0)
        for k in ("steps", "accepted", "sum_wait", "wait_cur", "cut", "nb"):
            assert int(st[k][c]) == int(ref["stats"][k]), (launches[0], c, k)
