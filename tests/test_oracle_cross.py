"""The two oracle restatements (plain C, gerrychain-0.2-faithful Python) agree bit-exactly,
and the canonical stream matches the Random123 Philox known answers."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G


def test_philox_known_answers(cref):
    from oracle.flipref import philox4x32_10
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, exp in kat:
        assert tuple(cref.philox(ctr, key)) == exp
        assert tuple(int(x) for x in philox4x32_10(*ctr, *key)) == exp


@pytest.mark.parametrize("base,al", [(0.1, 0), (1.0, 2), (G.SEC11_MU, 1), (10, 0)])
def test_c_oracle_equals_gc_faithful(cref, sec11, base, al):
    from oracle.flipref import GcFaithfulChain
    l1 = G.log1mp_table(sec11.n, 2)
    plan = G.sec11_plan(al, sec11.nodes)
    a0 = sec11.assignment_array(plan, [-1, 1])
    (lo, hi), (ilo, ihi) = G.population_bounds(sec11.n, 2, 0.1)
    gc = GcFaithfulChain(sec11, plan, base=base, pop_bounds=(lo, hi), seed=3, chain_id=al, log1mp=l1).run(250)
    r = cref.run(sec11, a0, base=base, pop_lo=ilo, pop_hi=ihi, seed=3, chain_id=al, n_steps=250, log1mp=l1,
                 trace_cap=100000)
    gtr = np.array(gc.trace, dtype=np.int64)
    tr = r["trace"]
    assert len(tr) == len(gtr)
    for i, f in enumerate(["draw", "v", "flags", "cut", "nb", "wait"]):
        assert np.array_equal(tr[f], gtr[:, i]), f
    assert np.array_equal(gc.assignment_ids(), r["final"])
    for k in ("steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb", "sum_wait"):
        assert gc.stats[k] == r["stats"][k], k


def test_tape_and_philox_agree(cref, sec11):
    from oracle.flipref import draw_tape
    l1 = G.log1mp_table(sec11.n, 2)
    a0 = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])
    _, (lo, hi) = G.population_bounds(sec11.n, 2, 0.1)
    tape = draw_tape(9, 4, 30000, k=2)
    r1 = cref.run(sec11, a0, base=0.8, pop_lo=lo, pop_hi=hi, seed=9, chain_id=4, n_steps=2000, log1mp=l1,
                  trace_cap=100000)
    r2 = cref.run(sec11, a0, base=0.8, pop_lo=lo, pop_hi=hi, seed=9, chain_id=4, n_steps=2000, log1mp=l1,
                  trace_cap=100000, tape=tape)
    assert np.array_equal(r1["trace"], r2["trace"])
    assert r1["stats"] == r2["stats"]


def test_oracle_rejects_invalid_initial_state(cref, sec11):
    a0 = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1]).copy()
    a0[sec11.index[(0, 5)]] = 1
    with pytest.raises(ValueError):
        cref.run(sec11, a0, base=1.0, pop_lo=0, pop_hi=10 ** 6, seed=0, chain_id=0, n_steps=1)


def test_oracle_stuck_cap(cref, sec11):
    a0 = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])
    # population bound pinned at exactly 798/798 -> no proposal can ever be valid
    r = cref.run(sec11, a0, base=1.0, pop_lo=798, pop_hi=798, seed=0, chain_id=0, n_steps=10, max_draws=5000)
    assert r["rc"] == 1 and r["stats"]["stuck"] == 1 and r["stats"]["steps"] == 0
    assert r["stats"]["inv_pop"] > 0


@pytest.mark.parametrize("nb_pairs", [False, True])
@pytest.mark.parametrize("which,k,base", [("sec11", 4, G.SEC11_MU), ("sec11", 4, 0.5), ("tri", 8, 1.0)])
def test_c_oracle_pair_equals_gc_faithful(cref, sec11, which, k, base, nb_pairs):
    """PAIR proposals (slow_reversible_propose over b_nodes pairs, grid_chain_sec11.py:117-130,
    151-153) for k > 2: the C restatement equals the gerrychain-faithful one -- with |b_nodes|
    counted as nodes (b_nodes_bi) or, ``nb_pairs``, as the pair updater's pairs (what
    len(part["b_nodes"]) is in a driver that registers it: rbn, and geom_wait's p)."""
    from oracle.flipref import GcFaithfulChain
    spec = sec11 if which == "sec11" else G.triangular_graph(12, 22)
    plan = G.quadrant_plan(spec.nodes) if which == "sec11" else G.strip_plan(spec, k)
    labels = list(range(k))
    a0 = spec.assignment_array(plan, labels)
    l1 = G.log1mp_table(spec.n, k, G.nb_width(spec, k, nb_pairs))
    pct = 0.05 if which == "sec11" else 0.1
    (lo, hi), (ilo, ihi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    gc = GcFaithfulChain(spec, plan, base=base, pop_bounds=(lo, hi), seed=5, chain_id=2, log1mp=l1,
                         pair=True, nb_pairs=nb_pairs).run(300)
    r = cref.run(spec, a0, base=base, pop_lo=ilo, pop_hi=ihi, seed=5, chain_id=2, n_steps=300, k=k,
                 labels=labels, log1mp=l1, trace_cap=100000, proposal=1, nb_pairs=nb_pairs, want_hist=True)
    assert r["nb_hist"].size == l1.size and r["nb_hist"].sum() == 301
    gtr = np.array(gc.trace, dtype=np.int64)
    tr = r["trace"]
    assert len(tr) == len(gtr) and len(tr) > 300
    for i, f in enumerate(["draw", "v", "flags", "cut", "nb", "wait"]):
        assert np.array_equal(tr[f], gtr[:, i]), f
    assert np.array_equal(gc.assignment_ids(), r["final"])
    for key in ("steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb", "sum_wait"):
        assert gc.stats[key] == r["stats"][key], key


def test_pair_k2_equals_bi_sign(cref, sec11):
    """With k = 2 the pair set has one district per boundary node: PAIR == BI_SIGN."""
    l1 = G.log1mp_table(sec11.n, 2)
    a0 = sec11.assignment_array(G.sec11_plan(1, sec11.nodes), [-1, 1])
    _, (lo, hi) = G.population_bounds(sec11.n, 2, 0.1)
    kw = dict(base=0.8, pop_lo=lo, pop_hi=hi, seed=4, chain_id=7, n_steps=1500, log1mp=l1, trace_cap=100000)
    r0 = cref.run(sec11, a0, proposal=0, **kw)
    r1 = cref.run(sec11, a0, proposal=1, **kw)
    assert np.array_equal(r0["trace"], r1["trace"])
    assert r0["stats"] == r1["stats"]


def test_c_oracle_pair_delaunay_equals_gc_faithful(cref):
    """Irregular planar dual graph with non-unit populations (C5's family), k = 6."""
    from oracle.flipref import GcFaithfulChain
    spec = G.delaunay_graph(300, seed=3)
    k = 6
    plan = G.bisection_plan(spec, k)
    a0 = spec.assignment_array(plan, list(range(k)))
    l1 = G.log1mp_table(spec.n, k)
    (lo, hi), (ilo, ihi) = G.population_bounds(int(spec.pop.sum()), k, 0.1)
    gc = GcFaithfulChain(spec, plan, base=1.5, pop_bounds=(lo, hi), seed=8, chain_id=1, log1mp=l1,
                         pair=True).run(300)
    r = cref.run(spec, a0, base=1.5, pop_lo=ilo, pop_hi=ihi, seed=8, chain_id=1, n_steps=300, k=k,
                 labels=list(range(k)), log1mp=l1, trace_cap=100000, proposal=1)
    gtr = np.array(gc.trace, dtype=np.int64)
    assert len(r["trace"]) == len(gtr)
    for i, f in enumerate(["draw", "v", "flags", "cut", "nb", "wait"]):
        assert np.array_equal(r["trace"][f], gtr[:, i]), f
    assert np.array_equal(gc.assignment_ids(), r["final"])


def test_bisection_plan_is_valid():
    import networkx as nx
    spec = G.delaunay_graph(2000, seed=1)
    plan = G.bisection_plan(spec, 18)
    a = spec.assignment_array(plan, list(range(18)))
    _, _, pops = G.cut_and_boundary(spec, a)
    (lo, hi), _ = G.population_bounds(int(spec.pop.sum()), 18, 0.1)
    assert pops.min() >= lo and pops.max() <= hi
    for d in range(18):
        assert nx.is_connected(spec.nx_graph.subgraph([n for n in spec.nodes if plan[n] == d]))


def test_oracle_variants_respect_their_constraints(cref, sec11):
    """The oracle's variant restatements keep what they promise: pinned edges stay cut,
    both districts keep a boundary_node, and accept-side constraints reject (a rejected
    step re-yields) instead of re-drawing."""
    from flipcomplexityempirical_amd import graphs as G
    from oracle import flipref as F
    a0 = sec11.assignment_array(G.sec11_plan(0, sec11.nodes), [-1, 1])
    _, (lo, hi) = G.population_bounds(sec11.n, 2, 0.1)
    frame = np.asarray([1 if (0 in nd or 39 in nd) else 0 for nd in sec11.nodes], dtype=np.uint8)
    pinned = np.asarray([(sec11.index[(19, 0)], sec11.index[(20, 0)]),
                         (sec11.index[(19, 39)], sec11.index[(20, 39)])], dtype=np.int32)
    r = cref.run(sec11, a0, base=1.0, pop_lo=lo, pop_hi=hi, seed=5, chain_id=0, n_steps=20000,
                 accept=F.ACCEPT_CUT, con_valid=F.CON_CONTIG | F.CON_POP | F.CON_BOUNDARY | F.CON_FIXED,
                 boundary=frame, pinned=pinned)
    fin = r["final"]
    assert all(fin[u] != fin[w] for u, w in pinned)
    assert len(set(fin[frame == 1].tolist())) == 2
    assert r["stats"]["accepted"] > 1000
    # uniform_accept with an empty Validator: invalid proposals become rejected steps
    r2 = cref.run(sec11, a0, base=1.0, pop_lo=lo, pop_hi=hi, seed=5, chain_id=0, n_steps=5000,
                  accept=F.ACCEPT_UNIFORM, con_valid=F.CON_EMPTY, con_accept=F.CON_CONTIG | F.CON_POP | F.CON_BOUNDARY,
                  boundary=frame)
    s2 = r2["stats"]
    assert s2["inv_contig"] == 0 and s2["inv_pop"] == 0 and s2["steps"] == s2["proposals"] == 5000
    assert 0 < s2["accepted"] < 5000


def test_recom_oracle_keeps_plans_valid(cref, sec11):
    """The ReCom restatement moves whole subtrees: every state it yields has contiguous
    districts inside the population bound, and it accepts every valid step at base 1."""
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import recom_run
    a0 = sec11.assignment_array(G.sec11_plan(2, sec11.nodes), [-1, 1])
    _, (lo, hi) = G.population_bounds(sec11.n, 2, 0.1)
    r = recom_run(sec11, a0, k=2, pop_target=sec11.n / 2, epsilon=0.05, pop_lo=lo, pop_hi=hi, seed=4, chain_id=1,
                  n_steps=50, trace_cap=200)
    s = r["stats"]
    assert s["steps"] == 50 and s["accepted"] == 50 and s["trees"] >= 50
    assert cref.districts_contiguous(sec11, r["final"], 2)
    cut, nb, pops = G.cut_and_boundary(sec11, r["final"])
    assert (cut, nb) == (s["cut"], s["nb"]) and lo <= pops.min() and pops.max() <= hi
    assert np.all(np.abs(np.array([pops[0], pops[1]]) - sec11.n / 2) < 0.05 * sec11.n / 2)


def test_c_oracle_pair_slot_bound_long_chain(cref):
    """The canonical PAIR slot bound (the state's largest foreign-district count; oracle/flipref.c)
    over 10,000 steps of a k = 5 triangular chain at base 1 (every valid proposal accepted, so
    the bound moves often): the C restatement equals the gerrychain-faithful one draw for draw,
    and a fixed bound (wmax) wastes more slot draws."""
    from oracle.flipref import GcFaithfulChain
    spec = G.triangular_graph(10, 18)
    k = 5
    plan = G.strip_plan(spec, k)
    labels = list(range(k))
    a0 = spec.assignment_array(plan, labels)
    l1 = G.log1mp_table(spec.n, k)
    (lo, hi), (ilo, ihi) = G.population_bounds(int(spec.pop.sum()), k, 0.3)
    steps = 10000
    gc = GcFaithfulChain(spec, plan, base=1.0, pop_bounds=(lo, hi), seed=9, chain_id=3, log1mp=l1,
                         pair=True).run(steps)
    r = cref.run(spec, a0, base=1.0, pop_lo=ilo, pop_hi=ihi, seed=9, chain_id=3, n_steps=steps, k=k,
                 labels=labels, log1mp=l1, trace_cap=200000, proposal=1)
    gtr = np.array(gc.trace, dtype=np.int64)
    assert len(r["trace"]) == len(gtr)
    for i, f in enumerate(["draw", "v", "flags", "cut", "nb", "wait"]):
        assert np.array_equal(r["trace"][f], gtr[:, i]), f
    assert np.array_equal(gc.assignment_ids(), r["final"])
    fixed = cref.run(spec, a0, base=1.0, pop_lo=ilo, pop_hi=ihi, seed=9, chain_id=3, n_steps=steps, k=k,
                     labels=labels, log1mp=l1, proposal=1, wmax=k - 1)
    assert fixed["stats"]["draws"] > r["stats"]["draws"]  # the fixed bound wastes more slot draws


@pytest.mark.parametrize("base,al,steps", [(1.0, 0, 300), (G.SEC11_MU, 1, 1500), (10, 2, 2000)])
def test_band_stream_c_equals_gc_faithful(cref, sec11, base, al, steps):
    """The band stream (nodes drawn over S = b_nodes + neighbours, rebuilt lazily) is the same
    in both restatements, S rebuilds included."""
    from oracle.flipref import GcFaithfulChain, STREAM_BAND
    l1 = G.log1mp_table(sec11.n, 2)
    plan = G.sec11_plan(al, sec11.nodes)
    a0 = sec11.assignment_array(plan, [-1, 1])
    (lo, hi), (ilo, ihi) = G.population_bounds(sec11.n, 2, 0.1)
    gc = GcFaithfulChain(sec11, plan, base=base, pop_bounds=(lo, hi), seed=5, chain_id=al, log1mp=l1, band=True)
    rebuilds = 0
    S = gc.band_set
    for _ in range(steps):
        gc.step()
        rebuilds += gc.band_set is not S
        S = gc.band_set
    r = cref.run(sec11, a0, base=base, pop_lo=ilo, pop_hi=ihi, seed=5, chain_id=al, n_steps=steps, log1mp=l1,
                 trace_cap=200000, stream=STREAM_BAND)
    gtr = np.array(gc.trace, dtype=np.int64)
    tr = r["trace"]
    assert len(tr) == len(gtr)
    for i, f in enumerate(["draw", "v", "flags", "cut", "nb", "wait"]):
        assert np.array_equal(tr[f], gtr[:, i]), f
    assert np.array_equal(gc.assignment_ids(), r["final"])
    for k in ("steps", "proposals", "draws", "accepted", "sum_cut", "sum_nb", "sum_wait"):
        assert gc.stats[k] == r["stats"][k], k
    if base == 10:
        assert rebuilds >= 2  # the rebuild rule is exercised
        # short boundary: the band stream wastes far fewer draws than the node stream
        assert r["stats"]["draws"] < 4 * r["stats"]["proposals"]
