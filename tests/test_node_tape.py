"""Node-tape replay of the reference's own proposal mechanism (north_star:
"bit-exact chain trajectories against the reference's own flip step when both are driven by
an identical replayed random stream").

``oracle.flipref.NativeRngChain`` runs the reference's flip step with its own random streams:
``random.choice(list(partition["b_nodes"]))`` (grid_chain_sec11.py:143) over CPython's set
order, gerrychain's ``random.choice`` of the contiguity start node, ``random.random()`` in
cut_accept (:179) and numpy's legacy ``geometric`` in geom_wait (:148), on gerrychain-0.2
structures (Partition dicts, cut-edge tuple sets, networkx Dijkstra).  With ``record=True`` it
writes the node tape: each proposal's node as a Lemire word, the 53-bit ``random()`` and
``random_sample()`` values as word pairs, and the initial state's wait words.  Replayed here
through the plain-C oracle (and on the device in test_node_tape_gpu.py), the trajectory must
come out identical, proposal by proposal."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G

FIELDS = ("draw", "v", "flags", "cut", "nb", "wait")
STATS = ("steps", "proposals", "draws", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb", "sum_wait")


def record(spec, plan, base, pct, seed, steps, k=2):
    """A recorded native-RNG chain: ``slow_reversible_propose_bi`` (k = 2) or, for k > 2,
    ``slow_reversible_propose`` over the (node, district) pairs (:117-130, :151-153)."""
    from oracle.flipref import NativeRngChain
    (lo, hi), _ = G.population_bounds(int(spec.pop.sum()), k, pct)
    ch = NativeRngChain(spec, plan, base=base, pop_bounds=(lo, hi), seed=seed,
                        log1mp=G.log1mp_table(spec.n, k), record=True, pair=k > 2)
    ch.run(steps)
    return ch


def wrap64(x: int) -> int:
    """A Python int as the int64 the C oracle and the device accumulate it in: k > 2 waits on
    graphs where 1 - p rounds to 1 saturate at 2^62, so their sums wrap."""
    return ((int(x) + (1 << 63)) % (1 << 64)) - (1 << 63)


CASES = {
    # C1: 10x10 grid, lambda = 1 (BASELINE config 1), and the critical base
    "c1_base1": (lambda: G.grid_graph(10, 10), lambda s: G.threshold_plan(s.nodes, 0, 5), 1.0, 0.1, 3000),
    "c1_mu": (lambda: G.grid_graph(10, 10), lambda s: G.threshold_plan(s.nodes, 0, 5), G.SEC11_MU, 0.1, 3000),
    # the reference's own lattices and plans
    "sec11_b08_al2": (G.sec11_graph, lambda s: G.sec11_plan(2, s.nodes), 0.8, 0.1, 1500),
    "sec11_b10_al0_p01": (G.sec11_graph, lambda s: G.sec11_plan(0, s.nodes), 10.0, 0.01, 1500),
    "frank_b03_al1": (G.frank_graph, lambda s: G.frank_plan(1, s.nodes), 0.3, 0.05, 1500),
}


# k > 2: the pair proposal slow_reversible_propose (grid_chain_sec11.py:117-130) -- BASELINE C3
# (sec11, k = 4 quadrants, pop 0.05, base mu), a C4-style triangular lattice (k = 8 strips) and
# a C5-style Delaunay dual (k = 18 bisection, lognormal populations)
PAIR_CASES = {
    "c3_sec11_k4_mu": (G.sec11_graph, lambda s: G.quadrant_plan(s.nodes), 4, G.SEC11_MU, 0.05, 2000),
    "c3_sec11_k4_b05": (G.sec11_graph, lambda s: G.quadrant_plan(s.nodes), 4, 0.5, 0.05, 1500),
    "tri40x78_k8": (lambda: G.triangular_graph(40, 78), lambda s: G.strip_plan(s, 8), 8, 1.0, 0.1, 1200),
    "delaunay2000_k18": (lambda: G.delaunay_graph(2000, seed=0), lambda s: G.bisection_plan(s, 18), 18, 2.0, 0.1,
                         1200),
}


@pytest.fixture(scope="module")
def recorded():
    out = {}
    for name, (mk, plan_of, base, pct, steps) in CASES.items():
        spec = mk()
        plan = plan_of(spec)
        out[name] = (spec, plan, base, pct, steps, record(spec, plan, base, pct, seed=4242 + len(out), steps=steps))
    return out


@pytest.mark.parametrize("name", sorted(CASES))
def test_c_oracle_replays_native_rng_trajectory(recorded, cref, name):
    spec, plan, base, pct, steps, ch = recorded[name]
    tape = ch.node_tape()
    assert tape.size == 6 * ch.stats["proposals"] and ch.stats["steps"] == steps
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), 2, pct)
    a0 = spec.assignment_array(plan, [-1, 1])
    r = cref.run(spec, a0, base=base, pop_lo=lo, pop_hi=hi, seed=0, chain_id=0, n_steps=steps,
                 log1mp=G.log1mp_table(spec.n, 2), tape=tape, trace_cap=len(ch.trace) + 8,
                 wait0_words=np.asarray(ch.wait0_words, dtype=np.uint32))
    exp = ch.trace_array()
    got = r["trace"]
    assert len(got) == len(exp)
    for f in FIELDS:
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, (name, f, bad[:5], got[bad[:3]], exp[bad[:3]])
    for k in STATS:
        assert int(r["stats"][k]) == int(ch.stats[k]), (name, k)
    assert np.array_equal(r["final"], ch.assignment_ids())
    # a real mixture of outcomes, not a degenerate stream
    fl = exp["flags"] & 0xFF
    assert (fl & 2).any() and ((fl & 1) & ~(fl >> 1) & 1).any() or base == 1.0
    assert (fl & 12).any()  # invalid proposals (contiguity or population) are replayed too


@pytest.fixture(scope="module")
def recorded_pair():
    out = {}
    for i, (name, (mk, plan_of, k, base, pct, steps)) in enumerate(sorted(PAIR_CASES.items())):
        spec = mk()
        plan = plan_of(spec)
        out[name] = (spec, plan, k, base, pct, steps, record(spec, plan, base, pct, seed=777 + i, steps=steps, k=k))
    return out


@pytest.mark.parametrize("name", sorted(PAIR_CASES))
def test_c_oracle_replays_native_rng_pair_trajectory(recorded_pair, cref, name):
    """k > 2: ``random.choice(list(pairs))`` over CPython's set order (:128), recorded as a node
    word and a slot word (the district's rank under the state's slot bound), replays through the
    C oracle's canonical PAIR stream proposal by proposal -- node, target district, verdict,
    |cut|, |B|, wait -- with the same final state and tallies."""
    spec, plan, k, base, pct, steps, ch = recorded_pair[name]
    tape = ch.node_tape()
    assert tape.size == 6 * ch.stats["proposals"] and ch.stats["steps"] == steps
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    a0 = spec.assignment_array(plan, list(range(k)))
    r = cref.run(spec, a0, base=base, pop_lo=lo, pop_hi=hi, seed=0, chain_id=0, n_steps=steps, k=k,
                 labels=list(range(k)), proposal=1, log1mp=G.log1mp_table(spec.n, k), tape=tape,
                 trace_cap=len(ch.trace) + 8, wait0_words=np.asarray(ch.wait0_words, dtype=np.uint32))
    exp = ch.trace_array()
    got = r["trace"]
    assert len(got) == len(exp)
    for f in FIELDS:
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, (name, f, bad[:5], got[bad[:3]], exp[bad[:3]])
    for key in STATS:
        assert int(r["stats"][key]) == wrap64(ch.stats[key]), (name, key)
    assert np.array_equal(r["final"], ch.assignment_ids())
    fl = exp["flags"] & 0xFF
    assert (fl & 2).any() and (fl & 12).any()
    # targets: more than one foreign district proposed per node somewhere (a real pair draw)
    tgt = (exp["flags"] >> 8) & 0xFF
    assert len(np.unique(tgt)) == k
    assert any(len(np.unique(tgt[exp["v"] == v])) > 1 for v in np.unique(exp["v"]))


def test_node_words_invert_lemire_and_u53():
    """Every node id has a word the exact Lemire map sends to it without rejection, and every
    53-bit double round-trips through the word pair."""
    from oracle.flipref import NativeRngChain, u53
    for N in (100, 800, 1596, 10100, 32767):
        th = (1 << 32) % N
        for v in (0, 1, N // 2, N - 2, N - 1):
            x0 = (((v + 1) << 32) - 1) // N
            assert (x0 * N) >> 32 == v and ((x0 * N) & 0xFFFFFFFF) >= th
    rng = np.random.RandomState(3)
    for _ in range(1000):
        u = rng.random_sample()
        a, b = NativeRngChain._u53_words(u)
        assert u53(a, b) == u
