"""The product sweep runner (flipcomplexityempirical_amd.sweep): every
configuration of the reference's sweeps (grid_chain_sec11.py:182-184, Frankenstein_chain.py:
182-184) in one device run per graph.

* replica 0 of a configuration writes the same files, byte for byte, as the single-chain
  ``MarkovChain(..., chain_id=i).run().write_outputs`` of that configuration (the reference's
  construction, :299-342);
* the per-configuration sums over replicas equal the sums of the chains' own statistics;
* the sweep's wait.txt values meet the reference-artifact pin (tests/reference_pin.py) -- see
  test_reference_pin_gpu.py, which now runs through this module.
"""
import filecmp
import json
import os

import numpy as np
import pytest

from flipcomplexityempirical_amd import chain as fc
from flipcomplexityempirical_amd import distributed as D
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.sweep import Sweep, sweep_configs

pytestmark = pytest.mark.gpu

SEED = 0x5A
STEPS = 20000


def reference_chain(cfg, chain_id, total_steps, seed):
    """The reference's own construction of one configuration's chain (grid_chain_sec11.py:299-342;
    Frankenstein_chain.py:327-370)."""
    graph = G.sec11_nx() if cfg.graph == "sec11" else G.frank_nx()
    nodes = sorted(graph.nodes())
    plan = (G.sec11_plan if cfg.graph == "sec11" else G.frank_plan)(cfg.alignment, nodes)

    def new_base(partition):
        return cfg.base

    updaters = {"population": fc.Tally("population"), "cut_edges": fc.cut_edges, "b_nodes": fc.b_nodes_bi,
                "base": new_base, "geom": fc.geom_wait}
    part = fc.Partition(graph, assignment=plan, updaters=updaters)
    popbound = fc.within_percent_of_ideal_population(part, cfg.pop)
    return fc.MarkovChain(fc.slow_reversible_propose_bi, fc.Validator([fc.single_flip_contiguous, popbound]),
                          accept=fc.cut_accept, initial_state=part, total_steps=total_steps, seed=seed,
                          chain_id=chain_id)


@pytest.mark.parametrize("graph", ["sec11", "frank"])
def test_sweep_files_equal_single_chain_runs(gpu, tmp_path, graph):
    cfgs = sweep_configs(graph)
    sw = Sweep(graph, replicas=2, total_steps=STEPS, seed=SEED).run()
    out = sw.write_outputs(str(tmp_path / "sweep"))
    assert out["summary"]["configs"][0]["key"] == cfgs[0].key
    frame = "sec11" if graph == "sec11" else "frank"
    shape, offset = ((40, 40), (0, 0)) if graph == "sec11" else ((20, 40), (0, 19))
    # a spread of configurations: every base and population of the sweep appears
    picks = sorted({0, 1, 2, len(cfgs) // 2, len(cfgs) - 1} | set(range(3, len(cfgs), 7)))
    for i in picks:
        res = reference_chain(cfgs[i], i, STEPS, SEED).run(series=True, frame=frame, corrected=True)
        paths = res.write_outputs(str(tmp_path / "single"), cfgs[i].key, shape=shape, offset=offset)
        assert len(paths) == 10  # wait.txt, end2, wca2, flip2, logflip2, edges, rce, rbn, slopes, angles
        for pth in paths:
            other = str(tmp_path / "sweep" / os.path.basename(pth))
            assert filecmp.cmp(pth, other, shallow=False), (cfgs[i].key, os.path.basename(pth))
    # the summary's wait.txt of replica 0 is the file's value
    summ = json.load(open(tmp_path / "sweep" / f"sweep_{graph}.json"))
    for i, c in enumerate(summ["configs"]):
        assert int(open(tmp_path / "sweep" / (c["key"] + "wait.txt")).read()) == c["wait_txt"][0]
    sw.close()


def test_sweep_grouped_sums_over_replicas(gpu):
    R = 3
    sw = Sweep("frank", replicas=R, total_steps=5000, seed=SEED + 1, series=False, corrected=False).run()
    st = sw._run.stats()
    red = sw.grouped()
    nc = sw.n_configs
    for j, f in enumerate(D.AGG_FIELDS):
        per = np.asarray(st[f], dtype=np.int64).reshape(R, nc).sum(axis=0)
        assert np.array_equal(red["scalars"][:, j], per), f
    # every yield of every replica is in its configuration's |cut| histogram
    assert np.array_equal(red["cut_hist"].sum(axis=1), np.full(nc, R * 5000))
    assert np.array_equal(red["chain_sum_wait"], np.asarray(st["sum_wait"]).reshape(R, nc))
    ch, _ = sw._run.hist()
    assert np.array_equal(red["cut_hist"], ch.reshape(R, nc, -1).sum(axis=0))
    nf, ps, lf = sw._run.flips()
    assert np.array_equal(red["last_flipped"], lf.reshape(R, nc, -1).max(axis=0))
    assert np.array_equal(red["part_sum"], ps.reshape(R, nc, -1).sum(axis=0))
    sw.close()


def test_sweep_subset_and_errors(gpu):
    cfgs = sweep_configs("sec11")
    assert len(cfgs) == 150 and len(sweep_configs("frank")) == 24
    assert cfgs[0].key == "2B10P1"  # pops outermost, then bases, alignments 2, 1, 0 (:182-184)
    with pytest.raises(ValueError):
        Sweep("sec11", configs=[sweep_configs("frank")[0]])
    with pytest.raises(ValueError):
        Sweep("nope")
    sw = Sweep("sec11", configs=cfgs[:4], replicas=1, total_steps=1000, seed=3, series=False).run()
    res = sw.results()
    assert sorted(res) == [0, 1, 2, 3]
    assert all(r.steps == 999 for r in res.values())
    sw.close()
