"""The reference's configuration sweeps as one device run per graph (SURVEY §8(b) callers).

The reference runs one 100,000-step chain per configuration, one after another
(``grid_chain_sec11.py:182-184``: 5 population tolerances x 10 bases x 3 start alignments = 150
configurations; ``Frankenstein_chain.py:182-184``: 4 x 2 x 3 = 24), and leaves per configuration
``{alignment}B{int(100 base)}P{int(100 pop)}`` files: ``wait.txt`` (``:410-411``) and the plotted
data (``:427-528``: cut_times per edge, the end state, part_sum, slopes / angles, num_flips,
lognum_flips).  Here every configuration of a graph -- times ``replicas`` independent chains
-- is one ``fc_run`` (per-chain bases and population bounds, ``fc_params.chain_pop_bounds``),
so the whole sweep is one launch per graph instead of 150 sequential chains on one CPU thread.

Chain g (global id) runs configuration ``g % n_configs`` as replica ``g // n_configs``, with the
Philox key (seed, g): replica 0 of configuration i is bit for bit
``chain.MarkovChain(..., seed=seed, chain_id=i).run()`` of that configuration, and its output
files are byte-identical to that chain's ``ChainResult.write_outputs`` (both go through
``ChainResult.from_arrays``).  Over N ranks the chains shard by global id (weak or strong, as the
caller sizes it); each rank writes the files of the replica-0 chains it owns, and the per
configuration sums over all replicas (``distributed.local_statistics`` /
``allreduce_statistics``: one SUM and one MAX all-reduce) are written beside them by rank 0.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from . import distributed as D
from . import graphs as G


@dataclass(frozen=True)
class SweepConfig:
    graph: str        # "sec11" or "frank"
    alignment: int    # start plan (grid_chain_sec11.py:195-214; Frankenstein_chain.py:207-246)
    base: float       # cut_accept base (:34)
    pop: float        # population tolerance (:36)

    @property
    def key(self) -> str:
        """The reference's file prefix (``grid_chain_sec11.py:323,410``)."""
        return f"{self.alignment}B{int(100 * self.base)}P{int(100 * self.pop)}"


def sweep_configs(graph: str) -> List[SweepConfig]:
    """The configurations of one reference sweep in its loop order (``for pop1 in pops: for base
    in bases: for alignment in [2, 1, 0]``, ``grid_chain_sec11.py:182-184``)."""
    if graph == "sec11":
        pops, bases = G.SEC11_POPS, G.SEC11_BASES
    elif graph == "frank":
        pops, bases = G.FRANK_POPS, G.FRANK_BASES
    else:
        raise ValueError(f"unknown sweep graph {graph!r} (sec11, frank)")
    return [SweepConfig(graph, al, b, p) for p in pops for b in bases for al in (2, 1, 0)]


# heatmap layout of the A2 arrays (grid_chain_sec11.py:440-446; Frankenstein_chain.py:468-474)
HEATMAP = {"sec11": ((40, 40), (0, 0)), "frank": ((20, 40), (0, 19))}


class _Cspec:
    """What ChainResult.from_arrays reads of a compiled chain (spec, labels)."""

    def __init__(self, spec, labels):
        self.spec, self.labels = spec, labels


class Sweep:
    """All configurations of one reference sweep (``graph`` = "sec11" / "frank") x ``replicas``
    chains on the device.  ``configs`` (optional) restricts the sweep to some of them.

    ``series``: keep the per-yield lists (``rce`` / ``rbn``, slopes / angles) through the device
    event log, as ``MarkovChain.run(series=True)`` does; ``corrected``: the corrected tallies
    beside the reference's quirky ones (FC_DIAG_FLIPS_EXACT, Rao-Blackwellised waits)."""

    def __init__(self, graph: str = "sec11", replicas: int = 1, total_steps: int = 100000, seed: int = 0,
                 device: int = 0, series: bool = True, corrected: bool = True,
                 configs: Optional[Sequence[SweepConfig]] = None, dist=None, dist_device=None,
                 force_collective: bool = False):
        self.graph = graph
        self.configs = list(configs) if configs is not None else sweep_configs(graph)
        if not self.configs or any(c.graph != graph for c in self.configs):
            raise ValueError("configs must be non-empty and all of the sweep's graph")
        if replicas < 1 or total_steps < 1:
            raise ValueError("replicas and total_steps must be >= 1")
        self.replicas, self.total_steps, self.seed = int(replicas), int(total_steps), int(seed)
        self.series, self.corrected = bool(series), bool(corrected)
        self.dist, self.dist_device = dist, dist_device
        self.force_collective = bool(force_collective)  # collectives even at world size 1
        self.world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.spec = G.sec11_graph() if graph == "sec11" else G.frank_graph()
        self.labels = [-1, 1]
        self.n_configs = len(self.configs)
        self.n_total = self.n_configs * self.replicas
        self.offset, self.count = D.shard(self.n_total, self.world, self.rank)
        self.gids = np.arange(self.offset, self.offset + self.count, dtype=np.int64)
        self.device = device
        self.timing: Dict[str, float] = {}
        self._run = None
        self._graph = None

    def config_of(self, g: int) -> SweepConfig:
        return self.configs[int(g) % self.n_configs]

    # ---- run ----------------------------------------------------------------------------
    def run(self) -> "Sweep":
        """Every chain of this rank's shard for ``total_steps`` yields (one launch)."""
        from .engine import FlipGraph, FlipRun, RunConfig
        if self.count == 0:
            return self
        sp = self.spec
        plans = {al: sp.assignment_array((G.sec11_plan if self.graph == "sec11" else G.frank_plan)(al, sp.nodes),
                                         self.labels) for al in (0, 1, 2)}
        cfgs = [self.config_of(g) for g in self.gids]
        inits = np.stack([plans[c.alignment] for c in cfgs])
        bases = np.asarray([c.base for c in cfgs], dtype=np.float64)
        bounds = np.asarray([G.population_bounds(int(sp.pop.sum()), 2, c.pop)[1] for c in cfgs], dtype=np.int64)
        diag = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS
        if self.series:
            diag |= _lib.FC_DIAG_SERIES
        if self.corrected:
            diag |= _lib.FC_DIAG_FLIPS_EXACT
        t0 = time.perf_counter()
        self._graph = FlipGraph(sp)
        cfg = RunConfig(seed=self.seed, chain_id_offset=int(self.offset), device=self.device, diag_mask=diag,
                        labels=tuple(self.labels), event_cap=self.total_steps if self.series else 0,
                        pop_lo=int(bounds[:, 0].min()), pop_hi=int(bounds[:, 1].max()))
        self._run = FlipRun(self._graph, inits, cfg, bases=bases, pop_bounds=bounds)
        t1 = time.perf_counter()
        if self.total_steps > 1:
            self._run.steps(self.total_steps - 1)
        self._run.sync()
        t2 = time.perf_counter()
        self.timing.update(setup_s=t1 - t0, device_s=t2 - t1, kernel_ms=float(self._run.last_ms()))
        self.kernel_name = self._run.kernel_name()
        return self

    # ---- results ------------------------------------------------------------------------
    def results(self, chains: Optional[Sequence[int]] = None) -> Dict[int, "object"]:
        """``ChainResult`` per global chain id of this rank (default: its replica-0 chains),
        read from the device once for all of them."""
        from .chain import ChainResult
        if self._run is None:
            raise RuntimeError("Sweep.run() first")
        t0 = time.perf_counter()
        want = [int(g) for g in (chains if chains is not None else self.gids[self.gids < self.n_configs])]
        run, sp = self._run, self.spec
        st = run.stats()
        ch, nh = run.hist()
        ct = run.cut_times()
        nf, ps, lf = run.flips()
        fin = run.state()
        ex = run.flips_exact() if self.corrected else None
        wexp = run.wait_expected() if self.corrected else None
        edges = sp.edges()
        cs = _Cspec(sp, self.labels)
        frame = G.slope_frame(sp, self.graph) if self.series else None
        chg = run.frame_series_changes(frame) if self.series else None
        out = {}
        for g in want:
            c = g - self.offset
            if not 0 <= c < self.count:
                raise ValueError(f"chain {g} is not on this rank")
            res = ChainResult.from_arrays(cs, edges, st, ch, nh, ct, nf, ps, lf, fin, c)
            if self.corrected:
                res.flip_count = {sp.nodes[i]: int(ex[0][c, i]) for i in range(sp.n)}
                res.occupancy = {sp.nodes[i]: int(ex[1][c, i]) for i in range(sp.n)}
                res.last_accept = {sp.nodes[i]: int(ex[2][c, i]) for i in range(sp.n)}
                res.waits_expected = float(wexp[c])
            if self.series:
                res.rce = run.yield_values("cut", c)
                res.rbn = run.yield_values("nb", c)
                res.slopes = run.changes_to_yields(chg, c, c, "slope")
                res.angles = run.changes_to_yields(chg, c, c, "angle")
            out[g] = res
        self.timing["results_s"] = self.timing.get("results_s", 0.0) + time.perf_counter() - t0
        return out

    def grouped(self) -> Dict[str, np.ndarray]:
        """Per-configuration sums over all replicas on all ranks (``[n_configs, ...]``: scalars
        by ``distributed.AGG_FIELDS``, |cut| / |B| histograms, cut_times, num_flips, part_sum;
        last_flipped by MAX), plus ``sum_wait`` / final ``cut`` / ``nb`` of every chain
        ``[replicas, n_configs]``."""
        run = self._run
        st = run.stats() if run is not None else None
        arrays = {}
        if run is not None:
            arrays["cut_hist"], arrays["nb_hist"] = run.hist()
            arrays["cut_times"] = run.cut_times()
            arrays["num_flips"], arrays["part_sum"], arrays["last_flipped"] = run.flips()
        else:  # a rank without chains still joins the collective with zero rows
            E, n = self.spec.n_edges, self.spec.n
            st = {f: np.zeros(0, dtype=np.int64) for f in D.AGG_FIELDS}
            arrays = {"cut_hist": np.zeros((0, E + 1)), "nb_hist": np.zeros((0, n + 1)),
                      "cut_times": np.zeros((0, E)), "num_flips": np.zeros((0, n)), "part_sum": np.zeros((0, n)),
                      "last_flipped": np.zeros((0, n))}
        groups = self.gids % self.n_configs
        red = D.allreduce_statistics(D.local_statistics(st, groups, self.n_configs, arrays), self.dist,
                                     self.dist_device, force=self.force_collective)
        per_chain = np.zeros((3, self.n_total), dtype=np.int64)
        if run is not None:
            per_chain[:, self.offset:self.offset + self.count] = (st["sum_wait"], st["cut"], st["nb"])
        per_chain = D.allreduce_sum(per_chain, self.dist, self.dist_device, force=self.force_collective)
        shape = (self.replicas, self.n_configs)
        red["chain_sum_wait"] = per_chain[0].reshape(shape)
        red["chain_cut"] = per_chain[1].reshape(shape)
        red["chain_nb"] = per_chain[2].reshape(shape)
        return red

    # ---- outputs ------------------------------------------------------------------------
    def write_outputs(self, directory: str) -> Dict[str, object]:
        """Each configuration's reference file set for its replica-0 chain (the rank that owns
        it writes it: ``ChainResult.write_outputs``), then, by rank 0, ``{prefix}replicas.npz``
        per configuration with the sums over all replicas and ``sweep_{graph}.json`` (the
        configuration table, every chain's wait.txt value, timings)."""
        t0 = time.perf_counter()
        shape, offset = HEATMAP[self.graph]
        written = 0
        res = self.results() if self._run is not None else {}
        for g, r in res.items():
            written += len(r.write_outputs(directory, self.config_of(g).key, shape=shape, offset=offset))
        t1 = time.perf_counter()
        red = self.grouped()
        t2 = time.perf_counter()
        summary = None
        if self.rank == 0:
            os.makedirs(directory, exist_ok=True)
            for i, c in enumerate(self.configs):
                np.savez(os.path.join(directory, c.key + "replicas.npz"),
                         scalars=red["scalars"][i], fields=np.asarray(D.AGG_FIELDS),
                         cut_hist=red["cut_hist"][i], nb_hist=red["nb_hist"][i], cut_times=red["cut_times"][i],
                         num_flips=red["num_flips"][i], part_sum=red["part_sum"][i],
                         last_flipped=red["last_flipped"][i], wait_txt=red["chain_sum_wait"][:, i],
                         final_cut=red["chain_cut"][:, i], final_nb=red["chain_nb"][:, i])
                written += 1
            summary = {"graph": self.graph, "replicas": self.replicas, "total_steps": self.total_steps,
                       "seed": self.seed, "ranks": self.world, "kernel": getattr(self, "kernel_name", None),
                       "configs": [{"key": c.key, "alignment": c.alignment, "base": c.base, "pop": c.pop,
                                    "wait_txt": [int(x) for x in red["chain_sum_wait"][:, i]]}
                                   for i, c in enumerate(self.configs)],
                       "timing": dict(self.timing, write_s=t1 - t0, reduce_s=t2 - t1)}
            with open(os.path.join(directory, f"sweep_{self.graph}.json"), "w") as f:
                json.dump(summary, f, indent=1)
            written += 1
        self.timing.update(write_s=t1 - t0, reduce_s=t2 - t1)
        return {"files": written, "summary": summary}

    def close(self):
        if self._run is not None:
            self._run.close()
            self._run = None
        if self._graph is not None:
            self._graph.close()
            self._graph = None


def run_reference_sweeps(directory: str, graphs: Sequence[str] = ("sec11", "frank"), replicas: int = 1,
                         total_steps: int = 100000, seed: int = 0, device: int = 0, dist=None,
                         dist_device=None) -> Dict[str, Dict[str, object]]:
    """Both reference sweeps (174 configurations), written under ``directory/<graph>/``."""
    out = {}
    for gname in graphs:
        sw = Sweep(gname, replicas=replicas, total_steps=total_steps, seed=seed, device=device, dist=dist,
                   dist_device=dist_device).run()
        out[gname] = sw.write_outputs(os.path.join(directory, gname))
        out[gname]["timing"] = dict(sw.timing)
        sw.close()
    return out


def main(argv=None):
    """``python -m flipcomplexityempirical_amd.sweep OUTDIR [--replicas R] [--steps T]``: the
    reference's sweeps on the device (one rank; under torch.distributed.run one per GPU)."""
    import argparse
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("outdir")
    ap.add_argument("--graphs", default="sec11,frank")
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100000, help="total_steps (yields incl. the start, :342)")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    dist, dev, local = None, None, int(os.environ.get("LOCAL_RANK", "0"))
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        import torch.distributed as tdist
        # FC_BENCH_BACKEND / FC_BENCH_DEVICE: rehearsal of several ranks on one GPU over gloo
        # (as bench.py); the real run is RCCL, one GPU per rank
        backend = os.environ.get("FC_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        local = int(os.environ.get("FC_BENCH_DEVICE", local))
        tdist.init_process_group(backend=backend)
        dist = tdist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dev = torch.device("cuda", local)
    out = run_reference_sweeps(args.outdir, [g for g in args.graphs.split(",") if g], args.replicas, args.steps,
                               args.seed, local, dist, dev)
    if dist is None or dist.get_rank() == 0:
        print(json.dumps({g: {"files": o["files"], "timing": o["timing"]} for g, o in out.items()}))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
