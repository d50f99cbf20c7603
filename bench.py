#!/usr/bin/env python3
"""Headline benchmark: flip proposals/s on the 40x40 sec11 grid, k = 2 (BASELINE.json).

``--workload`` selects another BASELINE config for side measurements (never the headline
line): c3 (sec11, k=4 pair proposals, 8192 chains/GPU), c4 (triangular 100x198, k=8),
c5 (Delaunay 10k nodes, k=18).  The default, c2, is the line the driver records.

Workload (BASELINE config C2, the largest single-GPU configuration of the metric):
the exact sec11 graph of ``grid_chain_sec11.py:186-260`` (N = 1596, E = 3116), 4096
independent chains per GPU, chain c (global id g) with base ``bases[g % 10]``
(``grid_chain_sec11.py:34``), start plan alignment ``(g // 10) % 3`` (``:195-214``),
population tolerance 0.1 (``:319``), Philox seed 0x5EED0002.  One bench "step" is one
launch advancing every chain by ``--chain-steps`` valid steps (default 100,000 = one whole
reference run, ``total_steps=100000`` at ``grid_chain_sec11.py:342``; 10 timed steps = the
1e6 steps per chain of BASELINE config C2).  Inputs are resident in HBM before the
timed region; the timed region is bracketed by barrier + device synchronisation.

N > 1: one process per GPU, chains sharded by global id with no data-path collective (weak
scaling); one RCCL all-reduce of the statistics at the end.  Under ``torch.distributed.run``
the ranks come from the environment and ``--gpus`` must equal ``WORLD_SIZE``; run directly
(``python bench.py --gpus N``) the script launches the N ranks itself, before any GPU call, and
exits with the first failing rank's status.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "flip proposals/sec (node) 40x40 grid k=2, 1/2/4/8 MI355X; % LDS/HBM roofline"
SEED = 0x5EED0002
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md chip-level parameters (spec)
LDS_PEAK_B128_GBS = 150000.0    # MI355X_MICROARCH.md §LDS: ~150 TB/s ds_read_b64/b128 aggregate
LDS_CUS, LDS_CLK_GHZ = 256, 2.4
# MI355X_MICROARCH.md §LDS, bytes per clock per CU by access width (one wave instruction of 64
# lanes): ds_read_u8 / u16 / b32 move 64 / 128 / 256 B in 2 LDS cycles; ds_write_b8 / b16 / b32
# move 64 / 128 / 256 B in 4 (a store's address and data transfer, 2 cycles per source dword)
LDS_READ_BPC = {1: 32.0, 2: 64.0, 4: 128.0}
LDS_WRITE_BPC = {1: 16.0, 2: 32.0, 4: 64.0}
# The chain state is LDS-resident (C1-C4 are LDS-bound; HBM only carries the
# per-launch state load / store), so the roofline is priced against the LDS aggregate -- at the
# rate of the access widths the algorithmic bytes come in (the path gathers bytes and dwords,
# not b128 rows: VERDICT r02 item 8), with the b128 aggregate kept beside it.
# Algorithmic bytes: per proposal R = 2 + 1 + 8 + 5*deg + 5*L + 8 and per
# accepted proposal W = 1 + 8 + 4*(deg+1) + 4 with deg = 4, L = 4 (sec11 interior).
MU_TRI = 4.150797226                         # connective constant of the triangular lattice


def r_mix(deg: float, ring_extra: float, extra4: float = 0.0) -> dict:
    """SURVEY §8(d) R by access width: boundary-list entry (2 B), a[v] (1 B), row_ptr pair (2 x
    4 B), per neighbour / ring cell col_idx (4 B) + a[] (1 B), two district pops (2 x 4 B), plus
    ``extra4`` bytes of further 4-byte reads (C3: k pops compared)."""
    return {2: 2.0, 1: 1.0 + deg + ring_extra, 4: 8.0 + 4 * deg + 4 * ring_extra + 8.0 + extra4}


def w_mix(deg: float) -> dict:
    """SURVEY §8(d) W by access width: a[v] (1 B), two pops, the boundary entries of v and its
    neighbours and the cut count (4 B each)."""
    return {1: 1.0, 4: 8.0 + 4 * (deg + 1) + 4.0}


def lds_mix_peak_gbs(rmix: dict, wmix: dict, acc_per_prop: float) -> float:
    """Aggregate LDS rate (GB/s) of the algorithmic byte mix: bytes per proposal over the LDS
    cycles the same accesses take at MI355X_MICROARCH.md's per-width rates, times 256 CUs at
    2.4 GHz."""
    byts = sum(rmix.values()) + acc_per_prop * sum(wmix.values())
    cyc = sum(b / LDS_READ_BPC[w] for w, b in rmix.items()) + acc_per_prop * sum(b / LDS_WRITE_BPC[w]
                                                                                  for w, b in wmix.items())
    return byts / cyc * LDS_CUS * LDS_CLK_GHZ


R_MIX, W_MIX = r_mix(4, 4), w_mix(4)
R_BYTES, W_BYTES = sum(R_MIX.values()), sum(W_MIX.values())   # 59, 33
L2_PEAK_GBS = 34500.0   # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate (4 MiB per XCD)


def r_split(deg: float, ring_extra: float, extra4: float = 0.0):
    """SURVEY §8(d)'s R split by where the bytes live on this implementation: the LDS-resident
    chain state (boundary entry, a[v], a[] of the neighbours and ring cells, the district
    populations; by access width) and the global node records every chain shares through L1 / L2
    (row_ptr pair, col_idx and ring indices: NodeRec, fc_device.h)."""
    lds = {2: 2.0, 1: 1.0 + deg + ring_extra, 4: 8.0 + extra4}
    glob = 8.0 + 4 * deg + 4 * ring_extra
    return lds, glob


def roofline_levels(W, props: float, acc: float, kernel_ms: float, traffic=None) -> dict:
    """Per-level roofline of one launch: the LDS-resident bytes against the
    LDS aggregate at their access-width mix, the global node-record bytes against the L2
    aggregate, the measured HBM bytes against HBM; ``bound`` = the level with the largest
    fraction."""
    t = kernel_ms * 1e-3
    acc_pp = acc / props if props else 0.0
    lds_b = sum(W.lds_mix.values()) * props + W.W * acc
    lds_peak = lds_mix_peak_gbs(W.lds_mix, W.wmix, acc_pp)
    glob_b = W.glob_bytes * props
    out = {"lds": {"bytes": lds_b, "achieved": lds_b / t / 1e9, "peak": lds_peak,
                   "frac": lds_b / t / 1e9 / lds_peak,
                   "per_proposal": W.lds_mix, "per_accept": W.W},
           "l2": {"bytes": glob_b, "achieved": glob_b / t / 1e9, "peak": L2_PEAK_GBS,
                  "frac": glob_b / t / 1e9 / L2_PEAK_GBS, "per_proposal": W.glob_bytes},
           "hbm": {"bytes": traffic, "achieved": traffic / t / 1e9 if traffic else None, "peak": HBM_PEAK_GBS,
                   "frac": traffic / t / 1e9 / HBM_PEAK_GBS if traffic else None}}
    out["bound"] = max((k for k in ("lds", "l2", "hbm") if out[k]["frac"] is not None), key=lambda k: out[k]["frac"])
    return out


class Workload:
    """One BASELINE config: graph, start plan and base of global chain g, bounds."""

    def __init__(self, name: str):
        from flipcomplexityempirical_amd import graphs as G
        from flipcomplexityempirical_amd import _lib
        self.name = name
        if name == "c2":
            self.spec = G.sec11_graph()
            self.k, self.pct, self.proposal, self.labels = 2, 0.1, _lib.FC_PROPOSE_BI_SIGN, [-1, 1]
            self.bases = list(G.SEC11_BASES)
            self._plans = [self.spec.assignment_array(G.sec11_plan(al, self.spec.nodes), [-1, 1]) for al in range(3)]
            self.plan_of = lambda g: (g // 10) % 3
            self.chains = 4096
            self.rmix, self.wmix = R_MIX, W_MIX
            # chain g runs configuration g % 30 of the sweep: base bases[g % 10], alignment (g // 10) % 3
            self.n_groups = 30
            self.group_desc = [{"base": self.bases[i % 10], "alignment": (i // 10) % 3} for i in range(30)]
            self.desc = ("C2: sec11 40x40 grid (N=1596, E=3116), k=2, 4096 chains/GPU, base bases[g%10], "
                         "alignment (g//10)%3, pop tol 0.1, seed 0x5EED0002")
            self.data = "synthetic: the reference's sec11 lattice (grid_chain_sec11.py:186-260) and start plans, Philox stream"
        elif name == "c3":
            self.spec = G.sec11_graph()
            self.k, self.pct, self.proposal, self.labels = 4, 0.05, _lib.FC_PROPOSE_PAIR, [0, 1, 2, 3]
            self.bases = [G.SEC11_MU]
            self._plans = [self.spec.assignment_array(G.quadrant_plan(self.spec.nodes), self.labels)]
            self.plan_of = lambda g: 0
            self.chains = 8192
            self.rmix, self.wmix = r_mix(4, 4, extra4=8), W_MIX   # k pops compared: two more int32 reads
            self.desc = "C3: sec11 40x40, k=4 quadrant plan, pair proposals, pop tol 0.05, base mu, 8192 chains/GPU"
            self.data = ("synthetic: the reference's sec11 lattice (grid_chain_sec11.py:186-260) with a k = 4 "
                         "quadrant plan, Philox stream")
        elif name == "c4":
            self.spec = G.triangular_graph(100, 198)
            self.k, self.pct, self.proposal = 8, 0.1, _lib.FC_PROPOSE_PAIR
            self.labels = list(range(8))
            self.bases = [1 / MU_TRI, 1.0, MU_TRI]
            self._plans = [self.spec.assignment_array(G.strip_plan(self.spec, 8), self.labels)]
            self.plan_of = lambda g: 0
            self.chains = 2048  # bench sizes it to the resident capacity (resident_chains)
            self.rmix, self.wmix = r_mix(6, 0), w_mix(6)
            self.data = ("synthetic: networkx triangular_lattice_graph(100, 198) with unit populations and a k = 8 "
                         "vertical-strip plan (BASELINE config 4), Philox stream")
            self.desc = (f"C4: triangular lattice 100x198 (N={self.spec.n}), k=8 vertical strips, pair proposals, "
                         "pop tol 0.1, base in {1/mu_tri, 1, mu_tri}, one wave of resident chains per GPU")
        elif name == "c5":
            self.spec = G.delaunay_graph(10000, seed=0)
            self.k, self.pct, self.proposal = 18, 0.1, _lib.FC_PROPOSE_PAIR
            self.labels = list(range(18))
            self.bases = [0.5, 1.0, 2.0]
            self._plans = [self.spec.assignment_array(G.bisection_plan(self.spec, 18), self.labels)]
            self.plan_of = lambda g: 0
            self.chains = 2048
            d = float(self.spec.degree().mean())
            self.rmix, self.wmix = r_mix(d, 0), w_mix(d)
            self.data = ("synthetic: Delaunay dual of 10^4 uniform points (scipy, seed 0), lognormal(0, 0.5) "
                         "populations, k = 18 recursive-bisection plan (BASELINE config 5), Philox stream")
            self.desc = ("C5: Delaunay dual of 10^4 uniform points (E=%d), lognormal pops, k=18 bisection plan, "
                         "pair proposals, pop tol 0.1, base in {0.5, 1, 2}, one wave of resident chains per GPU"
                         % self.spec.n_edges)
        else:
            raise ValueError(f"unknown workload {name}")
        self.lds_mix, self.glob_bytes = {"c2": r_split(4, 4), "c3": r_split(4, 4, extra4=8), "c4": r_split(6, 0)}.get(
            name) or r_split(float(self.spec.degree().mean()), 0)
        self.seed = SEED + {"c2": 0, "c3": 1, "c4": 2, "c5": 3}[name]
        self.R, self.W = sum(self.rmix.values()), sum(self.wmix.values())
        if name != "c2":  # one configuration per base
            self.n_groups = len(self.bases)
            self.group_desc = [{"base": b} for b in self.bases]

    def group_of(self, gids):
        """Configuration (group) id of global chains ``gids``: chain g runs configuration
        g % n_groups (C2: base bases[g % 10] and alignment (g // 10) % 3 are both fixed by g % 30)."""
        return np.asarray(gids, dtype=np.int64) % self.n_groups

    def base_of(self, g):
        return self.bases[g % len(self.bases)]

    def init_of(self, g):
        return self._plans[self.plan_of(g)]


LDS_GRANULE = 1280  # measured: a workgroup's LDS is allocated in 1280 B steps (C4, 12,944 B per chain:
                   # 11 one-wave workgroups per CU are resident, a 12th waits: 41.1 against 55.5 ms;
                   # C5 at 13,872 B holds 11 per CU, at 14,128 B only 10: 56.5 against 77.0 ms.
                   # 2048 B fits the first, not the second; 1280 B = 160 KiB / 128 fits both)


def resident_chains(fg, W, device: int = 0, flags: int = 0, tune=None) -> int:
    """Chains one GPU holds at once for workload W: CUs x min(LDS / chain LDS, 16 waves), the
    chain's LDS rounded up to the allocation granule."""
    import torch
    from flipcomplexityempirical_amd import graphs as G
    from flipcomplexityempirical_amd.engine import FlipRun, RunConfig
    _, (lo, hi) = G.population_bounds(int(W.spec.pop.sum()), W.k, W.pct)
    probe = FlipRun(fg, W.init_of(0)[None, :], RunConfig(k=W.k, labels=tuple(W.labels), proposal=W.proposal,
                                                         pop_lo=lo, pop_hi=hi, device=device, flags=flags, tune=tune))
    lds = probe.chain_lds_bytes()
    probe.close()
    cus = torch.cuda.get_device_properties(device).multi_processor_count if torch.cuda.is_available() else 256
    lds = -(-lds // LDS_GRANULE) * LDS_GRANULE
    return cus * max(1, min(160 * 1024 // lds, 16))


def measured_traffic(wname: str, kname: str, chains: int, chain_steps: int, root: str = ROOT, build_id: str = ""):
    """HBM bytes per launch of this kernel at this launch shape, from the separate rocprofv3
    FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md HBM section: (2 FETCH_SIZE + WRITE_SIZE)
    KiB): profiles/pmc_traffic.json for C2, the newest profiles/r*_side_pmc_<workload>.json for the
    k > 2 side lines.  A kernel name does not identify a revision, so a summary counts only when
    it records this run's library build id (as measured_l2).  Returns (bytes, profile,
    stale) -- (None, None, stale) when none matches, ``stale`` naming the newest summary of the
    same kernel and shape that was refused for its build id (or None)."""
    prof = os.path.join(root, "profiles")
    files = [os.path.join(prof, "pmc_traffic.json")] if wname == "c2" else \
        sorted(glob.glob(os.path.join(prof, f"r*_side_pmc_{wname}.json")), reverse=True)
    stale = None
    for fn in files:
        try:
            tj = json.load(open(fn))
        except (OSError, ValueError):
            continue
        if (tj.get("chains") == chains and tj.get("chain_steps") == chain_steps
                and tj.get("workload", "c2") == wname and kname in str(tj.get("kernel"))
                and tj.get("hbm_bytes_per_launch")):
            if build_id and tj.get("build_id") == build_id:
                return tj["hbm_bytes_per_launch"], "profiles/" + os.path.basename(fn), None
            if stale is None:
                stale = {"profile": "profiles/" + os.path.basename(fn), "build_id": tj.get("build_id"),
                         "hbm_bytes_per_launch": tj["hbm_bytes_per_launch"]}
    return None, None, stale


def measured_l2(wname: str, kname: str, chains: int, chain_steps: int, kernel_ms: float, build_id: str = ""):
    """The newest committed L1 / L2 counter summary of this workload's kernel at this launch shape
    (profiles/*_<workload>_l1l2.json, tools/gpu_cache_pmc.sh), rescaled to this run's launch time:
    L2 requests per launch priced at a 128-B line (an upper bound), hit rates, wave-state shares.
    The kernel name does not identify a kernel revision, so a summary counts only when it records
    the library build id (fc_build_id) of this run; else None (stale counters are not reported)."""
    import glob as _glob
    best = None
    for fn in sorted(_glob.glob(os.path.join(ROOT, "profiles", f"*_{wname}_l1l2.json"))):
        try:
            j = json.load(open(fn))
        except (OSError, ValueError):
            continue
        if (j.get("kernel") == kname and j.get("chains") == chains and j.get("chain_steps") == chain_steps
                and build_id and j.get("build_id") == build_id):
            best = (fn, j)
    if best is None:
        return None
    fn, j = best
    m = j["measured"]
    b = m.get("l2_bytes_upper")
    return {"profile": os.path.relpath(fn, ROOT), "l2_bytes_upper_per_launch": b,
            "l2_frac_upper": b / (kernel_ms * 1e-3) / 1e9 / L2_PEAK_GBS if b else None,
            "tcc_hit_rate": m.get("tcc_hit_rate"), "l1_hit_rate_est": m.get("l1_hit_rate_est"),
            "wait_any_frac": m.get("wait_any_frac"), "active_inst_any_frac": m.get("active_inst_any_frac")}


def sweep_leg(replicas: int, device: int) -> dict:
    """Side line: the reference's experiment as it is run (grid_chain_sec11.py:182-528,
    Frankenstein_chain.py:182-556) -- both sweeps, 174 configurations x ``replicas`` chains of
    100,000 yields, one launch per graph, every configuration's output set written (wait.txt, the
    heatmap arrays, cut_times, the per-yield rce / rbn / slope / angle lists) into a scratch
    directory that is removed afterwards.  Wall time from construction to the last file."""
    import shutil
    import tempfile
    from flipcomplexityempirical_amd import sweep as SW
    tmp = tempfile.mkdtemp(prefix="fc_sweep_")
    try:
        t0 = time.perf_counter()
        res = SW.run_reference_sweeps(tmp, replicas=replicas, device=device)
        wall = time.perf_counter() - t0
        nbytes = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(tmp) for f in fs)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    cfgs = sum(len(SW.sweep_configs(g)) for g in res)
    return {"configurations": cfgs, "replicas": replicas, "yields_per_chain": 100000, "wall_s": wall,
            "files": sum(r["files"] for r in res.values()), "bytes_written": nbytes,
            "per_graph": {g: {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r["timing"].items()}
                          for g, r in res.items()},
            "note": "flipcomplexityempirical_amd.sweep.run_reference_sweeps: one fc_run per graph (per-chain bases "
                    "and population bounds), full diagnostics + event log + corrected tallies, every "
                    "configuration's files written by ChainResult.write_outputs (the reference runs the 174 "
                    "configurations one after another on one CPU thread)"}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return int(so.getsockname()[1])


def launch_ranks(gpus: int) -> int:
    """``python bench.py --gpus N`` without a launcher: start N ranks of this script (one
    process per GPU, ``RANK`` = ``LOCAL_RANK`` = r, rendezvous on 127.0.0.1) and wait for them.
    Runs before anything touches the GPU (the parent never does); a rank that fails ends the
    others (their exact PIDs), and the first failing status is returned.  Rank 0 prints the
    line."""
    import signal
    import subprocess
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []

    def _term(signum, frame):  # a scheduler that signals only this PID: end the ranks too
        raise KeyboardInterrupt(f"signal {signum}")
    old_term = signal.signal(signal.SIGTERM, _term)
    status = 0
    try:
        for r in range(gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FC_BENCH_LAUNCHER="bench.py")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
        live = list(procs)
        while live:
            time.sleep(0.2)
            for pr in list(live):
                rc = pr.poll()
                if rc is None:
                    continue
                live.remove(pr)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    for other in live:
                        other.terminate()
    finally:
        # however this loop ends (a failed rank, SIGTERM, KeyboardInterrupt), no rank outlives
        # the launcher: terminate the live ones (their exact PIDs), then reap every child
        for pr in procs:
            if pr.poll() is None:
                pr.terminate()
        for pr in procs:
            try:
                pr.wait(timeout=30)
            except subprocess.TimeoutExpired:
                pr.kill()
                pr.wait()
        signal.signal(signal.SIGTERM, old_term)
    return status


def check_world(gpus: int):
    """``--gpus`` against the launcher's ``WORLD_SIZE``: None when they agree (or no launcher
    is involved), else the message to exit with."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != gpus:
        return f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}: the launcher and the request disagree"
    return None


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return None, 0, 1, int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # FC_BENCH_BACKEND / FC_BENCH_DEVICE only serve rehearsals of the N > 1 path on a
    # one-GPU box (several ranks on device 0 over gloo); the real run uses RCCL, one GPU per rank.
    backend = os.environ.get("FC_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    local = int(os.environ.get("FC_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:
        raise SystemExit(f"bench.py: rank {os.environ.get('RANK')} wants device {local} but {ndev} are visible "
                         "(FC_BENCH_DEVICE=0 + FC_BENCH_BACKEND=gloo rehearse several ranks on one GPU)")
    dist.init_process_group(backend=backend)
    return dist, dist.get_rank(), dist.get_world_size(), local


def device_identity(local: int) -> str:
    """This rank's device: the PCI bus id of HIP device ``local`` (fc_device_pci_id), or, with no
    GPU (the CPU launcher test), ``cpu:<host>:<pid>``."""
    import socket
    try:
        from flipcomplexityempirical_amd import _lib
        if _lib.device_count() > 0:
            import ctypes
            buf = ctypes.create_string_buffer(32)
            if _lib.load().fc_device_pci_id(int(local), buf, 32) == 0:
                return buf.value.decode()
    except Exception:  # no library / no device: the CPU identity below
        pass
    return f"cpu:{socket.gethostname()}:{os.getpid()}"


def gather_devices(dist, local: int) -> dict:
    """Every rank's device identity, gathered on all ranks (an N-GPU line shows
    that N distinct GPUs did the work).  ``distinct`` is False only in rehearsals that put several
    ranks on one device (FC_BENCH_DEVICE)."""
    me = {"rank": dist.get_rank() if dist is not None else 0, "local_rank": local,
          "device": device_identity(local), "host": __import__("socket").gethostname()}
    if dist is None:
        ids = [me]
    else:
        ids = [None] * dist.get_world_size()
        dist.all_gather_object(ids, me)
    keys = [(d["host"], d["device"]) for d in ids]
    return {"per_rank": ids, "distinct": len(set(keys)) == len(keys)}


def spawn_probe():
    """FC_BENCH_SPAWN_PROBE=1 (CPU test of the launcher, tests/test_bench_launch.py): each rank
    joins the process group over gloo, sums its rank, gathers every rank's device identity, and
    rank 0 prints what it saw."""
    import torch
    import torch.distributed as dist
    dist.init_process_group(backend="gloo")
    t = torch.tensor([float(dist.get_rank())])
    dist.all_reduce(t)
    devs = gather_devices(dist, int(os.environ.get("LOCAL_RANK", "0")))
    if dist.get_rank() == 0:
        print(json.dumps({"ranks_seen": dist.get_world_size(), "rank_sum": float(t.item()),
                          "launcher": os.environ.get("FC_BENCH_LAUNCHER", "external"), "devices": devs}), flush=True)
    dist.destroy_process_group()


def _cpu_worker(args):
    """One chain of the same workload on a gerrychain-faithful Python port: ``native`` is
    the reference's own proposal mechanism (``random.choice(list(b_nodes))``, :143, or for
    k > 2 ``random.choice`` over the (node, district) pairs, :128 / :151-153, with CPython /
    numpy Mersenne Twisters), ``philox`` the canonical-stream port."""
    gid, seconds, wname, kind = args
    sys.path.insert(0, ROOT)
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import GcFaithfulChain, NativeRngChain
    w = Workload(wname)
    spec = w.spec
    a = w.init_of(gid)
    plan = {spec.nodes[i]: w.labels[int(a[i])] for i in range(spec.n)}
    (lo, hi), _ = G.population_bounds(int(spec.pop.sum()), w.k, w.pct)
    if kind == "native":
        ch = NativeRngChain(spec, plan, base=w.base_of(gid), pop_bounds=(lo, hi), seed=w.seed * 1000003 + gid,
                            log1mp=G.log1mp_table(spec.n, w.k), pair=w.k > 2)
    else:
        ch = GcFaithfulChain(spec, plan, base=w.base_of(gid), pop_bounds=(lo, hi), seed=w.seed,
                             chain_id=gid, log1mp=G.log1mp_table(spec.n, w.k), pair=w.k > 2)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            ch.step()
    dt = time.perf_counter() - t0
    return ch.stats["proposals"], ch.stats["steps"], dt


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpu_share():
    """(usable, info): the CPUs this process can run on at once -- its affinity set, capped by
    a cgroup CPU quota (v2 ``cpu.max`` or v1 ``cpu.cfs_quota_us``) -- and the facts behind it.
    The CPU baseline runs one process per usable CPU (all host cores)."""
    import math
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = total
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return usable, {"host_cpus": total, "affinity_cpus": aff, "cgroup_quota_cpus": quota,
                    "cpu_model": cpu_model()}


def cpu_baseline(seconds: float, cores: int, wname: str = "c2", kind: str = "native"):
    """The reference's Python CPU path on the host cores: one chain per process, chain ids
    0..cores-1 of the workload (so every base of the C2 sweep is sampled), ``seconds`` each."""
    from concurrent.futures import ProcessPoolExecutor
    with ProcessPoolExecutor(max_workers=cores) as ex:
        res = list(ex.map(_cpu_worker, [(g, seconds, wname, kind) for g in range(cores)]))
    props = sum(r[0] for r in res)
    wall = max(r[2] for r in res)
    what = ("the reference's flip step under its own random streams (oracle/flipref.py NativeRngChain: "
            + ("random.choice(list(b_nodes)) at grid_chain_sec11.py:143" if Workload(wname).k == 2 else
               "random.choice over the (node, district) pairs of slow_reversible_propose, grid_chain_sec11.py:128 "
               "over :151-153")
            + ", random() at :179, np.random.geometric at :148, gerrychain-0.2 Partition / cut_edges / Dijkstra "
            "contiguity" + ("; where 1 - p rounds to 1.0 in double (C4 / C5: N^k beyond 2^53 |B|) its wait is "
                            "saturated at 2^62 like the C oracle's and the device's, where numpy's geometric gives "
                            "INT64_MIN -- sum_wait parity unpinned there" if Workload(wname).k > 2 else "")
            + ")" if kind == "native" else
            "gerrychain-0.2-faithful Python restatement on the canonical Philox stream "
            "(oracle/flipref.py GcFaithfulChain)")
    return {"value": props / wall, "unit": "proposals/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{what}; {cores} processes x 1 chain of the same workload (chain ids 0..{cores - 1}) "
                      f"for {seconds:.0f} s each from the start plans; {props} proposals"}


def c_oracle_rate(seconds: float, wname: str = "c2", g0: int = 0, stride: int = 1):
    """Single-core rate of the plain-C oracle on the same workload (extra, informational):
    chains g0, g0 + stride, ... of 20,000 steps each until ``seconds`` have passed."""
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import CRef
    w = Workload(wname)
    spec = w.spec
    cref = CRef()
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), w.k, w.pct)
    l1 = G.log1mp_table(spec.n, w.k)
    props, t0, g = 0, time.perf_counter(), g0
    while time.perf_counter() - t0 < seconds:
        r = cref.run(spec, w.init_of(g), base=w.base_of(g), pop_lo=lo, pop_hi=hi, seed=w.seed, chain_id=g,
                     n_steps=20000, log1mp=l1, k=w.k, labels=w.labels, proposal=w.proposal)
        props += r["stats"]["proposals"]
        g += stride
    return props / (time.perf_counter() - t0)


def _c_oracle_worker(args):
    sys.path.insert(0, ROOT)
    return c_oracle_rate(*args)


def c_oracle_allcores(seconds: float, cores: int, wname: str = "c2"):
    """The strong CPU baseline: the plain-C oracle, one process per core,
    process i running chains i, i + cores, ... (every base of the sweep is covered)."""
    from concurrent.futures import ProcessPoolExecutor
    with ProcessPoolExecutor(max_workers=cores) as ex:
        rates = list(ex.map(_c_oracle_worker, [(seconds, wname, i, cores) for i in range(cores)]))
    return {"value": float(sum(rates)), "unit": "proposals/s", "cores": cores, "kind": "port",
            "sample": f"plain-C oracle (oracle/flipref.c), {cores} processes, chains of 20,000 steps for "
                      f"{seconds:.0f} s each"}


def recom_leg(args) -> dict:
    """Side line ``--workload recom``: the reference's ``tree_proposal`` (partial(recom,
    pop_col="population", pop_target=ideal, epsilon=0.05, node_repeats=1), grid_chain_sec11.py:328-335)
    on sec11, k = 2, the population Validator (0.1), always_accept; 4096 chains per GPU, one launch =
    ``--chain-steps`` ReCom steps per chain (default here 20).  Device time from HIP events on the run's
    stream; the roofline prices each spanning tree's algorithmic bytes -- every adjacency entry read
    once (4 B x 2E), a weight per edge (4 B x E), the tree's parent and subtree population per node
    (8 B x n) and the relabelled assignment (1 B x n) -- against the LDS aggregate (the chain's
    working set is LDS-resident, fc_recom.hip).  CPU baseline: oracle/recomref.c, one process per
    usable CPU."""
    from flipcomplexityempirical_amd import _lib
    from flipcomplexityempirical_amd import graphs as G
    from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
    spec = G.sec11_graph()
    C = args.chains or 4096
    S = args.chain_steps
    plans = [spec.assignment_array(G.sec11_plan(al, spec.nodes), [-1, 1]) for al in range(3)]
    inits = np.stack([plans[c % 3] for c in range(C)])
    _, (lo, hi) = G.population_bounds(spec.n, 2, 0.1)
    seed = SEED + 0x10
    cfg = RunConfig(proposal=_lib.FC_PROPOSE_RECOM, seed=seed, pop_lo=lo, pop_hi=hi, base=1.0,
                    recom_pop_target=spec.n / 2, recom_epsilon=0.05, recom_node_repeats=1, diag_mask=0)
    run = FlipRun(FlipGraph(spec), inits, cfg)
    for _ in range(max(1, args.warmup)):
        run.steps(S)
    run.sync()
    run.timings()
    s0 = run.stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run.steps(S)
    run.sync()
    dt = time.perf_counter() - t0
    ms = run.timings()
    s1 = run.stats()
    steps = float((s1["steps"] - s0["steps"]).sum())
    trees = float((s1["bfs_levels"] - s0["bfs_levels"]).sum())
    roots = float((s1["bfs_calls"] - s0["bfs_calls"]).sum())
    kms = float(ms.mean())
    tree_bytes = 4 * 2 * spec.n_edges + 4 * spec.n_edges + 8 * spec.n + spec.n
    alg = tree_bytes * trees / args.steps
    lds_peak = LDS_READ_BPC[4] * LDS_CUS * LDS_CLK_GHZ  # b32 gathers
    out = {"metric": "recom steps/sec, sec11 40x40 k=2 (tree_proposal of grid_chain_sec11.py:328-335)",
           "value": steps / dt, "unit": "steps/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "dtype": "int8", "data": "synthetic",
           "config": {"workload": "ReCom on sec11 (N=1596), k=2, pop tol 0.1, always_accept, "
                                  f"{C} chains, {S} ReCom steps per chain per launch", "chains_per_gpu": C,
                      "chain_steps_per_launch": S},
           "kernel": run.kernel_name(), "kernel_ms": kms, "steps_per_s_kernel": steps / (ms.sum() * 1e-3),
           "trees_per_step": trees / steps, "roots_per_step": roots / steps,
           "build_id": _lib.build_id(),
           "roofline": {"bound": "lds", "achieved": alg / (kms * 1e-3) / 1e9, "peak": lds_peak, "unit": "GB/s",
                        "frac": alg / (kms * 1e-3) / 1e9 / lds_peak, "traffic": None,
                        "alg_bytes_per_tree": tree_bytes,
                        "note": "per spanning tree: adjacency 4 B x 2E + edge weight 4 B x E + parent / subtree "
                                "population 8 B x n + assignment 1 B x n, against the LDS b32 aggregate "
                                "(MI355X_MICROARCH.md §LDS: 128 B/clk/CU x 256 CUs x 2.4 GHz)"}}
    run.close()
    if not args.no_cpu_baseline:
        cores, share = host_cpu_share()
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(max_workers=cores) as ex:
            res = list(ex.map(_recom_cpu_worker, [(i, cores, min(args.cpu_seconds, 10.0), seed) for i in range(cores)]))
        out["cpu_baseline"] = {"value": sum(r[0] for r in res) / max(r[1] for r in res), "unit": "steps/s",
                               "cores": cores, "kind": "port", **share,
                               "sample": f"oracle/recomref.c, {cores} processes, chains of 50 steps from the start "
                                         f"plans for {min(args.cpu_seconds, 10.0):.0f} s each"}
    return out


def _recom_cpu_worker(args):
    i, stride, seconds, seed = args
    sys.path.insert(0, ROOT)
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import recom_run
    spec = G.sec11_graph()
    plans = [spec.assignment_array(G.sec11_plan(al, spec.nodes), [-1, 1]) for al in range(3)]
    _, (lo, hi) = G.population_bounds(spec.n, 2, 0.1)
    t0, n, c = time.perf_counter(), 0, i
    while time.perf_counter() - t0 < seconds:
        r = recom_run(spec, plans[c % 3], k=2, pop_target=spec.n / 2, epsilon=0.05, pop_lo=lo, pop_hi=hi,
                      seed=seed, chain_id=c, n_steps=50)
        n += r["stats"]["steps"]
        c += stride
    return n, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)  # 40 launches: ~2 s of timed GPU work per run
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chain-steps", type=int, default=100000)
    ap.add_argument("--chains", type=int, default=0, help="chains per GPU (0: the workload's)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5", "recom"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sweep-replicas", type=int, default=1,
                    help="side line (N = 1, c2): the reference's two sweeps -- all 174 configurations x R replicas, "
                         "100,000 yields each, every output file written (flipcomplexityempirical_amd.sweep); 0: skip")
    ap.add_argument("--full-diag-steps", type=int, default=6,
                    help="launches of the full-diagnostics side line (0: skip)")
    ap.add_argument("--acf-yields", type=int, default=10 * 65536,
                    help="C4 diagnostics leg: yields of the one series window the autocorrelation covers "
                         "(lags 1 .. 2^16; default 10 x 2^16)")
    ap.add_argument("--stream", default="auto", choices=["auto", "band", "node"],
                    help="k = 2 node stream (fc_params.stream, DESIGN.md §2): auto = node (the band stream "
                         "measured slower on C2, DESIGN.md §8)")
    ap.add_argument("--node-stream-steps", type=int, default=3,
                    help="k = 2 band runs: launches of the node-stream comparison line (0: skip)")
    ap.add_argument("--tune", default="",
                    help="launch tuning, e.g. nsub=2,hit_stop=24,prio_div=2:5:10 (fc_params.tune_*; "
                         "scheduling only)")
    ap.add_argument("--force-bfs", action="store_true",
                    help="FC_FLAG_FORCE_BFS: every proposal the ring rule does not prove valid goes to the device "
                         "search instead of the district-graph / planar rules (side lines only; with "
                         "--tune search_waves=4 the workgroup-cooperative search, BASELINE config 5)")
    ap.add_argument("--allow-variant", action="store_true",
                    help="load a profiling / experiment library (FC_LIB_PATH, FC_LIB_VARIANT): A/B tools only; "
                         "the line records fc_build_flags")
    args = ap.parse_args()

    bad = check_world(args.gpus)
    if bad:
        print(bad, file=sys.stderr, flush=True)
        sys.exit(2)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if os.environ.get("FC_BENCH_SPAWN_PROBE") == "1":
        spawn_probe()
        return

    dist, rank, world, local_rank = _dist()
    from flipcomplexityempirical_amd import _lib as _lib0
    _lib0.load(allow_variant=args.allow_variant)
    if args.workload == "recom":  # side line, one GPU
        if world > 1:
            raise SystemExit("bench.py --workload recom is a one-GPU side line")
        if args.chain_steps == 100000:
            args.chain_steps = 20
        print(json.dumps(recom_leg(args)), flush=True)
        return
    import torch
    from flipcomplexityempirical_amd import graphs as G
    from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig, parse_tune, pin_host, unpin_host
    from flipcomplexityempirical_amd import _lib

    tune = parse_tune(args.tune) or None
    run_flags = _lib.FC_FLAG_FORCE_BFS if args.force_bfs else 0
    W = Workload(args.workload)
    stream = "node" if args.stream == "auto" else args.stream
    spec = W.spec
    fg = FlipGraph(spec)
    from flipcomplexityempirical_amd import distributed as D
    C = args.chains or W.chains
    if not args.chains and W.name in ("c4", "c5"):
        # large graphs: one chain per workgroup, LDS-bound residency; size the launch to one
        # wave of resident chains (a second, partial wave would double the launch time)
        C = resident_chains(fg, W, local_rank, flags=run_flags, tune=tune)
    off, cnt = D.shard(C * world, world, rank)          # weak scaling: C chains per GPU
    gids = np.arange(off, off + cnt)
    inits = np.stack([W.init_of(int(g)) for g in gids])
    bases = np.asarray([W.base_of(int(g)) for g in gids])
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), W.k, W.pct)
    cfg = RunConfig(k=W.k, labels=tuple(W.labels), proposal=W.proposal, seed=W.seed, pop_lo=lo, pop_hi=hi,
                    chain_id_offset=int(off), device=local_rank, tune=tune, stream=stream, flags=run_flags)
    run = FlipRun(fg, inits, cfg, bases=bases)
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)

    def barrier_sync():
        run.sync()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        run.steps(args.chain_steps)
    barrier_sync()
    s0 = run.stats()
    run.timings()  # reset the per-launch event record
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run.steps(args.chain_steps)
    barrier_sync()
    t1 = time.perf_counter()
    launch_ms = run.timings()
    s1 = run.stats()
    kname = run.kernel_name()

    elapsed = t1 - t0
    props = float((s1["proposals"] - s0["proposals"]).sum())
    steps = float((s1["steps"] - s0["steps"]).sum())
    acc = float((s1["accepted"] - s0["accepted"]).sum())
    kernel_ms = float(launch_ms.mean()) if launch_ms.size else float("nan")

    # the one collective: per-base statistics summed over ranks (RCCL for N > 1)
    dev = None
    if dist is not None and dist.get_backend() == "nccl":
        dev = torch.device("cuda", local_rank)
    delta = {k: s1[k] - s0[k] for k in D.AGG_FIELDS}
    nb_ = len(W.bases)
    agg = D.allreduce_sum(D.group_aggregate(delta, gids % nb_, nb_), dist, dev)
    # per-rank record: each rank's mean launch time and timed-region wall time
    rank_rec = np.zeros((2, world), dtype=np.float64)
    rank_rec[:, rank] = (kernel_ms, elapsed)
    rank_rec = D.allreduce_sum(rank_rec, dist, dev)
    elapsed = D.allreduce_max(elapsed, dist, dev)
    kernel_ms = D.allreduce_max(kernel_ms, dist, dev)
    props, steps, acc = (float(agg[:, D.AGG_FIELDS.index(k)].sum()) for k in ("proposals", "steps", "accepted"))
    # every rank's device (PCI bus id): an N-GPU line must show N distinct GPUs; only a rehearsal
    # (FC_BENCH_DEVICE: several ranks on one device) may share one
    devices = gather_devices(dist, local_rank)
    if world > 1 and not devices["distinct"] and "FC_BENCH_DEVICE" not in os.environ:
        raise SystemExit(f"bench.py: ranks share a device: {devices['per_rank']}")

    node_out = None
    if stream == "band" and args.node_stream_steps > 0:
        # beside it (outside the timed region): the same workload on the node stream, whose draws
        # range over all n nodes (the round-2 kernel's stream)
        run.close()
        rn = FlipRun(fg, inits, RunConfig(k=W.k, labels=tuple(W.labels), proposal=W.proposal, seed=W.seed,
                                          pop_lo=lo, pop_hi=hi, chain_id_offset=int(off), device=local_rank,
                                          tune=tune, stream="node", flags=run_flags), bases=bases)
        rn.steps(args.chain_steps)
        rn.sync()
        if dist is not None:
            dist.barrier()
        n0 = rn.stats()
        rn.timings()
        tn0 = time.perf_counter()
        for _ in range(args.node_stream_steps):
            rn.steps(args.chain_steps)
        rn.sync()
        if dist is not None:
            dist.barrier()
        dtn = D.allreduce_max(time.perf_counter() - tn0, dist, dev)
        n1 = rn.stats()
        pn = float(D.allreduce_sum(np.asarray([float((n1["proposals"] - n0["proposals"]).sum())]), dist, dev)[0])
        dn = float(D.allreduce_sum(np.asarray([float((n1["draws"] - n0["draws"]).sum())]), dist, dev)[0])
        node_out = {"value": pn / dtn, "unit": "proposals/s", "launches": args.node_stream_steps,
                    "kernel": rn.kernel_name(), "kernel_ms": D.allreduce_max(float(rn.timings().mean()), dist, dev),
                    "draws_per_proposal": dn / pn if pn else None}
        rn.close()

    full_out = None
    if args.full_diag_steps > 0:
        # side line, outside the timed region above and on every rank: the same workload with
        # every per-yield tally of the reference's driver loop on (grid_chain_sec11.py:366-402:
        # cut / |B| histograms, per-edge cut_times, per-node num_flips / part_sum /
        # last_flipped), FULL instance; then the one §8(e) reduction of all of them
        run.close()
        # the reference's slope / angle lines (:371-394) need the per-step interface: on sec11
        # the kernel also logs every accepted flip, and after each launch the frame-series
        # kernel turns the log into per-event slope / angle, copied to the host as the
        # reference's lists (in chunks of chains)
        series = args.workload == "c2"
        # C4 (BASELINE config 4): the |cut| trace's autocorrelation at lags 1 .. 2^16 and the
        # hitting time of a target |cut| (10 % above the lowest start), on the device, per launch
        c4diag = args.workload == "c4"
        # C4: one series window over all its launches, long enough for the largest lag (VERDICT
        # r02 item 5): the leg runs as many launches as --acf-yields needs
        n_full = args.full_diag_steps
        if c4diag:
            n_full = max(n_full, -(-args.acf_yields // args.chain_steps))
        full = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_HIST | _lib.FC_DIAG_EDGES | _lib.FC_DIAG_FLIPS
        if series:
            full |= _lib.FC_DIAG_SERIES
        if c4diag:  # the config's own diagnostics: the accepted-flip log (ACF) and the hitting time
            full = _lib.FC_DIAG_WAIT | _lib.FC_DIAG_SERIES
        hit = (-1, -2)
        if c4diag:
            cut0 = min(G.cut_and_boundary(spec, inits[c])[0] for c in range(0, len(inits), max(1, len(inits) // 64)))
            hit = (int(np.ceil(1.1 * cut0)), 10 ** 9)
        cfg_f = RunConfig(k=W.k, labels=tuple(W.labels), proposal=W.proposal, seed=W.seed, pop_lo=lo, pop_hi=hi,
                          chain_id_offset=int(off), device=local_rank, diag_mask=full, tune=tune, stream=stream,
                          flags=run_flags,
                          event_cap=(n_full * args.chain_steps + 1 if c4diag else args.chain_steps + 1 if series else 0),
                          hit_lo=hit[0], hit_hi=hit[1])
        lags = [1 << i for i in range(17)]
        rf = FlipRun(fg, inits, cfg_f, bases=bases)
        frame = G.slope_frame(spec, "sec11") if series else None
        n_wu = max(1, args.warmup)
        for i in range(n_wu):  # untimed, as the headline leg's warmup launches
            if i and (series or c4diag):
                rf.series_reset()  # (the event log holds one window; the last warmup's sizes the buffers)
            rf.steps(args.chain_steps)
        barrier_sync_f = lambda: (rf.sync(), dist.barrier() if dist is not None else None)  # noqa: E731
        cp_buf = None
        if series:
            # setup, once, outside the timed leg: host buffers for the change points, sized from
            # the warmup launch's count (+50 %), page-locked (a per-launch pin would dominate)
            n_cp = int(rf.frame_series_changes(frame, query=True)["offsets"][-1])
            n_cp = n_cp + n_cp // 2 + 4 * C
            cp_buf = {"t": np.empty(n_cp, dtype=np.int64), "slope": np.empty(n_cp), "angle": np.empty(n_cp)}
            for b_ in cp_buf.values():
                pin_host(b_)
        if series or c4diag:
            rf.series_reset()
        barrier_sync_f()
        f0 = rf.stats()
        rf.timings()
        t_series, n_events, n_nan, n_changes, n_cp_fallback = 0.0, 0, 0, 0, 0
        t_checks = 0.0  # the bench line's own counts / NaN scan of the series (not the reference's work)
        t_pe, n_pe = 0.0, 0   # the per-event form, measured on the last launch only (outside the rates)
        t_acf, acf_out = 0.0, None
        fs_buf = None
        t0f = time.perf_counter()
        for it in range(n_full):
            rf.steps(args.chain_steps)
            if c4diag and it == n_full - 1:  # the whole window: every lag has yields - lag pairs
                rf.sync()
                ts = time.perf_counter()
                _, acf = rf.autocorr(lags)
                pairs = rf.autocorr_pairs(lags)
                acf_out = {"acf_mean": [float(x) for x in np.nanmean(acf, axis=0)],
                           "acf_min": [float(x) for x in np.nanmin(acf, axis=0)],
                           "acf_max": [float(x) for x in np.nanmax(acf, axis=0)],
                           "pairs_min": [int(x) for x in pairs.min(axis=0)],
                           "window_yields": int((rf.stats()["steps"] - rf.stats()["series_t0"] + 1).min())}
                t_acf += time.perf_counter() - ts
            if series:
                rf.sync()  # the launch is asynchronous: its time must not land in t_series
                ts = time.perf_counter()
                # the reference's slope / angle lists (:371-394) as what its plots draw
                # (:476-484): change points (t, slope, angle) of every chain, on the device, one
                # copy per array into pinned host buffers reused over the launches
                ch = rf.frame_series_changes(frame, out=cp_buf)
                t_series += time.perf_counter() - ts
                # the line's own checks (counts for the JSON, a scan of the angles): outside both
                # rates, timed apart
                tc = time.perf_counter()
                n_changes += int(ch["offsets"][-1])
                # more change points than the pinned buffers hold: a second native call into
                # fresh unpinned arrays (counted)
                n_cp_fallback += int(ch["offsets"][-1] > cp_buf["t"].size)
                n_events += int(rf.stats()["events"].sum())
                n_nan += int(np.isnan(ch["angle"]).sum())
                t_checks += time.perf_counter() - tc
                if it == n_full - 1:
                    # beside it, once: the per-event form (every event's slope / angle / frame-cut
                    # count) copied to the host in chunks of 256 chains
                    tp = time.perf_counter()
                    cap_all = int(rf.stats()["events"].max()) + 1
                    fs_buf = {"slope": np.empty(256 * cap_all), "angle": np.empty(256 * cap_all),
                              "n_cut": np.empty(256 * cap_all, dtype=np.int32)}
                    for c0 in range(0, C, 256):
                        fs = rf.frame_series(frame, chains=range(c0, min(C, c0 + 256)),
                                             out={k: v.reshape(1, -1) for k, v in fs_buf.items()})
                        n_pe += int(fs["len"].sum())
                    t_pe += time.perf_counter() - tp
                rf.series_reset()
        barrier_sync_f()
        dtf = D.allreduce_max(time.perf_counter() - t0f - t_pe - t_checks, dist, dev)
        if cp_buf is not None:
            for b_ in cp_buf.values():
                unpin_host(b_)
        kf = D.allreduce_max(float(rf.timings().mean()), dist, dev)
        diag_paths = rf.diag_paths()
        f1 = rf.stats()
        arrays = {}
        if full & _lib.FC_DIAG_HIST:
            arrays["cut_hist"], arrays["nb_hist"] = rf.hist()
        if full & _lib.FC_DIAG_EDGES:
            arrays["cut_times"] = rf.cut_times()
        if full & _lib.FC_DIAG_FLIPS:
            arrays["num_flips"], arrays["part_sum"], arrays["last_flipped"] = rf.flips()
        # per configuration: one row per (base, alignment) group, so an N-GPU
        # run of the sweep still yields every configuration's arrays (:383-384,396-400,416-419)
        red = D.allreduce_statistics(D.local_statistics(f1, W.group_of(gids), W.n_groups, arrays), dist, dev)
        pf = float((f1["proposals"] - f0["proposals"]).sum())
        pf = float(D.allreduce_sum(np.asarray([pf]), dist, dev)[0])
        yields = int(red["scalars"][:, D.AGG_FIELDS.index("steps")].sum()) + C * world
        t_series = D.allreduce_max(t_series, dist, dev)
        t_acf = D.allreduce_max(t_acf, dist, dev)
        full_out = {"value": pf / (dtf - t_series - t_acf), "unit": "proposals/s", "launches": n_full,
                    "value_with_frame_series_on_host": pf / dtf if series else None,
                    "kernel": rf.kernel_name(), "kernel_ms": kf,
                    "diag_paths": dict(diag_paths, note="fc_run_diag_paths: tally-log entries per chain granted / "
                                       "asked for (granted below asked: chains may apply tallies by atomics), and "
                                       "whether the change points ran one staged pass (1) or two (0); same outputs"),
                    "diag": ("waits + accepted-flip log -> |cut| autocorrelation and hitting time on the device "
                             "(BASELINE config 4)" if c4diag else
                             "waits + cut/|B| histograms + per-edge cut_times + per-node flips"
                             + (" + accepted-flip log -> slope / angle series (change points) on the device, "
                                "copied to the host" if series else "")
                             + " (the reference loop body, grid_chain_sec11.py:367-400)"),
                    "frame_series": {"ms_per_launch": t_series / max(n_full, 1) * 1e3,
                                     "events": n_events, "change_points": n_changes,
                                     "pinned_buffer_misses": n_cp_fallback,
                                     "pinned_buffer_entries": int(cp_buf["t"].size) if cp_buf else None,
                                     "events_per_s": n_events / t_series if t_series else None,
                                     "nan_angles_at_change_points": n_nan,
                                     "bench_checks_ms_per_launch": t_checks / max(n_full, 1) * 1e3,
                                     "bench_checks_note": "the line's own counts (events from the chain "
                                                          "records) and the NaN scan of the angles, timed apart "
                                                          "and outside both rates",
                                     "note": "fc_run_frame_series_changes over all chains after every launch: the "
                                             "(t, slope, angle) change points of the reference's per-yield slope / "
                                             "angle lists (:371-394), bitwise those lists when held over their "
                                             "yields (what :476-484 plot), copied into pinned host buffers",
                                     "per_event_form": {"ms_one_launch": t_pe * 1e3, "entries": n_pe,
                                                        "note": "fc_run_frame_series (one entry per event, slope / "
                                                                "angle / frame-cut count) over all chains in chunks "
                                                                "of 256, last launch only, outside both rates"}}
                    if series else None,
                    "c4_series": {"hit_window": list(hit), "hit_fraction": float((f1["hit_time"] >= 0).mean()),
                                  "lags": lags, **(acf_out or {}),
                                  "autocorr_ms": t_acf * 1e3,
                                  "note": "fc_run_autocorr (event log -> per-yield |cut| -> exact lag sums) over one "
                                          "series window spanning every launch of the leg (no reset), after the "
                                          "last launch; acf / pairs per lag over chains (pairs = yields - lag)"}
                    if c4diag else None,
                    "reduced": {"ranks": world, "collectives": "allreduce SUM (scalars, histograms, cut_times, "
                                "num_flips, part_sum) + allreduce MAX (last_flipped), one row per configuration",
                                "groups": W.n_groups, "group_of_chain": f"g % {W.n_groups}",
                                "yields": yields, "cut_hist_mass": int(red["cut_hist"].sum()) if "cut_hist" in red else None,
                                "cut_hist_mass_per_group_ok": (bool(np.array_equal(
                                    red["cut_hist"].sum(axis=1),
                                    red["scalars"][:, D.AGG_FIELDS.index("steps")] +
                                    np.bincount(W.group_of(np.arange(C * world)), minlength=W.n_groups)))
                                    if "cut_hist" in red else None),
                                "checksums": D.checksums(red),
                                "per_group": [dict(W.group_desc[i],
                                                   chains=int(np.sum(W.group_of(np.arange(C * world)) == i)),
                                                   sum_wait=int(red["scalars"][i, D.AGG_FIELDS.index("sum_wait")]),
                                                   checksums={nm: D.group_checksums({nm: a})[nm][i]
                                                              for nm, a in red.items() if nm != "scalars"})
                                              for i in range(W.n_groups)]}}
        rf.close()

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    value = props / elapsed
    per_launch_props = props / world / args.steps
    per_launch_acc = acc / world / args.steps
    alg_bytes = W.R * per_launch_props + W.W * per_launch_acc
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    acc_pp = per_launch_acc / per_launch_props if per_launch_props else 0.0
    lds_peak = lds_mix_peak_gbs(W.rmix, W.wmix, acc_pp)
    traffic, traffic_src, traffic_stale = measured_traffic(args.workload, kname, C, args.chain_steps,
                                                           build_id=_lib.build_id())
    levels = roofline_levels(W, per_launch_props, per_launch_acc, kernel_ms, traffic)
    l1l2 = measured_l2(args.workload, kname, C, args.chain_steps, kernel_ms, _lib.build_id())
    out = {
        "metric": METRIC if args.workload == "c2" else f"flip proposals/sec, side workload {args.workload}",
        "value": value, "unit": "proposals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int8",
        "ranks_seen": dist.get_world_size() if dist is not None else 1,
        "backend": dist.get_backend() if dist is not None else None,
        "launcher": os.environ.get("FC_BENCH_LAUNCHER") or ("torch.distributed.run" if dist is not None else None),
        "devices": devices,
        "per_rank_kernel_ms": [float(x) for x in rank_rec[0]],
        "per_rank_elapsed_s": [float(x) for x in rank_rec[1]],
        "build_flags": _lib.build_flags(),
        "build_id": _lib.build_id(),
        "hip_runtime": _lib.hip_runtime_path(),
        "data": W.data + (" (band node stream: draws over b_nodes + neighbours)" if stream == "band" else ""),
        "config": {"workload": W.desc, "graph": args.workload, "k": W.k, "chains_per_gpu": C,
                   "chain_steps_per_launch": args.chain_steps,
                   "parallelism": f"chains sharded over {world} GPU(s)", "tune": tune, "stream": stream},
        "steps_per_s": steps / elapsed,
        "per_base_proposals_per_s": {f"{b:.4g}": float(agg[i, 0]) / elapsed for i, b in enumerate(W.bases)},
        "accept_per_proposal": acc / props if props else None,
        "draws_per_proposal": float(agg[:, D.AGG_FIELDS.index("draws")].sum()) / props if props else None,
        "bfs_per_proposal": float((s1["bfs_calls"] - s0["bfs_calls"]).sum()) * world / props if props else None,
        "bfs_levels_per_search": (float((s1["bfs_levels"] - s0["bfs_levels"]).sum()) /
                                  float((s1["bfs_calls"] - s0["bfs_calls"]).sum()))
        if float((s1["bfs_calls"] - s0["bfs_calls"]).sum()) > 0 else None,
        "force_bfs": bool(args.force_bfs),
        "roofline": {"bound": levels["bound"], "achieved": levels[levels["bound"]]["achieved"],
                     "peak": levels[levels["bound"]]["peak"], "unit": "GB/s",
                     "frac": levels[levels["bound"]]["frac"], "traffic": traffic,
                     "levels": levels,
                     "levels_note": "SURVEY §8(d)'s algorithmic bytes split by where they live (bench.roofline_levels): "
                                    "lds = the LDS-resident chain state (per proposal %s B by access width, every "
                                    "write) against the LDS aggregate at that mix; l2 = the global node records "
                                    "(row_ptr pair, col_idx, ring indices: %.0f B per proposal) against the L2 "
                                    "aggregate (MI355X_MICROARCH.md §L2); hbm = measured bytes; bound = the largest "
                                    "fraction; achieved / peak / frac above are the bound level's"
                                    % (W.lds_mix, W.glob_bytes),
                     "l2_measured": l1l2,
                     "all_bytes_vs_lds": {"achieved": achieved, "peak": lds_peak, "frac": achieved / lds_peak,
                                          "peak_b128": LDS_PEAK_B128_GBS, "frac_b128": achieved / LDS_PEAK_B128_GBS},
                     "peak_note": "all_bytes_vs_lds: every algorithmic byte priced at the LDS aggregate of the byte "
                                  "mix (MI355X_MICROARCH.md §LDS: u8 / u16 / b32 reads 32 / 64 / 128 B/clk/CU, writes "
                                  "half; 256 CUs, 2.4 GHz; reads %s B, writes %s B per accept, %.3f accepts per "
                                  "proposal), the round-3 pricing" % (W.rmix, W.wmix, acc_pp),
                     "traffic_note": "HBM bytes per launch from rocprofv3 FETCH_SIZE/WRITE_SIZE passes of "
                                     "this kernel, run shape and library build (%s; gfx950 FETCH_SIZE doubled)"
                                     % (traffic_src or "none recorded for this build"),
                     "traffic_stale_build": traffic_stale,
                     "kernel": kname,
                     "kernel_ms": kernel_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "alg_bytes_per_proposal": W.R, "alg_bytes_per_accept": W.W,
                     "hbm": {"peak": HBM_PEAK_GBS, "frac_alg": achieved / HBM_PEAK_GBS,
                             "measured_gbs": (traffic / (kernel_ms * 1e-3) / 1e9) if traffic else None,
                             "frac_measured": (traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                             if traffic else None}},
    }
    if full_out is not None:
        out["full_diagnostics"] = full_out
    if world == 1 and args.workload == "c2" and args.sweep_replicas > 0:
        out["reference_sweeps"] = sweep_leg(args.sweep_replicas, local_rank)
    if node_out is not None:
        out["node_stream"] = node_out
    if not args.no_cpu_baseline:
        # rank 0 only (the other ranks have left), after every collective and outside the timed
        # region, so an N-GPU line carries its CPU baseline too: one process per CPU this job can
        # use -- every host core, unless the affinity set or a cgroup quota grants fewer (then the
        # host's figure is stated as an extrapolation)
        cores, share = host_cpu_share()
        try:
            kind = "native"
            cb = cpu_baseline(args.cpu_seconds, cores, args.workload, kind)
            cb.update(share)
            cb["cores_note"] = ("one process per usable CPU: os.sched_getaffinity, capped by the cgroup CPU quota; "
                                "host_cpus is the machine's count")
            if cores < share["host_cpus"]:
                cb["value_host_cpus_extrapolated"] = cb["value"] / cores * share["host_cpus"]
            out["cpu_baseline"] = cb
            if kind == "native":
                out["cpu_baseline_philox_port"] = cpu_baseline(min(5.0, args.cpu_seconds), cores, args.workload,
                                                               "philox")
            out["cpu_baseline_c_oracle_1core"] = c_oracle_rate(min(5.0, args.cpu_seconds), args.workload)
            out["cpu_baseline_c_oracle_allcores"] = c_oracle_allcores(min(5.0, args.cpu_seconds), cores, args.workload)
        except Exception as ex:  # report, never fake
            out["cpu_baseline"] = {"value": None, "error": repr(ex)}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
