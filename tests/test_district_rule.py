"""The district-graph contiguity rule of the k > 2 kernel (fc_kernels.hip ``district_rule``)
restated in Python and checked against the oracle's BFS restatement of
``single_flip_contiguous`` [gc-0.2] (grid_chain_sec11.py:22,340) on every boundary node of
chain states of the k > 2 workloads (C3 sec11 k = 4, C4 triangular k = 8, C5 Delaunay k = 6 / 18,
FRANK k = 3) and of enclave states -- a district wholly inside another, where removing a node
between two A-runs can leave A connected around the enclave.  CPU only."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd.engine import FlipGraph

O = 31  # bit / node of the outer face in the district graph


def face_adjacency(ring, meta, a):
    """adj[X]: districts sharing a face with X (ring pairs), bit O when X has an outer-face
    node; adj[O]: the districts with outer-face nodes (the kernel's adj table)."""
    adj = np.zeros(32, dtype=np.int64)
    for v in range(len(a)):
        L = int(meta[v]) & 0xff
        for j in range(L):
            w = ring[v][j]
            if a[w] != a[v]:
                adj[a[v]] |= 1 << int(a[w])
        if (int(meta[v]) >> 9) & 1:
            adj[a[v]] |= 1 << O
            adj[O] |= 1 << int(a[v])
    return adj


def district_rule(ring, meta, a, v, adj):
    """(valid, multi_run) for flipping v out of its district."""
    m = int(meta[v])
    L, nbr, gam = m & 0xff, (m >> 16) & 0xffff, (m >> 9) & 1
    A = int(a[v])
    cells = [int(a[ring[v][j]]) for j in range(L)] + ([O] if gam else [])
    isn = [(nbr >> j) & 1 for j in range(L)] + ([0] if gam else [])
    Lp = len(cells)
    inA = [c == A for c in cells]
    if not any(inA[j] and isn[j] for j in range(Lp)):
        return False, False
    if all(inA):
        return True, False
    s = next(j for j in range(Lp) if not inA[j])
    runs, cur = [], []
    for t in range(Lp):
        p = (s + 1 + t) % Lp
        if inA[p]:
            cur.append(p)
        elif cur:
            runs.append(cur)
            cur = []
    if cur:
        runs.append(cur)
    rel = [r for r in runs if any(isn[p] for p in r)]
    if len(rel) <= 1:
        return True, False
    relA = {p for r in rel for p in r}
    s0 = next(iter(relA))
    gaps, cur = [], None
    for t in range(1, Lp + 1):
        p = (s0 + t) % Lp
        if p in relA:
            if cur is not None:
                gaps.append(cur)
                cur = None
        else:
            cur = (cur or 0) | (0 if inA[p] else 1 << cells[p])
    if cur is not None:
        gaps.append(cur)
    seen, notA = 0, ~(1 << A)
    for D in gaps:
        comp, fr = D, D
        while fr:
            X = (fr & -fr).bit_length() - 1
            fr &= fr - 1
            nb = int(adj[X]) & notA & ~comp
            comp |= nb
            fr |= nb
        if comp & seen:
            return False, True
        seen |= comp
    return True, True


HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "flipcomplexityempirical_amd", "csrc")
_KLIB = {}


def _kernel_rule_lib(tmp_dir):
    """csrc/fc_ring.h's district_rule -- the function flip_kernel calls -- built for the host."""
    if "lib" not in _KLIB:
        if shutil.which("g++") is None:
            pytest.skip("no host C++ toolchain")
        so = os.path.join(str(tmp_dir), "district_rule_lib.so")
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", CSRC, "-o", so,
                        os.path.join(HERE, "native", "district_rule_lib.cpp")], check=True)
        lib = ctypes.CDLL(so)
        i32, u32 = ctypes.c_int32, ctypes.c_uint32
        lib.fc_test_district_rule.argtypes = [i32, ctypes.POINTER(i32), u32, u32, u32, i32, i32, ctypes.POINTER(u32)]
        lib.fc_test_district_rule.restype = ctypes.c_int
        _KLIB["lib"] = lib
    return _KLIB["lib"]


def kernel_rule(lib, ring, meta, a, v, adj):
    """The kernel's verdict for a flip of v whose old-district neighbours are not one run:
    district_rule(adv, inA, nbr, Ln, gam, A, adj) with the kernel's own inputs (ring cells'
    districts, padded entries = v itself; adj words as the kernel keeps them)."""
    R = ring.shape[1]
    m = int(meta[v])
    L, nbr, gam = m & 0xff, (m >> 16) & 0xffff, (m >> 9) & 1
    adv = np.ascontiguousarray(a[ring[v]].astype(np.int32))
    A = int(a[v])
    inA = int(sum(1 << j for j in range(L) if adv[j] == A))
    adjw = np.ascontiguousarray((adj & 0xffffffff).astype(np.uint32))
    return lib.fc_test_district_rule(R, adv.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), inA, nbr, L, gam, A,
                                     adjw.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))) == 1


def _check_states(cref, spec, states, lib=None):
    ring, meta = FlipGraph(spec).rings()
    e = spec.edges()
    tally = {"multi_valid": 0, "multi_invalid": 0, "checked": 0, "outer_multi_valid": 0}
    for a in states:
        adj = face_adjacency(ring, meta, a)
        bn = np.unique(e[a[e[:, 0]] != a[e[:, 1]]].reshape(-1))
        for v in bn:
            got, multi = district_rule(ring, meta, a, int(v), adj)
            ref = cref.flip_contiguous(spec, a, int(v)) == 1
            assert got == ref, (int(v), spec.nodes[int(v)], got, ref)
            m = int(meta[v])
            has_old = any(((m >> 16) >> j) & 1 and a[ring[v][j]] == a[v] for j in range(m & 0xff))
            if lib is not None and has_old:
                # every flip with an old-district neighbour (the kernel calls the rule off one-run rings)
                kr = kernel_rule(lib, ring, meta, a, int(v), adj)
                assert kr == ref, ("kernel district_rule", int(v), spec.nodes[int(v)], kr, ref)
            tally["checked"] += 1
            if multi:
                tally["multi_valid" if got else "multi_invalid"] += 1
                if got and (int(meta[v]) >> 9) & 1:
                    tally["outer_multi_valid"] += 1
    return tally


def _chain_states(cref, spec, a0, k, base, pct, steps_list, seed):
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    out = []
    for c, steps in enumerate(steps_list):
        r = cref.run(spec, a0, base=base, pop_lo=lo, pop_hi=hi, seed=seed, chain_id=c, n_steps=steps, k=k,
                     labels=list(range(k)), proposal=1)
        out.append(r["final"])
    return out


@pytest.mark.parametrize("name", ["sec11_k4", "tri_k8", "delaunay_k6", "delaunay_k18", "frank_k3"])
def test_district_rule_equals_bfs_on_workload_states(cref, name, tmp_path):
    if name == "sec11_k4":
        spec = G.sec11_graph()
        k, a0, base, pct = 4, None, 0.5, 0.05
        a0 = spec.assignment_array(G.quadrant_plan(spec.nodes), list(range(k)))
    elif name == "tri_k8":
        spec = G.triangular_graph(30, 58)
        k, base, pct = 8, 0.5, 0.1
        a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    elif name.startswith("delaunay"):
        spec = G.delaunay_graph(1500, seed=0)
        k = 6 if name.endswith("6") else 18
        base, pct = 1.0, 0.3
        a0 = spec.assignment_array(G.bisection_plan(spec, k), list(range(k)))
    else:
        spec = G.frank_graph()
        k, base, pct = 3, 0.5, 0.5
        a0 = spec.assignment_array({n: (0 if n[0] < 7 else 1 if n[0] < 14 else 2) for n in spec.nodes}, [0, 1, 2])
    states = _chain_states(cref, spec, a0, k, base, pct, [3000, 12000, 30000], seed=17)
    t = _check_states(cref, spec, states, lib=_kernel_rule_lib(tmp_path))
    assert t["checked"] > 1000 and t["multi_invalid"] > 0


ENCLAVES = ((7, 6), (7, 0), (7, 13), (12, 6), (13, 13), (7, 1), (1, 7), (12, 12))


def enclave_plan(spec, ex, ey):
    """k = 3 on a grid: district 2 a 3 x 3 block at (ex, ey) inside district 1 (x >= 6),
    district 0 the columns x < 6."""
    plan = {}
    for n in spec.nodes:
        x, y = n
        plan[n] = 2 if (ex <= x <= ex + 2 and ey <= y <= ey + 2) else (0 if x < 6 else 1)
    return spec.assignment_array(plan, [0, 1, 2])


def test_district_rule_enclaves(cref, tmp_path):
    """k = 3 on a 16 x 16 grid: district 2 starts as a 3 x 3 enclave inside district 1 (it
    touches neither district 0 nor the outer face), one column of district 1 away from
    district 0.  Nodes of that column between the enclave and district 0 have two A-runs whose
    gaps are not joined in the complement -- valid multi-run flips the old same-district rule
    could not decide; nearby enclave placements and short chains from them add more.  Enclaves
    one row or column from the outer face ((7, 1), (1, 7)) make outer nodes whose ring's A-runs
    are separated by the enclave and the outer-face wedge: valid flips, which the kernel's rule
    used to reject (the wedge took district A's bit on rings shorter than RMAX).
    Both the restatement and the kernel's own district_rule, built for the host, must equal
    the BFS."""
    spec = G.grid_graph(16, 16)
    states = []
    for ex, ey in ENCLAVES:
        a0 = enclave_plan(spec, ex, ey)
        states += [a0] + _chain_states(cref, spec, a0, 3, 4.0, 0.9, [5, 30, 200], seed=5 + ex + ey)
    t = _check_states(cref, spec, states, lib=_kernel_rule_lib(tmp_path))
    assert t["multi_valid"] > 0 and t["multi_invalid"] > 0 and t["outer_multi_valid"] > 0, t
