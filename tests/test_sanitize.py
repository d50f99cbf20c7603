"""Host sanitizer run: the native planar ring builder
(``csrc/fc_graph.cpp``, the body of ``fc_graph_create``, which walks faces of caller-supplied
CSR + positions) and the plain-C oracle (``oracle/flipref.c``), compiled with
``-fsanitize=address,undefined`` (``tests/sanitize/Makefile``) and driven on the reference's
lattices, the Delaunay workload and malformed CSR / position inputs.  Any sanitizer report
aborts the harness (``-fno-sanitize-recover=all``), so a clean exit with the expected verdict
is the pass condition.  CPU only."""
import fcntl
import os
import shutil
import subprocess

import numpy as np
import pytest

from flipcomplexityempirical_amd import graphs as G

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")
EXE = os.path.join(SAN, "build", "san_harness")


@pytest.fixture(scope="module")
def harness():
    if shutil.which("g++") is None or shutil.which("make") is None:
        pytest.skip("no host C++ toolchain")
    # one build at a time: pytest-xdist workers share tests/sanitize/build
    os.makedirs(os.path.join(SAN, "build"), exist_ok=True)
    with open(os.path.join(SAN, "build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            subprocess.run(["make", "-s", "-C", SAN], check=True)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return EXE


def _write(path, n, row, col, pop, pos=None, flags=0, k=2, n_steps=0, assign=None, nnz=None):
    row = np.asarray(row, dtype=np.int32)
    col = np.asarray(col, dtype=np.int32)
    with open(path, "wb") as f:
        np.asarray([n, col.size if nnz is None else nnz], dtype=np.int32).tofile(f)
        row.tofile(f)
        col.tofile(f)
        np.asarray(pop, dtype=np.int32).tofile(f)
        np.asarray([0 if pos is None else 1], dtype=np.int32).tofile(f)
        if pos is not None:
            np.asarray(pos, dtype=np.float64).reshape(-1).tofile(f)
        np.asarray([flags], dtype=np.uint32).tofile(f)
        np.asarray([k, n_steps], dtype=np.int32).tofile(f)
        if n_steps > 0:
            np.asarray(assign, dtype=np.int8).tofile(f)


def _run(exe, path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    res = subprocess.run([exe, path], capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0 and "ERROR: AddressSanitizer" not in res.stderr and "runtime error" not in res.stderr, \
        (res.returncode, res.stdout[-2000:], res.stderr[-4000:])
    return res.stdout


def _spec_case(spec, k, plan, steps):
    a = spec.assignment_array(plan, list(range(k))) if k > 2 else spec.assignment_array(plan, sorted(set(plan.values())))
    return dict(n=spec.n, row=spec.row_ptr, col=spec.col_idx, pop=spec.pop,
                pos=None if spec.pos is None else spec.pos, k=k, n_steps=steps, assign=a)


def _lattices():
    sec11, frank = G.sec11_graph(), G.frank_graph()
    tri = G.triangular_graph(30, 58)
    dl = G.delaunay_graph(1500, seed=0)
    return {
        "sec11": _spec_case(sec11, 2, G.sec11_plan(2, sec11.nodes), 2000),
        "frank": _spec_case(frank, 2, G.frank_plan(0, frank.nodes), 2000),
        "triangular_k4": _spec_case(tri, 4, G.strip_plan(tri, 4), 1000),
        "delaunay_k6": _spec_case(dl, 6, G.bisection_plan(dl, 6), 1000),
    }


@pytest.mark.parametrize("name", ["sec11", "frank", "triangular_k4", "delaunay_k6"])
def test_sanitized_graph_and_oracle_on_workloads(harness, tmp_path, name):
    c = _lattices()[name]
    p = str(tmp_path / f"{name}.bin")
    _write(p, c["n"], c["row"], c["col"], c["pop"], pos=c["pos"], k=c["k"], n_steps=c["n_steps"], assign=c["assign"])
    out = _run(harness, p)
    assert "GRAPH" in out and "ORACLE rc=0" in out, out
    # the same graph without positions (no planar rings) and with the exact rule disabled
    p2 = str(tmp_path / f"{name}_nopos.bin")
    _write(p2, c["n"], c["row"], c["col"], c["pop"], pos=None, flags=1)
    assert "GRAPH" in _run(harness, p2)


def test_sanitized_delaunay_10k(harness, tmp_path):
    """C5's graph: 10^4 points, ring length up to 16."""
    dl = G.delaunay_graph(10000, seed=0)
    p = str(tmp_path / "dl10k.bin")
    _write(p, dl.n, dl.row_ptr, dl.col_idx, dl.pop, pos=dl.pos)
    out = _run(harness, p)
    assert "GRAPH n=10000" in out, out


def _grid_csr(w, h):
    spec = G.grid_graph(w, h)
    return spec


def _malformed():
    g = _grid_csr(4, 4)
    n, row, col, pop, pos = g.n, g.row_ptr.copy(), g.col_idx.copy(), g.pop.copy(), g.pos.copy()
    cases = {}
    r = row.copy(); r[3], r[4] = r[4], r[3]
    cases["row_ptr_decreasing"] = (n, r, col, pop, pos, "non-decreasing")
    c = col.copy(); c[5] = n + 7
    cases["col_out_of_range"] = (n, row, c, pop, pos, "out of range")
    c = col.copy(); c[-1] = -3
    cases["col_negative"] = (n, row, c, pop, pos, "out of range")
    c = col.copy(); c[row[2]] = 2
    cases["self_loop"] = (n, row, c, pop, pos, "self loop")
    c = col.copy(); c[row[1]] = c[row[1] + 1]
    cases["duplicate_edge"] = (n, row, c, pop, pos, "duplicate")
    c = col.copy(); c[row[0]] = 10  # 0-1 becomes 0-10: 10 does not list 0, 1 still lists 0
    cases["asymmetric"] = (n, row, c, pop, pos, "symmetric")
    r = row.copy(); r[-1] -= 1
    cases["odd_nnz"] = (n, r, col[:-1], pop, pos, "odd")
    r = row.copy(); r[0] = 1
    cases["row_ptr0_nonzero"] = (n, r, col, pop, pos, "row_ptr[0]")
    r = row.copy(); r[-1] += 40
    cases["row_ptr_overrun"] = (n, r, col, pop, pos, "REJECTED")
    cases["empty_graph"] = (0, np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32), None, "positive")
    # star with 20 leaves: degree above the device limit
    star_row = np.concatenate([[0, 20], 20 + np.arange(1, 21)]).astype(np.int32)
    star_col = np.concatenate([np.arange(1, 21), np.zeros(20)]).astype(np.int32)
    star_pos = np.concatenate([[[0.0, 0.0]], [[np.cos(t), np.sin(t)] for t in np.linspace(0, 6, 20)]])
    cases["degree_above_16"] = (21, star_row, star_col, np.ones(21, np.int32), star_pos, "degree")
    # positions that break the planar ring builder's assumptions: NaN, coincident, crossing
    p = pos.copy(); p[5] = [np.nan, 1.0]
    cases["nan_position"] = (n, row, col, pop, p, "finite")
    p = pos.copy(); p[6] = p[5]
    cases["coincident_positions"] = (n, row, col, pop, p, None)
    p = pos.copy(); p[[5, 10]] = p[[10, 5]]
    cases["crossing_edges"] = (n, row, col, pop, p, None)
    p = pos.copy() * 1e300
    cases["huge_positions"] = (n, row, col, pop, p, None)
    # K5: non-planar whatever the positions
    k5r = np.arange(0, 21, 4, dtype=np.int32)
    k5c = np.asarray([j for i in range(5) for j in range(5) if j != i], dtype=np.int32)
    k5p = np.asarray([[np.cos(2 * np.pi * i / 5), np.sin(2 * np.pi * i / 5)] for i in range(5)])
    cases["k5_nonplanar"] = (5, k5r, k5c, np.ones(5, np.int32), k5p, None)
    # two components
    two_r = np.asarray([0, 1, 2, 3, 4], np.int32)
    two_c = np.asarray([1, 0, 3, 2], np.int32)
    cases["disconnected"] = (4, two_r, two_c, np.ones(4, np.int32), np.asarray([[0, 0], [1, 0], [5, 0], [6, 0]], float),
                             None)
    return cases


@pytest.mark.parametrize("name", sorted(_malformed()))
def test_sanitized_malformed_inputs(harness, tmp_path, name):
    """Malformed CSR is rejected with a message, never read out of bounds; odd positions
    (NaN, coincident, crossing, huge, non-planar, disconnected) give a graph whose exactness
    bits the builder decides without undefined behaviour."""
    n, row, col, pop, pos, expect = _malformed()[name]
    p = str(tmp_path / f"{name}.bin")
    _write(p, n, row, col, pop, pos=pos)
    out = _run(harness, p)
    if expect is None:
        assert "GRAPH" in out or "REJECTED" in out, out
    else:
        assert "REJECTED" in out and expect in out, out
