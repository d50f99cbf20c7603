"""bench.py's measured HBM traffic (roofline.traffic): the counter passes of the same kernel at the
same launch shape and library build only -- profiles/pmc_traffic.json for C2, the newest
r*_side_pmc_<w>.json for the k > 2 side lines -- else null, with the refused summary named as
stale (a kernel name does not identify a revision)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _put(root, name, **kw):
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    json.dump(kw, open(os.path.join(root, "profiles", name), "w"))


def test_side_line_takes_newest_matching_profile(tmp_path):
    r = str(tmp_path)
    k = "void fc::flip_kernel<8, 2, 3, false, 2>(fc::KParams)"
    b = dict(build_id="B1")
    _put(r, "r04a_side_pmc_c3.json", workload="c3", kernel=k, chains=8192, chain_steps=20000, hbm_bytes_per_launch=1.0, **b)
    _put(r, "r05a_side_pmc_c3.json", workload="c3", kernel=k, chains=8192, chain_steps=20000, hbm_bytes_per_launch=2.0, **b)
    _put(r, "r05b_side_pmc_c3.json", workload="c3", kernel=k, chains=4096, chain_steps=20000, hbm_bytes_per_launch=3.0, **b)
    kn = "fc::flip_kernel<8, 2, 3, false, 2>"
    mt = lambda *a, bid="B1": bench.measured_traffic(*a, root=r, build_id=bid)  # noqa: E731
    assert mt("c3", kn, 8192, 20000) == (2.0, "profiles/r05a_side_pmc_c3.json", None)
    assert mt("c3", kn, 4096, 20000) == (3.0, "profiles/r05b_side_pmc_c3.json", None)
    assert mt("c3", kn, 8192, 10000) == (None, None, None)  # another launch shape
    assert mt("c3", "fc::flip_kernel<8, 4, 3, false, 2>", 8192, 20000) == (None, None, None)
    assert mt("c4", kn, 8192, 20000) == (None, None, None)
    # counters of another build: not this run's traffic, named as stale
    val, src, stale = mt("c3", kn, 8192, 20000, bid="B2")
    assert (val, src) == (None, None) and stale == {"profile": "profiles/r05a_side_pmc_c3.json", "build_id": "B1",
                                                    "hbm_bytes_per_launch": 2.0}


def test_c2_reads_pmc_traffic_json(tmp_path):
    r = str(tmp_path)
    k = "void fc::flip2_kernel<8, 4, false, false, false, false>(fc::KParams)"
    _put(r, "pmc_traffic.json", workload="c2", kernel=k, chains=4096, chain_steps=100000, hbm_bytes_per_launch=5.0,
         build_id="B1")
    _put(r, "r05a_side_pmc_c2.json", workload="c2", kernel=k, chains=4096, chain_steps=100000, hbm_bytes_per_launch=9.0,
         build_id="B1")
    kn = "fc::flip2_kernel<8, 4, false, false, false, false>"
    assert bench.measured_traffic("c2", kn, 4096, 100000, root=r, build_id="B1") == (5.0, "profiles/pmc_traffic.json", None)
    assert bench.measured_traffic("c2", kn, 2048, 100000, root=r, build_id="B1") == (None, None, None)
    assert bench.measured_traffic("c2", kn, 4096, 100000, root=r)[:2] == (None, None)  # no build id: refused


def test_committed_profiles_cover_the_bench_lines():
    """Committed counter summaries exist for the default bench line and the side lines (of this
    build, or named as stale when the sources changed since)."""
    for args in (("c2", "fc::flip2_kernel<8, 4, false, false, false, false>", 4096, 100000),
                 ("c3", "fc::flip_kernel<8, 2, 3, false, 2>", 8192, 20000),
                 ("c4", "fc::flip_kernel<8, 2, 3, false, 1>", 2816, 20000),
                 ("c5", "fc::flip_kernel<16, 4, 3, false, 1>", 2816, 20000)):
        val, _, stale = bench.measured_traffic(*args, build_id="current")
        assert val or stale, args
