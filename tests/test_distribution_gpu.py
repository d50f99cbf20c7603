"""The device chain (canonical Philox stream) against the native-RNG fixtures of the
reference's flip step -- see tests/test_distribution.py for the statistics and fixtures."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
from flipcomplexityempirical_amd import graphs as G
from tests.test_distribution import (C3_K, CASES, assert_same_distribution, assert_same_distribution_c3, fixture,
                                     setup, setup_c3, summarize, summarize_c3)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,bi", CASES)
def test_device_matches_native_rng(gpu, cfg, bi):
    fix = fixture(cfg)
    T, base = int(fix["T"]), float(fix["bases"][bi])
    spec, a0, lo, hi = setup(cfg)
    C = 4096
    shape = cfg != "c1"
    diag = _lib.FC_DIAG_WAIT | (_lib.FC_DIAG_SERIES if shape else 0)
    run = FlipRun(FlipGraph(spec), np.stack([a0] * C),
                  RunConfig(seed=0xD15C0 + bi, pop_lo=lo, pop_hi=hi, base=base, diag_mask=diag,
                            event_cap=T + 1 if shape else 0))
    run.steps(T)
    st, fin = run.stats(), run.state()
    got = summarize(spec, fin, st["wait_cur"], st["sum_cut"], st["sum_nb"], T)
    if shape:
        # the interface angle after every accepted flip, from the device's frame-series kernel
        # (fc_run_frame_series: boundary_slope + the driver's angle line), weighted by the
        # yields each state lasts
        frame = G.slope_frame(spec, "sec11")
        am, ae = np.full(C, np.nan), np.full(C, np.nan)
        for c0 in range(0, C, 1024):  # chunks of chains (10,000-step windows: 10^4 events each)
            fs = run.frame_series(frame, chains=range(c0, c0 + 1024))
            for j in range(1024):
                c = c0 + j
                ev = run.events(c)
                n = int(fs["len"][j])
                assert n == ev.size + 1
                w = np.diff(np.concatenate([[0], ev["t"], [T + 1]]))
                ang, two = fs["angle"][j, :n], fs["n_cut"][j, :n] == 2
                if two.any():
                    am[c] = float(np.sum(ang[two] * w[two]) / np.sum(w[two]))
                ae[c] = ang[-1] if two[-1] else np.nan
        got["angle_mean"], got["angle_end"] = am, ae
    assert_same_distribution(fix, bi, got, f"device {cfg}")


@pytest.mark.parametrize("bi", [0, 1])
def test_device_c3_matches_native_rng_pair(gpu, bi):
    """C3 at its per-GPU production shape (8192 chains; the general-k kernel with the multi-flip
    commit, canonical Philox PAIR stream) against the reference's pair proposal under native RNG
    (native_rng_c3.npz): KS on the end state's cut, boundary, population and shape statistics,
    the time-averaged cut and boundary, and the geometric wait."""
    fix = fixture("c3")
    T, base = int(fix["T"]), float(fix["bases"][bi])
    spec, a0, lo, hi = setup_c3()
    C = 8192
    run = FlipRun(FlipGraph(spec), np.stack([a0] * C),
                  RunConfig(k=C3_K, labels=tuple(range(C3_K)), proposal=_lib.FC_PROPOSE_PAIR, seed=0xC3C3 + bi,
                            pop_lo=lo, pop_hi=hi, base=base, diag_mask=_lib.FC_DIAG_WAIT))
    run.steps(T)
    st, fin = run.stats(), run.state()
    assert int(st["steps"].min()) == T
    got = summarize_c3(spec, fin, st["wait_cur"], st["sum_cut"], st["sum_nb"], T)
    assert_same_distribution_c3(fix, bi, got, "device c3")
