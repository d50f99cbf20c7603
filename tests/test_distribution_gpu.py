"""The device chain (canonical Philox stream) against the native-RNG fixtures of the
reference's flip step -- see tests/test_distribution.py for the statistics and fixtures."""
import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig
from tests.test_distribution import CASES, assert_same_distribution, fixture, setup, summarize

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,bi", CASES)
def test_device_matches_native_rng(gpu, cfg, bi):
    fix = fixture(cfg)
    T, base = int(fix["T"]), float(fix["bases"][bi])
    spec, a0, lo, hi = setup(cfg)
    C = 4096
    run = FlipRun(FlipGraph(spec), np.stack([a0] * C),
                  RunConfig(seed=0xD15C0 + bi, pop_lo=lo, pop_hi=hi, base=base, diag_mask=_lib.FC_DIAG_WAIT))
    run.steps(T)
    st, fin = run.stats(), run.state()
    got = summarize(spec, fin, st["wait_cur"], st["sum_cut"], st["sum_nb"], T)
    assert_same_distribution(fix, bi, got, f"device {cfg}")
