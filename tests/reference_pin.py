"""Statistical pin against the reference's own artifacts.

Every one of the 174 reference configurations -- 150 sec11 ``{alignment}B{100 base}P{100 pop}``
(``grid_chain_sec11.py:182-184``: 5 pops x 10 bases x 3 alignments) and 24 FRANK
(``Frankenstein_chain.py:182-184``) -- is re-run for 100,000 yields (``total_steps=100000``,
``:342``) with the reference's graph, start plan, population bound and base.  The runs are
compared with what the reference wrote:

* ``wait.txt`` (``:410-411``): per (graph, base, pop) the mean of our sums against the mean of
  the reference's three (one per alignment), as a z-score whose sigma is pooled over every pop
  of that base (within-group deviations of both samples); and per (graph, base) pooled over the
  pops;
* the final ``|cut edges|`` and ``|b_nodes|`` per (graph, base) against the decoded
  ``*end2.png`` final states (``:440-450``), two-sample KS.

Used by ``test_oracle_golden.py`` (the C oracle) and ``test_reference_pin_gpu.py`` (the device).
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Tuple

import numpy as np

from flipcomplexityempirical_amd import graphs as G

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_artifacts.npz")
Z_MAX = 4.0          # |z| bound per group (58 (graph, base, pop) groups; observed max ~2.8)
KS_P_MIN = 1e-3


def parse(key: str) -> Tuple[int, int, int]:
    m = re.match(r"^(\d)B(\d+)P(\d+)$", key)
    return int(m.group(1)), int(m.group(2)), int(m.group(3))


def configs() -> List[Tuple[str, int, float, float, str]]:
    """(graph, alignment, base, pop, key) of every reference artifact, with the exact float
    base / pop the reference used (``int(100 * x)`` names the file, :323)."""
    gold = np.load(GOLD)
    out = []
    for tag, bases, pops in (("sec11", G.SEC11_BASES, G.SEC11_POPS), ("frank", G.FRANK_BASES, G.FRANK_POPS)):
        for key in gold[f"{tag}_keys"]:
            al, b, p = parse(str(key))
            base = [x for x in bases if int(100 * x) == b]
            pct = [x for x in pops if int(100 * x) == p]
            assert len(base) == 1 and len(pct) == 1, key
            out.append((tag, al, base[0], pct[0], str(key)))
    return out


def spec_of(tag: str):
    return G.sec11_graph() if tag == "sec11" else G.frank_graph()


def start_plan(spec, tag: str, al: int) -> np.ndarray:
    plan = (G.sec11_plan if tag == "sec11" else G.frank_plan)(al, spec.nodes)
    return spec.assignment_array(plan, [-1, 1])


def decoded_end_states() -> Dict[Tuple[str, int], np.ndarray]:
    """(graph, 100 base) -> [n, 2] final (|cut|, |B|) of the reference's decoded end2 states."""
    gold = np.load(GOLD)
    out: Dict[Tuple[str, int], list] = {}
    for tag in ("sec11", "frank"):
        spec = spec_of(tag)
        for key, img in zip(gold[f"{tag}_keys"], gold[f"{tag}_end"]):
            _, b, _ = parse(str(key))
            a = np.zeros(spec.n, dtype=np.int8)
            for i, nd in enumerate(spec.nodes):
                a[i] = 0 if img[nd[0], nd[1] + (19 if tag == "frank" else 0)] == -1 else 1
            c, nb, _ = G.cut_and_boundary(spec, a)
            out.setdefault((tag, b), []).append((c, nb))
    return {k: np.asarray(v) for k, v in out.items()}


def check(results: List[Tuple[Tuple, int, int, int]]) -> Dict[str, float]:
    """``results``: ((graph, alignment, base, pop, key), sum_wait, final cut, final |B|) per
    run.  Asserts the pins above; returns the worst statistics for the record."""
    from scipy import stats
    gold = np.load(GOLD)
    ref_w: Dict[Tuple, list] = {}
    for tag in ("sec11", "frank"):
        for key, w in zip(gold[f"{tag}_keys"], gold[f"{tag}_wait"]):
            _, b, p = parse(str(key))
            ref_w.setdefault((tag, b, p), []).append(float(w))
    our_w: Dict[Tuple, list] = {}
    our_end: Dict[Tuple, list] = {}
    for (tag, al, base, pct, key), w, cut, nb in results:
        _, b, p = parse(key)
        our_w.setdefault((tag, b, p), []).append(float(w))
        our_end.setdefault((tag, b), []).append((cut, nb))
    assert set(our_w) == set(ref_w), "every (graph, base, pop) group of the reference is re-run"
    # sigma per (graph, base): within-group deviations of both samples, pooled over the pops
    sig = {}
    for gb in {k[:2] for k in ref_w}:
        dev, dof = [], 0
        for k in ref_w:
            if k[:2] != gb:
                continue
            for xs in (our_w[k], ref_w[k]):
                x = np.asarray(xs)
                dev.append(x - x.mean())
                dof += x.size - 1
        sig[gb] = float(np.sqrt(np.sum(np.concatenate(dev) ** 2) / dof))
    worst_z = 0.0
    for k in sorted(ref_w):
        o, r = np.asarray(our_w[k]), np.asarray(ref_w[k])
        z = (o.mean() - r.mean()) / (sig[k[:2]] * np.sqrt(1 / o.size + 1 / r.size))
        assert abs(z) <= Z_MAX, ("wait.txt mean", k, o.mean(), r.mean(), z)
        worst_z = max(worst_z, abs(z))
    for gb in sorted(sig):
        o = np.concatenate([our_w[k] for k in our_w if k[:2] == gb])
        r = np.concatenate([ref_w[k] for k in ref_w if k[:2] == gb])
        z = (o.mean() - r.mean()) / (sig[gb] * np.sqrt(1 / o.size + 1 / r.size))
        assert abs(z) <= Z_MAX, ("wait.txt mean per base", gb, o.mean(), r.mean(), z)
    ends = decoded_end_states()
    worst_p = 1.0
    for gb, r in sorted(ends.items()):
        o = np.asarray(our_end[gb])
        for j, what in enumerate(("final |cut|", "final |B|")):
            pv = stats.ks_2samp(o[:, j], r[:, j]).pvalue
            assert pv > KS_P_MIN, (what, gb, o[:, j].mean(), r[:, j].mean(), pv)
            worst_p = min(worst_p, pv)
    return {"max_abs_z": worst_z, "min_ks_p": worst_p}
