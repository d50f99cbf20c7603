"""The RCCL branch of the one statistics reduction on real hardware.

Multi-rank runs on the CPU use gloo (tests/test_distributed.py); the 8-GPU bench uses backend
"nccl" (RCCL on ROCm) with device tensors.  A world-size-1 process group on the box's GPU runs
that branch here: ``force=True`` makes ``distributed.allreduce_*`` and ``Sweep.grouped`` call the
collectives instead of short-circuiting at one rank, on int64 SUM, int64 MAX and float64 MAX
device tensors.  At one rank a reduction is the identity, so every result must equal the
host-side numpy reduction of the same per-chain data bit for bit.

It runs in a fresh process (tests/rccl_worker.py) that starts torch's HIP runtime before loading
the flip-chain library, the order of bench.py's N > 1 path: one HIP runtime per process (the
pytest process has already loaded the library, and a second runtime there finds no GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_collectives_and_sweep_grouped(gpu):
    res = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py")], capture_output=True, text=True,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["backend"] == "nccl"
    bad = [k for k, v in out["checks"].items() if not v]
    assert not bad, (bad, out)
    ops = {(op, dt) for op, dt, dev in out["collective_calls"]}
    assert all(dev.startswith("cuda") for _, _, dev in out["collective_calls"])
    assert any("SUM" in op and "int64" in dt for op, dt in ops)
    assert any("MAX" in op and "int64" in dt for op, dt in ops)
    assert any("MAX" in op and "float64" in dt for op, dt in ops)
