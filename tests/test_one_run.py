"""The planar run rule's loop-free ring test (``csrc/fc_ring.h``, used by both flip kernels)
against the interval-counting statement of the rule, exhaustively on rings of up to 10 cells
and on random rings of 11-16 (``tests/native/one_run_check.cpp``).  CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "flipcomplexityempirical_amd", "csrc")


def test_one_run_matches_interval_statement(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no host C++ toolchain")
    exe = str(tmp_path / "one_run_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC, "-o", exe,
                    os.path.join(HERE, "native", "one_run_check.cpp")], check=True)
    res = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.strip().endswith("bad 0")
