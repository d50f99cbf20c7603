"""bench.py's rank handling on CPU: ``--gpus N`` run directly launches N
ranks itself, and a launcher whose WORLD_SIZE disagrees with ``--gpus`` is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update({k: str(v) for k, v in kw.items()})
    return env


def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE=3, RANK=0, LOCAL_RANK=0),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=3" in r.stderr
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=_env(WORLD_SIZE=8, RANK=0, LOCAL_RANK=0),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr


def test_gpus_n_launches_n_ranks():
    for n in (2, 3):
        r = subprocess.run([sys.executable, BENCH, "--gpus", str(n)], env=_env(FC_BENCH_SPAWN_PROBE=1),
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout  # rank 0 alone prints
        rec = json.loads(lines[0])
        devs = rec.pop("devices")
        assert rec == {"ranks_seen": n, "rank_sum": float(n * (n - 1) // 2), "launcher": "bench.py"}
        # every rank's device identity, and that they are distinct
        assert [d["rank"] for d in devs["per_rank"]] == list(range(n)) and devs["distinct"] is True
        assert [d["local_rank"] for d in devs["per_rank"]] == list(range(n))


def test_failing_rank_fails_the_launch():
    # every rank dies at the rendezvous (no such backend): the parent returns non-zero, no hang
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "c2"],
                       env=_env(FC_BENCH_BACKEND="no_such_backend", FC_BENCH_DEVICE=0),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
