"""bench.py --gpus N forms N ranks by itself (VERDICT r03 "next" #1): without WORLD_SIZE in the
environment the parent starts N child processes of bench.py (rank r on LOCAL_RANK r, rendezvous at
127.0.0.1) before anything touches the GPU, relays rank 0's line and fails if any rank fails.  The
self-test path forms a gloo world on the CPU and all-reduces rank + 1."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(extra), capture_output=True,
                          text=True, timeout=180, env=env)


def test_launcher_forms_gloo_world_of_two():
    r = _run("--gpus", "2", "--launcher-selftest")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["ranks"] == 2 and d["sum"] == 3.0 and d["master_addr"] == "127.0.0.1"
    assert sorted(d["local_ranks"]) == [0, 1]


def test_launcher_fails_when_a_rank_fails():
    r = _run("--gpus", "3", "--launcher-selftest", "--launcher-selftest-fail-rank", "1")
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr
