"""CPU checks of bench.py's reporting helpers (the GPU timing itself runs only on the box):
the algorithmic bytes per env-step of SURVEY.md 8(d), the committed PMC traffic lookup, and the
cpu_baseline record (the oracle on the host's threads and on one thread)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]
import bench  # noqa: E402


def test_algorithmic_bytes_match_survey():
    # 579 B (2v2), 1 257 B (5v5) per envs_v1 env-step, 554 B per v0 env-step,
    # with float32 observations
    assert bench.algo_bytes_per_env_step("v1", 2, 4) == 579
    assert bench.algo_bytes_per_env_step("v1", 5, 4) == 1257
    assert bench.algo_bytes_per_env_step("v0", 2, 4) == 554


@pytest.mark.parametrize("n", [2, 5])
def test_committed_traffic_entry(n):
    traffic, src = bench.pmc_traffic("v1", n, 65536)
    assert src is not None and src.startswith("profiles/")
    algo = bench.algo_bytes_per_env_step("v1", n, 4) * 65536
    # measured HBM bytes per launch: at least the algorithmic ones (the arbiter cache and spill
    # area come on top), and not wildly more
    assert algo <= traffic < 1.5 * algo


def test_cpu_threads_all_host_cores(monkeypatch):
    # the restatement on ALL host cores -- the affinity mask, whatever OMP_NUM_THREADS says
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_threads() == len(os.sched_getaffinity(0))
    assert bench.omp_share() == 3
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.omp_share() is None


@pytest.mark.parametrize("kind", ["v1", "v0"])
def test_cpu_baseline_record(kind, monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    r = bench.cpu_baseline(kind, 2, budget_s=0.2, B=256)
    T = len(os.sched_getaffinity(0))
    assert r["unit"] == "env-steps/s" and r["kind"] == "port"
    assert r["all_cores"]["threads"] == T and r["all_cores"]["value"] > 0
    assert r["single_thread"]["threads"] == 1 and r["single_thread_value"] > 0
    if T != 2:
        assert r["omp_share"]["threads"] == 2 and r["omp_share"]["value"] > 0
    runs = [x for x in (r["all_cores"], r["omp_share"], r["quota_run"]) if x]
    best = max(runs, key=lambda x: x["value"])  # the reported baseline is the host's best configuration
    assert r["value"] == best["value"] and r["cores"] == best["threads"]
    assert "%d OpenMP threads" % r["cores"] in r["sample"]
    assert r["host"]["nproc"] >= 1 and "reference_v0_python" in r
    if kind == "v1":
        c1 = r["c1"]  # 1 env, 1 thread, 100 000 steps
        assert c1["envs"] == 1 and c1["cores"] == 1 and c1["steps"] == 100000 and c1["value"] > 0
        assert c1["episodes"] == 100000 // 300  # fixed 300-step episodes


def test_vec_run_matches_single_env_runs():
    # the all-core loop is orc_v1_run per env: same episodes and returns whatever the thread count
    from oracle import oracle as O
    import ctypes as C
    a = O.V1Vec(16, N=2, seed=3)
    a.reset()
    eps_a, ret_a = a.run(650, 1234, 4)
    L = O.lib()
    eps_b, ret_b = 0, 0.0
    for i in range(16):
        e = O.OrcV1()
        L.orc_v1_init(C.byref(e), 2, 105.0, 68.0, 30.0, 3, i)
        import numpy as np
        L.orc_v1_reset(C.byref(e), np.zeros(20).ctypes.data)
        r = C.c_double()
        eps_b += L.orc_v1_run(C.byref(e), 650, 1234, C.byref(r))
        ret_b += r.value
    assert eps_a == eps_b == 16 * 2 and abs(ret_a - ret_b) <= 1e-9 * max(1.0, abs(ret_b))


def test_metric_labels_per_config():
    # the headline metric is BASELINE.json's, and only the 2v2 envs_v1 config carries it
    import json
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert bench.metric_of("v1", 2, 65536) == json.load(f)["metric"]
    assert "5v5" in bench.metric_of("v1", 5, 65536) and bench.metric_of("v1", 5, 65536) != bench.METRIC
    assert "hard-coded" in bench.metric_of("v0", 2, 65536)
    assert bench.workload_of("v1", 2, 65536, 1).startswith("C2:")
    assert bench.workload_of("v1", 2, 65536, 8).startswith("C4:")
    assert bench.workload_of("v1", 5, 65536, 1).startswith("C5:")
    assert bench.workload_of("v0", 2, 65536, 1).startswith("C3:")


def test_c1_line():
    import json
    import subprocess
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--kind", "c1"], capture_output=True,
                         text=True, timeout=300, check=True).stdout.strip().splitlines()
    line = json.loads(out[-1])
    assert line["n_gpus"] == 0 and line["steps"] == 100000 and line["value"] > 0
    assert line["host"]["cpu_model"] is not None or line["host"]["nproc"] >= 1
