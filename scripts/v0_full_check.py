"""Futbol-v0 (C3) at the benchmark's size against the portable oracle, every env bit for bit
(diagnostic; the -m gpu tests check 1 024 envs x 900 steps and the reference's own goldens):
B envs x T steps from reset, synthetic actions, obs / reward / done (+ terminal observations) compared
at every step, both opponent modes.  Prints one JSON line per mode.

    python scripts/v0_full_check.py --envs 65536 --steps 600
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import O  # noqa: E402


def run(B, T, random_opp, seed):
    from gym_futbol_amd import FutbolVecEnv
    venv = FutbolVecEnv("v0", B, seed=seed, dtype=torch.float64, random_opp=random_opp)
    ora = O.V0Vec(B, seed=seed, random_opp=random_opp, portable=True)
    first = None
    if not np.array_equal(venv.reset().cpu().numpy(), ora.reset()):
        first = 0
    t0 = time.perf_counter()
    shots = 0
    for t in range(T):
        if first is not None:
            break
        a = venv.random_actions(t)
        obs, rew, done, info = venv.step(a)
        o2, r2, d2, term2 = ora.step(a.cpu().numpy().astype(np.int32).reshape(-1))
        o1, r1, d1 = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        ok = (np.array_equal(d1, d2) and np.array_equal(r1.view(np.uint64), r2.view(np.uint64))
              and np.array_equal(o1.view(np.uint64), o2.view(np.uint64)))
        if ok and d1.any():
            ok = np.array_equal(info["terminal_observation"].cpu().numpy()[d1].view(np.uint64), term2[d1].view(np.uint64))
        if not ok:
            first = t + 1
        shots += int((o1[:, 4, 4] >= 4).sum())
    return {"kind": "v0", "random_opp": random_opp, "envs": B, "steps": T, "seed": seed,
            "first_divergence": first, "shots": shots, "seconds": round(time.perf_counter() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=600)
    a = ap.parse_args()
    bad = 0
    for random_opp in (False, True):
        r = run(a.envs, a.steps, random_opp, seed=11 + int(random_opp))
        print(json.dumps(r), flush=True)
        bad += r["first_divergence"] is not None
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
