"""Diagnostic: first-step obs differences of the N=9 instance against the oracle (which envs / components)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd"), os.path.join(ROOT, "tests")]
import torch
from oracle import oracle as O
from gym_futbol_amd import FutbolVecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 9
B = 64
for dt in (torch.float64, torch.float32):
    venv = FutbolVecEnv("v1", B, device="cuda:0", seed=7 + n, dtype=dt, number_of_player=n)
    ora = O.V1Vec(B, N=n, seed=7 + n, portable=True)
    o_gpu = venv.reset().cpu().numpy(); o_cpu = ora.reset()
    print(dt, "reset equal", np.array_equal(o_gpu.astype(np.float64), o_cpu.astype(o_gpu.dtype).astype(np.float64)))
    for t in range(3):
        a = venv.random_actions(t, seed=1234)
        obs, rew, done, info = venv.step(a)
        o2, r2, d2, _ = ora.step(a.cpu().numpy().astype(np.int32))
        o1 = obs.cpu().numpy().astype(np.float64); o2 = o2.astype(obs.cpu().numpy().dtype).astype(np.float64)
        bad = np.argwhere(o1 != o2)
        print(" step", t, "n bad", len(bad), "envs", sorted(set(bad[:, 0].tolist()))[:20], "cols", sorted(set(bad[:, 1].tolist()))[:40])
        if len(bad):
            e, c = bad[0]
            print("  env", e, "col", c, "gpu", o1[e, c], "cpu", o2[e, c], "actions", a[e].cpu().numpy().tolist())
    venv.close()
