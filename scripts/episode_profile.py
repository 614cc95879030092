"""Per-step duration of the env-step launch over two episodes (all envs in lockstep from reset),
to see how the step cost varies with the episode phase.  Prints mean us per 25-step bucket."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]
import numpy as np
import torch
from gym_futbol_amd import FutbolVecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
B = 65536
v = FutbolVecEnv("v1", B, device="cuda:0", seed=0, dtype=torch.float32, number_of_player=n)
v.reset()
L = v.episode_steps
acts = torch.empty((2 * L, B, v.action_dim), dtype=torch.uint8, device="cuda:0")
for t in range(2 * L):
    v.random_actions(t, seed=1234, out=acts[t])
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * L + 1)]
s = torch.cuda.current_stream()
ev[0].record(s)
for t in range(2 * L):
    v.step_raw(acts[t])
    ev[t + 1].record(s)
torch.cuda.synchronize()
us = np.array([ev[t].elapsed_time(ev[t + 1]) * 1e3 for t in range(2 * L)])
out = {"players": n, "episode_steps": L, "mean_us": float(us.mean()),
       "bucket_us": [round(float(us[i:i + 25].mean()), 2) for i in range(0, 2 * L, 25)]}
print(json.dumps(out))
