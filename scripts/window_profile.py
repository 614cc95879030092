"""Where the driver's short timed region (K = 20 steps) loses time: one hipGraph of K step launches
replayed back to back through two episodes (all envs in lockstep from reset; fresh synthetic
actions per window, drawn untimed into the graph's input buffer), each replay timed twice -- HIP
events around it on the replay stream (the GPU's time for the K steps, inter-kernel gaps included)
and host wall time from a synchronized start to the synchronize after it (what bench.py's timed
region measures).  Prints per-window us per step for both and their difference
(the fixed launch + synchronize cost of one region).

    python scripts/window_profile.py [players] [K]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gym_futbol_amd import FutbolVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B = 65536
dev = torch.device("cuda:0")
v = FutbolVecEnv("v1", B, device=dev, seed=0, dtype=torch.float32, number_of_player=n)
v.reset()
L = v.episode_steps
abuf = torch.empty((K, B, v.action_dim), dtype=torch.uint8, device=dev)
v.random_actions_steps(K, 0, seed=1234, out=abuf)
s = torch.cuda.Stream(dev)
main = torch.cuda.current_stream(dev)
g = torch.cuda.CUDAGraph()
s.wait_stream(main)
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        for t in range(K):
            v.step_raw(abuf[t])
main.wait_stream(s)
torch.cuda.synchronize(dev)
# back to the episode start: the capture did not run the steps, reset puts every env at step 0
v.reset()
torch.cuda.synchronize(dev)
with torch.cuda.stream(s):
    g.replay()  # the first replay pays the graph's upload
torch.cuda.synchronize(dev)
v.reset()
torch.cuda.synchronize(dev)
nwin = (2 * L) // K
ev_us, wall_us = [], []
for w in range(nwin):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # fresh actions for every window (untimed): replaying one K-step action pattern over and over
    # drives the players into the walls and makes the mid-episode steps contact-heavy (40 us)
    v.random_actions_steps(K, w * K, seed=1234, out=abuf)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        e0.record(s)
        g.replay()
        e1.record(s)
    torch.cuda.synchronize(dev)
    wall_us.append((time.perf_counter() - t0) * 1e6)
    ev_us.append(e0.elapsed_time(e1) * 1e3)
ev_us, wall_us = np.array(ev_us), np.array(wall_us)
out = {"players": n, "K": K, "episode_steps": L,
       "window_start_step": [(w * K) % L for w in range(nwin)],
       "events_us_per_step": [round(float(x) / K, 2) for x in ev_us],
       "wall_us_per_step": [round(float(x) / K, 2) for x in wall_us],
       "fixed_us_per_region": [round(float(a - b), 1) for a, b in zip(wall_us, ev_us)],
       "mean_events_us_per_step": float(ev_us.mean() / K), "mean_wall_us_per_step": float(wall_us.mean() / K),
       "median_fixed_us": float(np.median(wall_us - ev_us))}
print(json.dumps(out))
