"""Fixed cost of a short timed region (the driver's K = 20 bench line): wall time of
(graph replay + synchronize) for graphs of n step launches at the same episode phase (every
measurement starts 140 steps after a reset), n = 1, 2, 20; the fixed cost is the intercept."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gym_futbol_amd import FutbolVecEnv  # noqa: E402

B = 65536
v = FutbolVecEnv("v1", B, device="cuda:0", seed=0, dtype=torch.float32, number_of_player=2)
acts = v.random_actions_steps(200, 0, seed=7)
s = torch.cuda.Stream()
graphs = {}
for n in (1, 2, 20):
    g = torch.cuda.CUDAGraph()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in range(n):
                v.step_raw(acts[140 + t])
    torch.cuda.current_stream().wait_stream(s)
    graphs[n] = g
res = {n: [] for n in graphs}
for rep in range(12):
    for n, g in graphs.items():
        v.reset()
        for t in range(140):
            v.step_raw(acts[t])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        res[n].append(time.perf_counter() - t0)
for n in graphs:
    print("n=%2d  median %.1f us  min %.1f us" % (n, np.median(res[n]) * 1e6, min(res[n]) * 1e6))
m = {n: np.median(res[n]) * 1e6 for n in res}
per = (m[20] - m[2]) / 18
print("per step %.2f us, fixed %.1f us" % (per, m[2] - 2 * per))
