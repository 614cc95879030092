"""first 2-step rollout chunk whose state differs from two futbol_step calls"""
import os, sys
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import gym_futbol_amd as gf
from helpers import v1_dense_cache
B, K = 512, 350
a = gf.make("Futbol2v2-v1", num_envs=B, seed=21)
b = gf.make("Futbol2v2-v1", num_envs=B, seed=21)
a.reset(); b.reset()
acts = a.random_actions_steps(K, 0, seed=5)
for k in range(0, K, 2):
    b.rollout(acts[k:k + 2])
    a.step(acts[k]); a.step(acts[k + 1])
    sa, sb = a.get_state(), b.get_state()
    diff = [f for f in sa if not np.array_equal(np.asarray(sa[f]), np.asarray(sb[f]))]
    if diff:
        print("chunk at step", k, "differs in", diff)
        nc = (sa["meta"].astype(np.uint64) >> np.uint64(8)) & np.uint64(0x3FF)
        x, y = sa["ckey"].reshape(-1, B), sb["ckey"].reshape(-1, B)
        for c, i in np.argwhere(x != y)[:6]:
            print("  entry", c, "env", i, "ncache", int(nc[i]), "a %#x b %#x" % (x[c, i], y[c, i]),
                  "a col", [hex(v) for v in x[:8, i]], "b col", [hex(v) for v in y[:8, i]])
            m = int(sa["meta"][i]); print("  meta a %#x b %#x steps %d" % (m, int(sb["meta"][i]), (m >> 18) & 0x3fff))
        x, y = sa["cjn"].reshape(-1, B), sb["cjn"].reshape(-1, B)
        for c, i in np.argwhere(x != y)[:4]:
            print("  jn entry", c, "env", i, "ncache", int(nc[i]), "a", x[:6, i], "b", y[:6, i])
        break
else:
    print("no difference")
