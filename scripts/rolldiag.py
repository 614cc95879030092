import os, sys
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import gym_futbol_amd as gf
B, K = 512, int(sys.argv[1]) if len(sys.argv) > 1 else 350
a = gf.make("Futbol2v2-v1", num_envs=B, seed=21)
b = gf.make("Futbol2v2-v1", num_envs=B, seed=21)
a.reset(); b.reset()
acts = a.random_actions_steps(K, 0, seed=5)
obs, rew, done, term = b.rollout(acts)
for k in range(K):
    a.step(acts[k])
sa, sb = a.get_state(), b.get_state()
for f in sa:
    x, y = np.asarray(sa[f]), np.asarray(sb[f])
    if not np.array_equal(x, y):
        d = np.nonzero((x != y).reshape(x.shape[0], -1).any(1) if x.ndim > 1 else (x != y))[0]
        print("field", f, "shape", x.shape, "ndiff", len(d), "first idx", d[:10])
        i = d[0]
        print("   a:", x.reshape(x.shape[0], -1)[i][:8] if x.ndim > 1 else x[d[:6]], "b:", y.reshape(y.shape[0], -1)[i][:8] if y.ndim > 1 else y[d[:6]])
print("done K", K)
from helpers import v1_dense_cache
exa, aga, jna = v1_dense_cache(sa, 2, B)
exb, agb, jnb = v1_dense_cache(sb, 2, B)
print("live membership equal", np.array_equal(exa, exb), "ages equal", np.array_equal(aga[exa], agb[exb]) if np.array_equal(exa, exb) else None,
      "jn equal", np.array_equal(jna[exa], jnb[exb]) if np.array_equal(exa, exb) else None)
bad = np.nonzero((exa != exb).any(1))[0]
print("envs with different live cache", bad[:10])
nc = (sa["meta"].astype(np.uint64) >> np.uint64(8)) & np.uint64(0x3FF)
for f in ("ckey",):
    x, y = sa[f].reshape(-1, B), sb[f].reshape(-1, B)
    d = np.argwhere(x != y)
    for c, i in d[:8]:
        print("entry", c, "env", i, "ncache", int(nc[i]), "a %#x b %#x" % (x[c, i], y[c, i]))
