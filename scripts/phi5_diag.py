"""Diagnostic (GPU): where does the 5v5 float-output instance built with phi-node-folding
threshold 20 (libfutbol_amd_phi5.so) depart from its float64 twin?  Steps both side by side and
reports the first step, env, output fields and state fields that differ."""
import os
import sys

import numpy as np
import torch

os.environ.setdefault("FUTBOL_LIB_VARIANT", "phi5")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]
from gym_futbol_amd import FutbolVecEnv  # noqa: E402

n, B = 5, 128
a64 = FutbolVecEnv("v1", B, seed=3, dtype=torch.float64, number_of_player=n)
a32 = FutbolVecEnv("v1", B, seed=3, dtype=torch.float32, number_of_player=n)
a64.reset()
a32.reset()
for t in range(310):
    act = a64.random_actions(t)
    o64, r64, d64, _ = a64.step(act)
    o32, r32, d32, _ = a32.step(act)
    s64, s32 = a64.get_state(), a32.get_state()
    bad_state = [k for k in s64 if not np.array_equal(s64[k], s32[k])]
    bad_obs = ~(o64.float() == o32).all(1)
    bad_rew = r64.float() != r32
    bad_done = d64 != d32
    if bad_state or bool(bad_obs.any()) or bool(bad_rew.any()) or bool(bad_done.any()):
        print("first difference at step", t)
        print("state fields differing:", bad_state)
        for k in bad_state:
            d = np.nonzero(s64[k] != s32[k])[0]
            print("  %s: %d elements, first idx %s: f64-ctx %s f32-ctx %s" % (k, len(d), d[:8], s64[k][d[:4]], s32[k][d[:4]]))
        e = torch.nonzero(bad_obs | bad_rew | bad_done).flatten().cpu().numpy()
        print("envs with differing outputs:", e[:16], "count", len(e))
        if len(e):
            i = int(e[0])
            cols = torch.nonzero(o64[i].float() != o32[i]).flatten().cpu().numpy()
            print("env", i, "obs cols", cols, "f64", o64[i][cols].cpu().numpy(), "f32", o32[i][cols].cpu().numpy())
            print("env", i, "reward", float(r64[i]), float(r32[i]), "done", bool(d64[i]), bool(d32[i]))
            meta = int(s64["meta"][i])
            print("env", i, "meta f64-ctx %#x f32-ctx %#x" % (meta, int(s32["meta"][i])))
        break
else:
    print("no difference in 310 steps")
