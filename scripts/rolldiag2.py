"""dead arbiter-cache slots: step kernel vs rollout kernel vs another library's step kernel"""
import os, sys, subprocess
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd"), os.path.join(ROOT, "tests")]
import numpy as np
if len(sys.argv) > 2:  # child: one path, dump ckey
    import torch
    import gym_futbol_amd as gf
    B, K = 512, 350
    a = gf.make("Futbol2v2-v1", num_envs=B, seed=21)
    a.reset()
    acts = a.random_actions_steps(K, 0, seed=5)
    if sys.argv[1] == "roll":
        a.rollout(acts)
    else:
        for k in range(K):
            a.step(acts[k])
    s = a.get_state()
    np.savez(sys.argv[2], **{k: np.asarray(v) for k, v in s.items()})
    sys.exit(0)
runs = {}
for name, lib, mode in (("main_step", "", "step"), ("main_roll", "", "roll"), ("head_step", "head", "step"), ("head_roll", "head", "roll")):
    env = dict(os.environ, FUTBOL_LIB_VARIANT=lib)
    out = "/tmp/%s.npz" % name
    subprocess.check_call([sys.executable, __file__, mode, out], env=env)
    runs[name] = np.load(out)
names = list(runs)
for i in range(len(names)):
    for j in range(i + 1, len(names)):
        x, y = runs[names[i]], runs[names[j]]
        diff = [f for f in x.files if not np.array_equal(x[f], y[f])]
        print(names[i], "vs", names[j], "fields differing:", diff, [int((x[f] != y[f]).sum()) for f in diff])
