"""The instance matrix of tests/test_gpu_instances.py at a larger workload (diagnostic): every compiled
step-kernel instance of the given team sizes (f64 / f32 outputs x default / runtime geometry x one step
/ open-loop rollout), B envs x T steps from reset, obs / reward / done bit for bit against the portable
oracle (which steps the envs on all host threads).  Prints one JSON line per instance.

  python scripts/diag_instance_big.py --players 9 --envs 2048 --steps 320
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import O  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", default="9")
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=320)
    ap.add_argument("--chunk", type=int, default=40, help="rollout launch length")
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 8))
    a = ap.parse_args()
    from gym_futbol_amd import FutbolVecEnv
    B, T = a.envs, a.steps
    bad = 0
    for n in [int(x) for x in a.players.split(",")]:
        seed = 31 + n
        gen = FutbolVecEnv("v1", B, seed=seed, number_of_player=n)
        acts = gen.random_actions_steps(T, 0, seed=5)
        gen.close()
        a_np = acts.cpu().numpy().astype(np.int32)
        t0 = time.time()
        ora = O.V1Vec(B, N=n, seed=seed, portable=True)
        ref0 = ora.reset()
        ro, rr, rd = [], [], []
        for t in range(T):
            o, r, d, _ = ora.step(a_np[t], nthreads=a.threads)
            ro.append(o)
            rr.append(r)
            rd.append(np.asarray(d, bool))
        ref = (np.stack(ro), np.stack(rr), np.stack(rd))
        t_ora = time.time() - t0
        for dtype in (torch.float64, torch.float32):
            npdt = np.float64 if dtype == torch.float64 else np.float32
            want = (ref[0].astype(npdt), ref[1].astype(npdt), ref[2])
            for generic in (False, True):
                os.environ["FUTBOL_GENERIC"] = "1" if generic else "0"
                for rollout in (False, True):
                    venv = FutbolVecEnv("v1", B, seed=seed, dtype=dtype, number_of_player=n)
                    o0 = venv.reset().cpu().numpy()
                    res = {"N": n, "dtype": "f64" if dtype == torch.float64 else "f32",
                           "geometry": "generic" if generic else "default", "launch": "rollout" if rollout else "step",
                           "envs": B, "steps": T, "oracle_s": round(t_ora, 1)}
                    first = None
                    if not np.array_equal(o0.view(np.uint8), ref0.astype(npdt).view(np.uint8)):
                        first = ("reset obs", -1, -1)
                    t = 0
                    while t < T and first is None:
                        k = min(a.chunk, T - t) if rollout else 1
                        if rollout and k > 1:
                            obs, rew, done, _ = venv.rollout(acts[t:t + k])
                        else:
                            o_, r_, d_, _ = venv.step(acts[t])
                            obs, rew, done = o_[None], r_[None], d_[None]
                        g = (obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool))
                        for what, gg, ww in zip(("obs", "reward", "done"), g, (w[t:t + k] for w in want)):
                            gg = gg.reshape(ww.shape)
                            diff = (gg != ww) if what == "done" else \
                                (gg.view(np.uint8).reshape(gg.shape + (-1,)) != ww.view(np.uint8).reshape(ww.shape + (-1,))).any(-1)
                            if diff.any():
                                w0 = np.argwhere(diff)[0].tolist()
                                first = (what, t + w0[0], w0[1])
                                res["differing_entries"] = int(diff.sum())
                                break
                        t += k
                    venv.close()
                    res["first_divergence"] = first
                    bad += first is not None
                    print(json.dumps(res), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
