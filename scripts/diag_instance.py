"""Locate the first divergence of one envs_v1 step-kernel instance from the oracle (diagnostic).

Runs the same workload as tests/test_gpu_instances.py (B envs, seed 31 + N, actions
random_actions_steps(T, 0, seed=5)) on one instance of the library selected by FUTBOL_LIB_VARIANT, and
compares the full state (p, v, v_bias of every body, the arbiter cache, meta) with the portable oracle:
  step instance:    after every step;
  rollout instance: a fresh context per prefix length k (k = 2, 3, ...), one rollout launch of k steps,
                    state compared after it (the state in the middle of a launch is not observable).
Prints one JSON line per compared point with the differing fields and envs, and stops after the
first divergent point (+ --extra more).  TEST / DIAGNOSTIC INFRASTRUCTURE (uses the oracle).

  FUTBOL_LIB_VARIANT=kx6 python scripts/diag_instance.py --n 5 --dtype f32 --generic 1 --rollout 1 --T 8
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import O, v1_dense_cache, v1_oracle_bodies, v1_oracle_dense_cache  # noqa: E402
import torch  # noqa: E402


def state_diff(venv, ora, n, B):
    st = venv.get_state()
    ob = v1_oracle_bodies(ora.envs, n, B)
    nb = 2 * n + 1
    out = {}
    for f in ("px", "py", "vx", "vy", "bx", "by"):
        g = st[f].reshape(nb, B).view(np.uint64)
        w = ob[f].reshape(nb, B).view(np.uint64)
        bad = np.argwhere(g != w)
        if len(bad):
            k, i = bad[0]
            out[f] = {"count": int(len(bad)), "envs": sorted(set(int(x) for x in bad[:, 1]))[:16],
                      "first": [int(k), int(i), float(st[f].reshape(nb, B)[k, i]), float(ob[f].reshape(nb, B)[k, i])]}
    ex, age, jn = v1_dense_cache(st, n, B)
    ex2, age2, jn2 = v1_oracle_dense_cache(ora.envs, n, B)
    for name, a, b in (("cache_members", ex, ex2), ("cache_age", np.where(ex, age, -1), np.where(ex2, age2, -1)),
                       ("cache_jn", np.where(ex, jn, 0.0).view(np.uint64), np.where(ex2, jn2, 0.0).view(np.uint64))):
        bad = np.argwhere(a != b)
        if len(bad):
            out[name] = {"count": int(len(bad)), "envs": sorted(set(int(x) for x in bad[:, 0]))[:16],
                         "first": [int(x) for x in bad[0]]}
    meta = st["meta"].astype(np.uint64)
    owner = (meta & np.uint64(7)).astype(np.int64)
    ev = (meta >> np.uint64(32)).astype(np.int64)
    for name, a, b in (("owner", owner, np.array([ora.envs[i].owner for i in range(B)])),
                       ("event", ev, np.array([ora.envs[i].event for i in range(B)]))):
        bad = np.flatnonzero(a != b)
        if len(bad):
            out[name] = {"count": int(len(bad)), "envs": [int(x) for x in bad[:16]]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--generic", type=int, default=0)
    ap.add_argument("--rollout", type=int, default=0)
    ap.add_argument("--B", type=int, default=96)
    ap.add_argument("--T", type=int, default=60)
    ap.add_argument("--k0", type=int, default=2, help="rollout: first prefix length")
    ap.add_argument("--extra", type=int, default=0)
    a = ap.parse_args()
    os.environ["FUTBOL_GENERIC"] = "1" if a.generic else "0"
    from gym_futbol_amd import FutbolVecEnv
    n, B, T = a.n, a.B, a.T
    seed = 31 + n
    dtype = torch.float64 if a.dtype == "f64" else torch.float32
    gen = FutbolVecEnv("v1", B, seed=seed, number_of_player=n)
    acts = gen.random_actions_steps(T, 0, seed=5)
    gen.close()
    a_np = acts.cpu().numpy().astype(np.int32)
    tag = dict(n=n, dtype=a.dtype, generic=a.generic, rollout=a.rollout, B=B,
               variant=os.environ.get("FUTBOL_LIB_VARIANT", ""))
    left = a.extra + 1
    if not a.rollout:
        venv = FutbolVecEnv("v1", B, seed=seed, dtype=dtype, number_of_player=n)
        ora = O.V1Vec(B, N=n, seed=seed, portable=True)
        venv.reset()
        ora.reset()
        for t in range(T):
            venv.step(acts[t])
            ora.step(a_np[t])
            d = state_diff(venv, ora, n, B)
            if d:
                print(json.dumps(dict(tag, step=t, diff=d, invalid_hex=hex(venv.invalid_actions()))), flush=True)
                left -= 1
                if not left:
                    break
        else:
            print(json.dumps(dict(tag, step=T, diff={})), flush=True)
        venv.close()
        return
    ora = O.V1Vec(B, N=n, seed=seed, portable=True)
    ora.reset()
    done_steps = 0
    for k in range(a.k0, T + 1):
        while done_steps < k:
            ora.step(a_np[done_steps])
            done_steps += 1
        venv = FutbolVecEnv("v1", B, seed=seed, dtype=dtype, number_of_player=n)
        venv.reset()
        venv.rollout(acts[:k])
        d = state_diff(venv, ora, n, B)
        inv = venv.invalid_actions()
        venv.close()
        if d:
            print(json.dumps(dict(tag, steps=k, diff=d, invalid_hex=hex(inv))), flush=True)
            left -= 1
            if not left:
                break
    else:
        print(json.dumps(dict(tag, steps=T, diff={})), flush=True)


if __name__ == "__main__":
    main()
