"""The benchmark's workload at its full size, on the GPU, EVERY env compared with the oracle at
every step: B = 65 536 envs per context (1 024 one-wave blocks: one wave per SIMD, every XCD),
float32 outputs (the bench's kernel instance), synthetic device actions, auto-reset across an
episode boundary -- C2 (2v2), C5 (5v5) and C3 (v0, hard-coded opponent); 10v10 (`Futbol-v1`) for 80
steps; and the open-loop rollout instance of 2v2 / 5v5 (two 30-step launches).

The portable oracle steps the same 65 536 global env ids beside the kernel (OpenMP over the box's
CPU share, ~10 s of oracle per config), and obs / reward / done (and the terminal observations of
the finishing envs) of all envs are compared bit for bit -- the f32 outputs against the oracle's
f64 values cast to f32.  The first diverging env and step are reported.
"""
import os

import numpy as np
import pytest
import torch

from helpers import O

pytestmark = pytest.mark.gpu
B = 65536
# the GPU box's CPU share (OMP_NUM_THREADS is set to it there); os.cpu_count() is the whole machine
NT = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1))


def _first_bad(eq_rows):
    bad = np.flatnonzero(~eq_rows)
    return int(bad[0]) if bad.size else None


def _check(kind, n, T, period):
    from gym_futbol_amd import FutbolVecEnv
    kw = {"number_of_player": n} if kind == "v1" else {"random_opp": False}
    seed = 21 + n
    venv = FutbolVecEnv(kind, B, seed=seed, dtype=torch.float32, **kw)
    if kind == "v1":
        ora = O.V1Vec(B, N=n, seed=seed, portable=True)
    else:
        ora = O.V0Vec(B, seed=seed, random_opp=False, portable=True)
    o = venv.reset().cpu().numpy().reshape(B, -1)
    o_ref = ora.reset().reshape(B, -1).astype(np.float32)
    assert np.array_equal(o.view(np.uint32), o_ref.view(np.uint32)), "reset obs differ"
    compared = 0
    for t in range(T):
        a = venv.random_actions(t, seed=777)
        obs, rew, done, info = venv.step(a)  # (asynchronous on the device while the oracle steps)
        a_np = a.cpu().numpy().astype(np.int32)
        o2, r2, d2, term2 = ora.step(a_np if kind == "v1" else a_np.reshape(-1), nthreads=NT)
        o1 = obs.cpu().numpy().reshape(B, -1)
        r1, d1 = rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        o2 = o2.reshape(B, -1).astype(np.float32)
        eq = (d1 == d2) & (r1.view(np.uint32) == r2.astype(np.float32).view(np.uint32))
        eq &= (o1.view(np.uint32) == o2.view(np.uint32)).all(axis=1)
        i = _first_bad(eq)
        assert i is None, "%s N=%d: env %d differs at step %d (%d envs differ)" % (kind, n, i, t, int((~eq).sum()))
        if d1.any():
            t1 = info["terminal_observation"].cpu().numpy().reshape(B, -1)[d1]
            t2 = term2.reshape(B, -1)[d1].astype(np.float32)
            teq = (t1.view(np.uint32) == t2.view(np.uint32)).all(axis=1)
            assert teq.all(), "%s N=%d: terminal obs of env %d at step %d" % (
                kind, n, int(np.flatnonzero(d1)[_first_bad(teq)]), t)
        # the size-independent properties: lockstep episode ends, finite values, reward bounds
        assert d1.all() == ((t + 1) % period == 0) and d1.any() == d1.all(), "episode end at step %d" % t
        assert np.isfinite(o1).all() and np.isfinite(r1).all() and np.abs(r1).max() < 1500.0
        compared += B
    assert compared == B * T
    venv.close()


@pytest.mark.parametrize("n", [2, 5])
def test_v1_full_size_every_env(n):
    _check("v1", n, 320, 300)


def test_v1_10v10_full_size_every_env():
    """Futbol-v1 (N = 10) at the same 65 536 envs: 80 steps (its oracle is ~5x the 5v5 one)"""
    _check("v1", 10, 80, 300)


@pytest.mark.parametrize("n", [2, 5])
def test_v1_full_size_rollout_every_env(n):
    """The open-loop rollout instance (bench.py's open_loop_rollout companion line) at the full size: 2
    launches of 30 steps, every env's obs / reward / done of every step against the oracle"""
    from gym_futbol_amd import FutbolVecEnv
    seed = 41 + n
    venv = FutbolVecEnv("v1", B, seed=seed, dtype=torch.float32, number_of_player=n)
    ora = O.V1Vec(B, N=n, seed=seed, portable=True)
    o = venv.reset().cpu().numpy()
    assert np.array_equal(o.view(np.uint32), ora.reset().astype(np.float32).view(np.uint32))
    K = 30
    for c in range(2):
        acts = venv.random_actions_steps(K, c * K, seed=99)
        obs, rew, done, _ = venv.rollout(acts)
        a_np = acts.cpu().numpy().astype(np.int32)
        o1, r1, d1 = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool)
        for t in range(K):
            o2, r2, d2, _ = ora.step(a_np[t], nthreads=NT)
            eq = (d1[t] == d2) & (r1[t].view(np.uint32) == r2.astype(np.float32).view(np.uint32))
            eq &= (o1[t].reshape(B, -1).view(np.uint32) == o2.reshape(B, -1).astype(np.float32).view(np.uint32)).all(axis=1)
            i = _first_bad(eq)
            assert i is None, "rollout N=%d: env %d differs at step %d" % (n, i, c * K + t)
    venv.close()


def test_v0_full_size_every_env():
    _check("v0", 0, 420, 401)
