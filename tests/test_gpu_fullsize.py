"""The benchmark's workload at its full size, on the GPU: B = 65 536 envs per context (1 024
one-wave blocks: one wave per SIMD, every XCD), float32 outputs (the bench's kernel instance),
synthetic device actions, auto-reset across an episode boundary.  A per-env oracle of the same
global env id checks a spread sample of the envs (first / last blocks, every block's last lane)
bit for bit at every step; all envs are checked for the size-independent properties (episode
ends exactly at step 300 / 401, finite observations, rewards within the reference's bounds).
"""
import numpy as np
import pytest
import torch

from helpers import O

pytestmark = pytest.mark.gpu
B = 65536


def _sample_ids():
    ids = set(range(0, 64)) | set(range(B - 64, B)) | set(range(63, B, 64 * 37)) | set(range(4096, B, 8191))
    return np.array(sorted(ids))


def _check(kind, n, T, period):
    from gym_futbol_amd import FutbolVecEnv
    kw = {"number_of_player": n} if kind == "v1" else {"random_opp": False}
    seed = 21 + n
    venv = FutbolVecEnv(kind, B, seed=seed, dtype=torch.float32, **kw)
    ids = _sample_ids()
    if kind == "v1":
        oras = [O.V1Vec(1, N=n, seed=seed, env_id_base=int(i), portable=True) for i in ids]
    else:
        oras = [O.V0Vec(1, seed=seed, env_id_base=int(i), random_opp=False, portable=True) for i in ids]
    o = venv.reset().cpu().numpy()
    o_ref = np.stack([ora.reset()[0] for ora in oras])
    assert np.array_equal(o[ids], o_ref.astype(np.float32))
    for t in range(T):
        a = venv.random_actions(t, seed=777)
        obs, rew, done, info = venv.step(a)
        a_np = a.cpu().numpy().astype(np.int32)
        o1, r1, d1 = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        assert d1.all() == ((t + 1) % period == 0) and d1.any() == d1.all(), "episode end at step %d" % t
        assert np.isfinite(o1).all() and np.isfinite(r1).all()
        assert np.abs(r1).max() < 1500.0
        for k, (i, ora) in enumerate(zip(ids, oras)):
            ai = a_np[i] if kind == "v1" else a_np[i].reshape(-1)
            o2, r2, d2, _ = ora.step(ai[None, :] if kind == "v1" else ai)
            assert d1[i] == d2[0], "env %d done at step %d" % (i, t)
            assert o1[i].tobytes() == o2[0].astype(np.float32).tobytes(), "env %d obs at step %d" % (i, t)
            assert r1[i].tobytes() == np.float32(r2[0]).tobytes(), "env %d reward at step %d" % (i, t)
    venv.close()


@pytest.mark.parametrize("n", [2, 5])
def test_v1_full_size(n):
    _check("v1", n, 320, 300)


def test_v0_full_size():
    _check("v0", 0, 420, 401)
