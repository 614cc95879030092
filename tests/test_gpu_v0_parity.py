"""v0 FutbolEnv kernel (hard-coded opponent / random opponent) on the GPU.

 * bit-for-bit vs oracle/liboracle_portable.so on free-running rollouts;
 * vs the REFERENCE's own outputs (tests/golden/v0_*.npz, produced by running
   gym_futbol/envs/futbol_env.py under the same RNG tape): discrete outputs
   (done, reward's discrete part, owner row) exact, floats within 1e-9 (the
   only differences are libm pow/sin/cos vs the kernel's correctly-rounded
   x*x and portable sin/cos; north-star tolerance is 1e-5).
"""
import os

import numpy as np
import pytest
import torch

from helpers import O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _venv(B, seed, random_opp, dtype=torch.float64, **kw):
    from gym_futbol_amd import FutbolVecEnv
    return FutbolVecEnv("v0", B, seed=seed, dtype=dtype, random_opp=random_opp, **kw)


@pytest.mark.parametrize("random_opp", [False, True])
def test_free_running_bit_exact(random_opp):
    B, T, seed = 1024, 900, 5 + int(random_opp)
    venv = _venv(B, seed, random_opp)
    ora = O.V0Vec(B, seed=seed, random_opp=random_opp, portable=True)
    assert np.array_equal(venv.reset().cpu().numpy(), ora.reset())
    shots = 0
    for t in range(T):
        a = venv.random_actions(t)
        obs, rew, done, info = venv.step(a)
        o2, r2, d2, term2 = ora.step(a.cpu().numpy().astype(np.int32).reshape(-1))
        o1, r1, d1 = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        assert np.array_equal(d1, d2), "done differs at %d" % t
        # bitwise (also the sign of zero)
        assert np.array_equal(r1.view(np.uint64), r2.view(np.uint64)), "reward differs at %d (max %g)" % (
            t, np.abs(r1 - r2).max())
        assert np.array_equal(o1.view(np.uint64), o2.view(np.uint64)), "obs differs at %d (max %g)" % (
            t, np.abs(o1 - o2).max())
        if d1.any():
            assert np.array_equal(info["terminal_observation"].cpu().numpy()[d1].view(np.uint64),
                                  term2[d1].view(np.uint64))
        shots += int((o1[:, 4, 4] >= 4).sum())
    assert shots > 0


@pytest.mark.parametrize("fname", ["v0_hardcoded_opp.npz", "v0_random_opp.npz"])
def test_against_reference_goldens(fname):
    g = np.load(os.path.join(GOLDEN, fname))
    E, T = g["actions"].shape
    venv = _venv(E, int(g["seed"]), bool(g["random_opp"]))
    o = venv.reset().cpu().numpy()
    assert np.array_equal(o, g["obs0"])
    maxd = 0.0
    for t in range(T):
        a = torch.as_tensor(g["actions"][:, t].astype(np.uint8).reshape(E, 1), device=venv.device)
        obs, rew, done, _ = venv.step(a)
        o, r, d = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        assert np.array_equal(d, g["done"][:, t].astype(bool)), "done differs at %d" % t
        assert np.array_equal(o[:, 5], g["obs"][:, t, 5]), "owner row differs at %d" % t
        assert np.allclose(r, g["reward"][:, t], rtol=0, atol=1e-9), t
        assert np.allclose(o, g["obs"][:, t], rtol=0, atol=1e-9), (t, np.abs(o - g["obs"][:, t]).max())
        maxd = max(maxd, float(np.abs(o - g["obs"][:, t]).max()))
    print("max |kernel - reference| over %s: %g" % (fname, maxd))


def test_tuple_actions_and_flags():
    """action_as_int=False (Tuple action space), one_goal_end, only_reward_goal."""
    B, seed = 512, 9
    for kw in ({"action_as_int": False}, {"one_goal_end": True}, {"only_reward_goal": True}):
        venv = _venv(B, seed, False, **kw)
        ora = O.V0Vec(B, seed=seed, random_opp=False, portable=True,
                      **{k: v for k, v in kw.items() if k != "action_as_int"})
        venv.reset()
        ora.reset()
        for t in range(450):
            a = venv.random_actions(t)
            obs, rew, done, _ = venv.step(a)
            an = a.cpu().numpy().astype(np.int32)
            an = an[:, 0] * 4 + an[:, 1] if an.shape[1] == 2 else an.reshape(-1)
            o2, r2, d2, _ = ora.step(an)
            assert np.array_equal(done.cpu().numpy(), d2), (kw, t)
            assert np.array_equal(rew.cpu().numpy(), r2), (kw, t)
            assert np.array_equal(obs.cpu().numpy(), o2), (kw, t)
