"""Policy in the loop on the GPU: the reference's trained 2v2 policy played on
the HIP env.  Statistical anchor for the v1 path, whose physics (pymunk / Chipmunk) cannot run
here: the reference notebook prints evaluate_policy(model1, Futbol2v2-v1, 10 episodes) =
2027.02 +/- 1519.25.  A policy evaluated on an env with different dynamics, observations or
rewards would not keep that performance; the random policy is the control."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_trained_policy_matches_published_evaluation():
    import os
    import gym_futbol_amd as gf
    from gym_futbol_amd.evaluation import evaluate_policy
    from gym_futbol_amd.policy import SB2MlpPolicy
    npz = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sb2_2v2_model1.npz")
    venv = gf.make("Futbol2v2-v1", num_envs=16384, seed=5)
    pol = SB2MlpPolicy.from_npz(npz, [5] * 4, venv.device)
    m, s, r, lens = evaluate_policy(venv, pol)
    assert (lens == 300).all()
    se = np.hypot(1519.25 / np.sqrt(10), s / np.sqrt(len(r)))
    assert abs(m - 2027.02) < 3.3 * se, (m, s)

    class Random:
        def act(self, obs, deterministic=True, out=None):
            return out.random_(0, 5)
    m0, s0, r0, _ = evaluate_policy(venv, Random())
    assert m - m0 > 10 * np.hypot(s, s0) / np.sqrt(len(r)), (m, m0)   # the trained policy is far better
    venv.close()
