"""PPO2 on the GPU env: the notebook's CustomPolicy / PPO2 defaults trained
on 4096 Futbol2v2-v1 envs through VecMonitor with an EvalCallback.  Learning is checked
statistically (deterministic evaluation over 2048 first episodes, before vs after), the logs
against stable-baselines 2's formats."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_ppo2_trains_on_gpu_env(tmp_path):
    import gym_futbol_amd as gf
    from gym_futbol_amd.evaluation import evaluate_policy
    env = gf.VecMonitor(gf.make("Futbol2v2-v1", num_envs=4096, seed=3), str(tmp_path), env_id="Futbol2v2-v1")
    eval_env = gf.make("Futbol2v2-v1", num_envs=2048, seed=77)
    model = gf.PPO2("CustomPolicy", env, seed=0)
    m0, s0, _, _ = evaluate_policy(eval_env, model.policy)
    cb = gf.EvalCallback(eval_env, n_eval_episodes=256, eval_freq=4 * model.n_steps, log_path=str(tmp_path),
                         best_model_save_path=str(tmp_path), verbose=0)
    model.learn(int(6e6), callback=cb)
    assert len(model.logs) == 11 and model.num_timesteps == 11 * model.n_batch
    assert all(np.isfinite([r["policy_loss"], r["value_loss"], r["policy_entropy"]]).all() for r in model.logs)
    m1, s1, r1, lens = evaluate_policy(eval_env, model.policy)
    assert (lens == 300).all()
    se = np.hypot(s0, s1) / np.sqrt(2048)
    assert m1 - m0 > 6 * se, (m0, m1, se)   # the trained policy is much better than the initial one
    env.close()
    assert len(env.episode_rewards) == 4096 * (model.num_timesteps // 4096 // 300)
    df = gf.load_results(str(tmp_path))
    assert len(df) == len(env.episode_rewards) and (df["l"] == 300).all()
    z = np.load(os.path.join(str(tmp_path), "evaluations.npz"), allow_pickle=False)
    assert z["results"].shape == (2, 256, 1) and z["ep_lengths"].shape == (2, 256)
    assert (z["ep_lengths"] == 300).all()
    pol = gf.PPO2.load_policy(os.path.join(str(tmp_path), "best_model.pt"), eval_env.device)
    assert isinstance(pol, gf.ActorCritic)


def test_a2c_runs_on_gpu_env():
    """A2C (SB2 defaults: n_steps 5, RMSProp) on 4096 GPU envs: mechanics and finite losses."""
    import gym_futbol_amd as gf
    env = gf.make("Futbol2v2-v1", num_envs=4096, seed=4)
    model = gf.A2C("CustomPolicy", env, seed=0)
    model.learn(4096 * 5 * 120, log_interval=30)
    assert model.num_timesteps == 4096 * 5 * 120
    assert all(np.isfinite([r["policy_loss"], r["value_loss"], r["policy_entropy"]]).all() for r in model.logs)
    assert any(r["ep_reward_mean"] is not None for r in model.logs)   # 600 steps: two episodes ended
    obs = env.reset()
    a, _ = model.predict(obs, deterministic=True)
    assert a.shape == (4096, 4) and a.dtype == torch.int64 and int(a.max()) <= 4
    env.close()
