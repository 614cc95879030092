"""PPO2 and A2C and Monitor / EvalCallback (§8(f) #4) on the CPU, driven by a small
torch env with the FutbolVecEnv surface (the GPU env itself is exercised in test_gpu_train.py).

* GAE against a plain-Python restatement of stable-baselines 2's PPO2 Runner loop, and the
  minibatch loss (clipped surrogate, clipped value loss, entropy, approxkl, clipfrac) against numpy;
* learning: PPO2 solves a contextual bandit (reward 1 for picking the arg-max observation);
* save / load round trip (torch.load weights_only=True);
* VecMonitor CSV (SB2 Monitor format) and EvalCallback's evaluations.npz (the keys, dtypes and
  shapes of the reference's gym_futbol/envs_v1/2v2/logs/evaluations.npz)."""
import json
import os

import numpy as np
import pytest
import torch

from gym_futbol_amd import spaces as sp
from gym_futbol_amd.monitor import EvalCallback, VecMonitor, load_results
from gym_futbol_amd.ppo import PPO2, ActorCritic, gae_returns


class BanditEnv:
    """B envs; obs = 5 random scores + 1; action MultiDiscrete([5, 3]); reward 1 when action[0]
    is the arg-max score; episodes of `ep_len` steps with auto-reset."""

    def __init__(self, B=64, ep_len=10, seed=0):
        self.num_envs, self.episode_steps, self.device = B, ep_len, torch.device("cpu")
        self.action_space = sp.MultiDiscrete([5, 3])
        self.observation_space = sp.Box(-np.inf, np.inf, shape=(6,))
        self.action_dim = 2
        self.g = torch.Generator().manual_seed(seed)
        self.t = torch.zeros(B, dtype=torch.int64)

    def _obs(self):
        o = torch.randn((self.num_envs, 6), generator=self.g)
        o[:, 5] = 1.0
        self.obs = o
        return o

    def reset(self, mask=None):
        self.t.zero_()
        return self._obs()

    def step(self, actions):
        a = torch.as_tensor(actions).long()
        rew = (a[:, 0] == self.obs[:, :5].argmax(1)).float()
        self.t += 1
        done = self.t >= self.episode_steps
        self.t[done] = 0
        return self._obs(), rew, done, {}


def test_gae_matches_sb2_runner_loop():
    rng = np.random.default_rng(0)
    T, B, gamma, lam = 7, 5, 0.99, 0.95
    rew, val = rng.normal(size=(T, B)), rng.normal(size=(T, B))
    dones = (rng.random((T, B)) < 0.3).astype(np.float64)
    last_val, last_done = rng.normal(size=B), (rng.random(B) < 0.3).astype(np.float64)
    # stable-baselines PPO2 Runner._run, written out as in its published source
    adv = np.zeros_like(rew)
    lastgaelam = 0
    for step in reversed(range(T)):
        if step == T - 1:
            nextnonterminal, nextvalues = 1.0 - last_done, last_val
        else:
            nextnonterminal, nextvalues = 1.0 - dones[step + 1], val[step + 1]
        delta = rew[step] + gamma * nextvalues * nextnonterminal - val[step]
        adv[step] = lastgaelam = delta + gamma * lam * nextnonterminal * lastgaelam
    ret = gae_returns(*(torch.as_tensor(x) for x in (rew, val, dones, last_val, last_done)), gamma, lam)
    assert np.allclose(ret.numpy(), adv + val, rtol=1e-12, atol=1e-12)


def test_policy_heads_and_distribution():
    pol = ActorCritic(20, [5] * 4, [256, 256, dict(pi=[128, 128], vf=[128, 128])])
    shapes = [tuple(p.shape) for p in pol.parameters()]
    assert (256, 20) in shapes and (128, 256) in shapes and (20, 128) in shapes and (1, 128) in shapes
    obs = torch.randn(32, 20)
    logits, v = pol(obs)
    assert logits.shape == (32, 20) and v.shape == (32,)
    a = pol.sample(logits, generator=torch.Generator().manual_seed(1))
    nlp, ent = pol.neglogp_entropy(logits, a)
    ref = -sum(torch.log_softmax(g, 1).gather(1, a[:, k:k + 1])[:, 0]
               for k, g in enumerate(torch.split(logits, [5] * 4, 1)))
    assert torch.allclose(nlp, ref) and (ent > 0).all() and (ent <= 4 * np.log(5) + 1e-6).all()
    assert torch.equal(pol.act(obs).long(), torch.stack([g.argmax(1) for g in torch.split(logits, [5] * 4, 1)], 1))


def test_ppo_learns_contextual_bandit(tmp_path):
    env = BanditEnv(B=64, ep_len=10)
    model = PPO2([dict(pi=[32], vf=[32])], env, n_steps=16, nminibatches=4, noptepochs=4, learning_rate=3e-3,
                 ent_coef=0.0, seed=0)
    model.learn(total_timesteps=64 * 16 * 40)
    assert len(model.logs) == 40
    first, last = model.logs[0], model.logs[-1]
    assert all(np.isfinite([r["policy_loss"], r["value_loss"], r["approxkl"]]).all() for r in model.logs)
    assert last["ep_reward_mean"] > 7.0 > first["ep_reward_mean"], (first["ep_reward_mean"], last["ep_reward_mean"])
    # deterministic play picks the arg-max score
    obs = env.reset()
    a, _ = model.predict(obs, deterministic=True)
    assert (a[:, 0] == obs[:, :5].argmax(1)).float().mean() > 0.9
    # save / load round trip with the safe loader
    path = str(tmp_path / "m.pt")
    model.save(path)
    m2 = PPO2.load(path, env)
    a2, _ = m2.predict(obs, deterministic=True)
    assert torch.equal(a, a2) and m2.n_steps == 16 and m2.num_timesteps == model.num_timesteps


def test_clip_semantics():
    """cliprange_vf None -> the policy clip range; < 0 -> no value clipping (SB2 convention)."""
    env = BanditEnv(B=8)
    for cvf in (None, -1.0, 0.5):
        m = PPO2("MlpPolicy", env, n_steps=8, nminibatches=2, noptepochs=1, cliprange_vf=cvf, seed=1)
        m.learn(8 * 8 * 2)
        assert len(m.logs) == 2
    with pytest.raises(ValueError):
        PPO2("MlpPolicy", env, n_steps=5, nminibatches=3)
    with pytest.raises(ValueError):
        PPO2("NoSuchPolicy", env)


def test_vec_monitor_csv(tmp_path):
    env = BanditEnv(B=16, ep_len=10)
    mon = VecMonitor(env, str(tmp_path), env_id="Bandit", flush_every=7)
    mon.reset()
    returns = torch.zeros(16, dtype=torch.float64)
    expect = []
    for t in range(35):
        a = torch.randint(0, 5, (16, 2))
        _, r, d, _ = mon.step(a)
        returns += r.double()
        for i in np.nonzero(d.numpy())[0]:
            expect.append(float(returns[i]))
            returns[i] = 0
    mon.close()
    assert sorted(mon.episode_rewards) == sorted(expect) and len(expect) == 48
    assert mon.episode_lengths == [10] * 48
    with open(tmp_path / "monitor.csv") as f:
        head = json.loads(f.readline()[1:])
        assert head["env_id"] == "Bandit" and f.readline().strip() == "r,l,t"
    df = load_results(str(tmp_path))
    assert list(df.columns) == ["r", "l", "t"] and len(df) == 48 and (df["l"] == 10).all()


def test_eval_callback_writes_sb2_evaluations(tmp_path):
    env, eval_env = BanditEnv(B=32, ep_len=10, seed=1), BanditEnv(B=8, ep_len=10, seed=2)
    cb = EvalCallback(eval_env, n_eval_episodes=5, eval_freq=16, log_path=str(tmp_path),
                      best_model_save_path=str(tmp_path), verbose=0)
    model = PPO2([dict(pi=[16], vf=[16])], env, n_steps=16, nminibatches=2, noptepochs=2, seed=0)
    model.learn(32 * 16 * 3, callback=cb)
    z = np.load(tmp_path / "evaluations.npz", allow_pickle=False)
    assert sorted(z.files) == ["ep_lengths", "results", "timesteps"]
    assert z["timesteps"].dtype == np.int64 and z["results"].dtype == np.float32 and z["ep_lengths"].dtype == np.int64
    assert z["results"].shape == (3, 5, 1) and z["ep_lengths"].shape == (3, 5)
    assert z["timesteps"].tolist() == [32 * 16, 32 * 32, 32 * 48] and (z["ep_lengths"] == 10).all()
    assert os.path.exists(tmp_path / "best_model.pt")
    assert isinstance(PPO2.load_policy(str(tmp_path / "best_model.pt")), ActorCritic)


def test_a2c_returns_match_sb2_discount_with_dones():
    from gym_futbol_amd.a2c import discounted_returns
    rng = np.random.default_rng(3)
    T, B, gamma = 5, 6, 0.99
    rew = rng.normal(size=(T, B))
    dones = (rng.random((T, B)) < 0.3).astype(np.float64)
    last = rng.normal(size=B)

    def discount_with_dones(rewards, dones_, g):  # stable-baselines a2c/utils.py, as published
        discounted, r = [], 0
        for reward, done in zip(rewards[::-1], dones_[::-1]):
            r = reward + g * r * (1.0 - done)
            discounted.append(r)
        return discounted[::-1]

    exp = np.zeros((T, B))
    for n in range(B):
        r, d = list(rew[:, n]), list(dones[:, n])
        if d[-1] == 0:
            exp[:, n] = discount_with_dones(r + [last[n]], d + [0], gamma)[:-1]
        else:
            exp[:, n] = discount_with_dones(r, d, gamma)
    got = discounted_returns(*(torch.as_tensor(x) for x in (rew, dones, last)), gamma)
    assert np.allclose(got.numpy(), exp, rtol=1e-12, atol=1e-12)


def test_tf_rmsprop_update():
    from gym_futbol_amd.a2c import TFRMSProp
    p = torch.nn.Parameter(torch.tensor([1.0, -2.0], dtype=torch.float64))
    opt = TFRMSProp([p], lr=0.1, alpha=0.9, eps=1e-5)
    p.grad = torch.tensor([0.5, 2.0], dtype=torch.float64)
    opt.step()
    ms = 0.9 * 1.0 + 0.1 * np.array([0.25, 4.0])        # TF1 initialises the slot to ones
    assert np.allclose(p.detach().numpy(), np.array([1.0, -2.0]) - 0.1 * np.array([0.5, 2.0]) / np.sqrt(ms + 1e-5))


def test_a2c_learns_contextual_bandit():
    from gym_futbol_amd import A2C
    env = BanditEnv(B=64, ep_len=10)
    model = A2C([dict(pi=[32], vf=[32])], env, learning_rate=5e-3, ent_coef=0.0, seed=0)
    model.learn(total_timesteps=64 * 5 * 1200, log_interval=200)
    obs = env.reset()
    a, _ = model.predict(obs, deterministic=True)
    assert (a[:, 0] == obs[:, :5].argmax(1)).float().mean() > 0.9
    # SB2's RMSProp slot starts at 1 (small first steps), so A2C needs ~1000 updates here
    assert model.logs[-1]["ep_reward_mean"] > 6.5 > 3.0 > model.logs[1]["ep_reward_mean"]


def test_ppo_loss_matches_numpy_restatement():
    """ppo_loss against SB2 PPO2's loss written out in numpy (ppo2.py setup_model / _train_step)."""
    from gym_futbol_amd.ppo import ppo_loss
    torch.manual_seed(0)
    pol = ActorCritic(6, [5, 3], [dict(pi=[8], vf=[8])])
    rng = np.random.default_rng(1)
    n = 64
    obs = torch.as_tensor(rng.normal(size=(n, 6)))
    act = torch.as_tensor(np.stack([rng.integers(0, 5, n), rng.integers(0, 3, n)], 1))
    ret, val = torch.as_tensor(rng.normal(size=n) * 3), torch.as_tensor(rng.normal(size=n))
    nlp_old = torch.as_tensor(rng.uniform(1.0, 3.0, n))
    clip, clip_vf, ent_c, vf_c = 0.2, 0.2, 0.01, 0.5
    loss, parts = ppo_loss(pol, obs, act, ret, val, nlp_old, clip, clip_vf, ent_c, vf_c)
    with torch.no_grad():
        logits, v = pol(obs)
    lg, v = logits.double().numpy(), v.double().numpy()
    R, V, NLP0 = ret.numpy(), val.numpy(), nlp_old.numpy()

    def logsoftmax(x):
        m = x.max(1, keepdims=True)
        return x - m - np.log(np.exp(x - m).sum(1, keepdims=True))
    l0, l1 = logsoftmax(lg[:, :5]), logsoftmax(lg[:, 5:])
    a = act.numpy()
    nlp = -(l0[np.arange(n), a[:, 0]] + l1[np.arange(n), a[:, 1]])
    ent = -(np.exp(l0) * l0).sum(1) - (np.exp(l1) * l1).sum(1)
    advs = R - V
    advs = (advs - advs.mean()) / (advs.std() + 1e-8)
    vclip = V + np.clip(v - V, -clip_vf, clip_vf)
    vf_loss = 0.5 * np.mean(np.maximum((v - R) ** 2, (vclip - R) ** 2))
    ratio = np.exp(NLP0 - nlp)
    pg_loss = np.mean(np.maximum(-advs * ratio, -advs * np.clip(ratio, 1 - clip, 1 + clip)))
    expect = pg_loss - ent.mean() * ent_c + vf_loss * vf_c
    assert abs(float(loss.detach()) - expect) < 1e-5 * max(1.0, abs(expect))
    p = parts.numpy()
    assert np.allclose(p[:3], [pg_loss, vf_loss, ent.mean()], rtol=1e-5, atol=1e-6)
    assert abs(p[3] - 0.5 * np.mean((nlp - NLP0) ** 2)) < 1e-5
    assert abs(p[4] - np.mean(np.abs(ratio - 1) > clip)) < 1e-6
