"""A2C on the GPU env: the other stable-baselines algorithm the north star names ("PPO/A2C can
train unchanged"), restated from stable-baselines 2.10's `A2C` (absent from this image) with its
defaults: n_steps 5, gamma 0.99, vf_coef 0.25, ent_coef 0.01, max_grad_norm 0.5,
learning_rate 7e-4 (constant schedule), RMSProp(alpha 0.99, epsilon 1e-5).

  * Runner: n_steps steps of every env; returns R_t = r_t + gamma * R_{t+1} * (1 - done_t)
    (`discount_with_dones`), bootstrapped with V(s_T) for envs whose last step did not end an
    episode.
  * Loss: mean(A * neglogp) - ent_coef * entropy + vf_coef * mean((V - R)^2), A = R - V(s_t)
    (no advantage normalisation); gradients clipped to `max_grad_norm`.
  * RMSProp as TensorFlow 1 implements it (what SB2 ran): the mean-square slot starts at 1,
    ms = alpha * ms + (1 - alpha) * g^2, p -= lr * g / sqrt(ms + epsilon).
The policy is the same SB2 FeedForwardPolicy as PPO2 (`ppo.ActorCritic`).
"""
import json
import time

import numpy as np
import torch

from .ppo import CUSTOM_NET_ARCH, MLP_NET_ARCH, ActorCritic, _schedule, explained_variance


class TFRMSProp(torch.optim.Optimizer):
    """tf.train.RMSPropOptimizer(decay, epsilon), momentum 0, non-centered."""

    def __init__(self, params, lr=7e-4, alpha=0.99, eps=1e-5):
        super().__init__(params, dict(lr=lr, alpha=alpha, eps=eps))

    @torch.no_grad()
    def step(self):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if "ms" not in st:
                    st["ms"] = torch.ones_like(p)
                ms = st["ms"]
                ms.mul_(g["alpha"]).addcmul_(p.grad, p.grad, value=1.0 - g["alpha"])
                p.addcdiv_(p.grad, torch.sqrt(ms + g["eps"]), value=-g["lr"])


def discounted_returns(rewards, dones, last_values, gamma):
    """SB2 A2CRunner: dones[t] = the step t ended an episode; bootstrap with last_values where
    the last step did not end one.  rewards / dones [T, B], last_values [B] -> returns [T, B]."""
    T = rewards.shape[0]
    ret = torch.empty_like(rewards)
    r = last_values * (1.0 - dones[T - 1])
    for t in reversed(range(T)):
        r = rewards[t] + gamma * r * (1.0 - dones[t]) if t < T - 1 else rewards[t] + gamma * r
        ret[t] = r
    return ret


class A2C:
    """A2C(policy, env, ...) with SB2's constructor arguments and learn()/predict()/save()."""

    def __init__(self, policy, env, gamma=0.99, n_steps=5, vf_coef=0.25, ent_coef=0.01, max_grad_norm=0.5,
                 learning_rate=7e-4, alpha=0.99, epsilon=1e-5, lr_schedule="constant", verbose=0, seed=None,
                 device=None):
        from .vec_env import SB3VecEnv
        self.env = env.venv if isinstance(env, SB3VecEnv) else env
        self.gamma, self.n_steps = float(gamma), int(n_steps)
        self.vf_coef, self.ent_coef, self.max_grad_norm = float(vf_coef), float(ent_coef), float(max_grad_norm)
        self.learning_rate, self.lr_schedule = learning_rate, lr_schedule
        if lr_schedule not in ("constant", "linear"):
            raise ValueError("lr_schedule must be 'constant' or 'linear'")
        self.verbose = int(verbose)
        self.n_envs = int(self.env.num_envs)
        self.n_batch = self.n_envs * self.n_steps
        self.device = torch.device(device if device is not None else getattr(self.env, "device", "cpu"))
        self.generator = torch.Generator(device=self.device)
        self.generator.manual_seed(0 if seed is None else int(seed))
        nvec = getattr(self.env.action_space, "nvec", None)
        nvec = [int(n) for n in (nvec if nvec is not None else [self.env.action_space.n])]
        obs_dim = int(np.prod(self.env.observation_space.shape))
        if isinstance(policy, ActorCritic):
            self.policy = policy
        else:
            arch = policy
            if isinstance(policy, str):
                if policy not in ("MlpPolicy", "CustomPolicy"):
                    raise ValueError("unknown policy %r" % policy)
                arch = MLP_NET_ARCH if policy == "MlpPolicy" else CUSTOM_NET_ARCH
            with torch.random.fork_rng(devices=[]):
                torch.manual_seed(0 if seed is None else int(seed))
                self.policy = ActorCritic(obs_dim, nvec, arch)
        self.policy.to(self.device)
        self.optimizer = TFRMSProp(self.policy.parameters(), lr=float(_schedule(learning_rate)(1.0)), alpha=alpha,
                                   eps=epsilon)
        self.num_timesteps = 0
        self._obs = None
        self.logs = []

    def learn(self, total_timesteps, callback=None, log_interval=100, reset_num_timesteps=True):
        if reset_num_timesteps:
            self.num_timesteps = 0
        if self._obs is None:
            self._obs = self.env.reset().float().clone()
            self._ep_ret = torch.zeros(self.n_envs, dtype=torch.float64, device=self.device)
        if callback is not None and hasattr(callback, "init_callback"):
            callback.init_callback(self)
        T, B, dev = self.n_steps, self.n_envs, self.device
        n_updates = int(total_timesteps) // self.n_batch
        lr0 = float(_schedule(self.learning_rate)(1.0))
        fin = torch.zeros(2, dtype=torch.float64, device=dev)
        t_start = time.time()
        for update in range(1, n_updates + 1):
            obs_buf = torch.empty((T,) + tuple(self._obs.shape), dtype=torch.float32, device=dev)
            act_buf = torch.empty((T, B, len(self.policy.nvec)), dtype=torch.int64, device=dev)
            rew_buf = torch.empty((T, B), dtype=torch.float32, device=dev)
            done_buf = torch.empty((T, B), dtype=torch.float32, device=dev)
            with torch.no_grad():
                for t in range(T):
                    obs_buf[t].copy_(self._obs)
                    logits, _ = self.policy(self._obs)
                    a = self.policy.sample(logits, generator=self.generator)
                    act_buf[t] = a
                    obs, rew, done, _ = self.env.step(a.to(torch.uint8))
                    self._obs.copy_(obs)
                    rew_buf[t].copy_(rew)
                    db = done.bool()
                    done_buf[t].copy_(db.float())
                    self._ep_ret += rew.double()
                    fin[0] += torch.where(db, self._ep_ret, torch.zeros_like(self._ep_ret)).sum()
                    fin[1] += db.double().sum()
                    self._ep_ret.masked_fill_(db, 0.0)
                    self.num_timesteps += B
                    if callback is not None and callback.on_step(self) is False:
                        return self
                _, last_v = self.policy(self._obs)
                ret = discounted_returns(rew_buf, done_buf, last_v, self.gamma)
            lr = lr0 if self.lr_schedule == "constant" else lr0 * (1.0 - (update - 1.0) / n_updates)
            for g in self.optimizer.param_groups:
                g["lr"] = lr
            obs_f = obs_buf.reshape((T * B,) + tuple(obs_buf.shape[2:]))
            logits, v = self.policy(obs_f)
            nlp, ent = self.policy.neglogp_entropy(logits, act_buf.reshape(T * B, -1))
            R = ret.reshape(-1)
            adv = (R - v).detach()
            pg_loss = (adv * nlp).mean()
            vf_loss = ((v - R) ** 2).mean()
            entropy = ent.mean()
            loss = pg_loss - entropy * self.ent_coef + vf_loss * self.vf_coef
            self.optimizer.zero_grad(set_to_none=True)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
            self.optimizer.step()
            if update % log_interval == 0 or update == 1 or update == n_updates:
                fsum, fcnt = (float(x) for x in fin.cpu())
                fin.zero_()
                rec = {"nupdates": update, "total_timesteps": self.num_timesteps,
                       "policy_loss": float(pg_loss.detach()), "value_loss": float(vf_loss.detach()),
                       "policy_entropy": float(entropy.detach()),
                       "explained_variance": explained_variance(v.detach(), R),
                       "ep_reward_mean": fsum / fcnt if fcnt else None, "time_elapsed": time.time() - t_start}
                self.logs.append(rec)
                if self.verbose:
                    print(json.dumps(rec), flush=True)
        return self

    @torch.no_grad()
    def predict(self, observation, deterministic=False):
        is_np = not isinstance(observation, torch.Tensor)
        obs = torch.as_tensor(np.asarray(observation) if is_np else observation, device=self.device)
        single = obs.dim() == len(self.env.observation_space.shape)
        if single:
            obs = obs[None]
        logits, _ = self.policy(obs)
        a = self.policy.sample(logits, deterministic, generator=self.generator)
        if single:
            a = a[0]
        return (a.cpu().numpy() if is_np else a), None

    def save(self, path):
        torch.save({"state_dict": {k: v.detach().cpu() for k, v in self.policy.state_dict().items()},
                    "obs_dim": self.policy.obs_dim, "nvec": self.policy.nvec,
                    "net_arch": json.dumps(self.policy.net_arch),
                    "hyper": json.dumps({"gamma": self.gamma, "n_steps": self.n_steps, "vf_coef": self.vf_coef,
                                         "ent_coef": self.ent_coef, "max_grad_norm": self.max_grad_norm}),
                    "num_timesteps": self.num_timesteps}, path)
