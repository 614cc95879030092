"""PPO2 on the GPU env: the training loop of the reference's notebook
(colab_notebook.ipynb:779-866: `model = PPO2(CustomPolicy, DummyVecEnv([lambda: env] * 8))`,
`model.learn(total_timesteps=5 * 10**4, callback=eval_callback)`), for B envs resident on one
GPU.

stable-baselines 2.10's PPO2 (absent from this image) is restated from its published
algorithm, hyperparameter for hyperparameter (defaults = the values decoded from the
reference's model zips):
  * Runner: `n_steps` steps of every env; at each step the policy samples one categorical per
    MultiDiscrete sub-action, the env steps with DummyVecEnv auto-reset, `dones[t]` marks that
    obs[t] starts a new episode, and the value of the last obs bootstraps the rollout.
  * GAE(gamma, lam) backwards over the rollout; returns = advantages + values.
  * `noptepochs` passes over a random permutation of the n_envs * n_steps samples, cut into
    `nminibatches` minibatches.  Per minibatch: advantages normalised with the minibatch mean
    and (population) std + 1e-8; ratio = exp(old_neglogp - neglogp);
    loss = mean(max(-A ratio, -A clip(ratio, 1 +- cliprange))) - ent_coef * entropy
           + vf_coef * 0.5 * mean(max((v - R)^2, (v_old + clip(v - v_old, +-cliprange_vf) - R)^2))
    with cliprange_vf = None meaning "same as cliprange" and a negative value meaning no value
    clipping (SB2's convention); gradients clipped to a global norm of `max_grad_norm`;
    Adam(learning_rate, eps=1e-5).
  * `learning_rate` / `cliprange` are constants or callables of the remaining-progress
    fraction 1 - (update - 1) / n_updates (SB2 `get_schedule_fn`).
The policy is SB2's FeedForwardPolicy (`MlpPolicy`): `net_arch` = shared sizes followed by an
optional dict(pi=[...], vf=[...]), tanh, orthogonal init (gain sqrt(2) hidden, 0.01 policy
head, 1 value head), zero biases.  The notebook's `CustomPolicy` is CUSTOM_NET_ARCH.

Everything stays on the device: the HIP step kernel writes obs / reward / done into the env's
buffers, torch copies them into the rollout storage, and the only host synchronisation per
update is the logging at its end.  The dense layers run as hipBLASLt GEMMs through torch.
"""
import json
import math
import time

import numpy as np
import torch

CUSTOM_NET_ARCH = [256, 256, dict(pi=[128, 128], vf=[128, 128])]  # colab_notebook.ipynb:782
MLP_NET_ARCH = [dict(pi=[64, 64], vf=[64, 64])]  # SB2 MlpPolicy default


def _schedule(v):
    return v if callable(v) else (lambda frac, _v=float(v): _v)


def _parse_arch(net_arch):
    shared, pi, vf = [], [], []
    for layer in net_arch:
        if isinstance(layer, int):
            if pi or vf:
                raise ValueError("shared layers must precede the pi/vf dict in net_arch")
            shared.append(int(layer))
        else:
            pi = [int(x) for x in layer.get("pi", [])]
            vf = [int(x) for x in layer.get("vf", [])]
    return shared, pi, vf


def _linear(n_in, n_out, gain):
    lin = torch.nn.Linear(n_in, n_out)
    torch.nn.init.orthogonal_(lin.weight, gain=gain)
    torch.nn.init.zeros_(lin.bias)
    return lin


class ActorCritic(torch.nn.Module):
    """SB2 FeedForwardPolicy with a MultiCategorical (MultiDiscrete) or Categorical head."""

    def __init__(self, obs_dim, nvec, net_arch=CUSTOM_NET_ARCH):
        super().__init__()
        self.obs_dim = int(obs_dim)
        self.nvec = [int(n) for n in nvec]
        self.net_arch = net_arch
        shared, pi, vf = _parse_arch(net_arch)
        g = math.sqrt(2.0)

        def mlp(sizes, n_in):
            layers = []
            for n in sizes:
                layers.append(_linear(n_in, n, g))
                n_in = n
            return torch.nn.ModuleList(layers), n_in

        self.shared, n = mlp(shared, self.obs_dim)
        self.pi_net, npi = mlp(pi, n)
        self.vf_net, nvf = mlp(vf, n)
        self.pi_head = _linear(npi, sum(self.nvec), 0.01)
        self.vf_head = _linear(nvf, 1, 1.0)

    @staticmethod
    def _run(x, layers):
        for lin in layers:
            x = torch.tanh(lin(x))
        return x

    def forward(self, obs):
        """obs [B, obs_dim] -> (logits [B, sum(nvec)], value [B])."""
        h = self._run(obs.reshape(obs.shape[0], -1).float(), self.shared)
        return self.pi_head(self._run(h, self.pi_net)), self.vf_head(self._run(h, self.vf_net))[:, 0]

    def _groups(self, logits):
        return torch.split(logits, self.nvec, dim=1)

    def neglogp_entropy(self, logits, actions):
        """-log p(actions) and the entropy of the MultiCategorical (sums over sub-actions)."""
        nlp = torch.zeros(logits.shape[0], device=logits.device)
        ent = torch.zeros_like(nlp)
        for k, g in enumerate(self._groups(logits)):
            lp = torch.log_softmax(g, dim=1)
            nlp = nlp - lp.gather(1, actions[:, k:k + 1].long())[:, 0]
            ent = ent - (lp.exp() * lp).sum(1)
        return nlp, ent

    def sample(self, logits, deterministic=False, generator=None):
        """int64 actions [B, len(nvec)]: per-group argmax, or a Gumbel-max sample."""
        out = []
        for g in self._groups(logits):
            if deterministic:
                out.append(g.argmax(dim=1))
            else:
                u = torch.rand(g.shape, device=g.device, generator=generator).clamp_(1e-20, 1.0)
                out.append((g - torch.log(-torch.log(u))).argmax(dim=1))
        return torch.stack(out, dim=1)

    @torch.no_grad()
    def act(self, obs, deterministic=True, out=None, generator=None):
        """uint8 actions for the env (the `evaluate_policy` interface of policy.SB2MlpPolicy)."""
        logits, _ = self.forward(obs)
        a = self.sample(logits, deterministic, generator)
        if out is None:
            return a.to(torch.uint8)
        out.copy_(a)
        return out


def explained_variance(y_pred, y):
    """1 - Var[y - y_pred] / Var[y] (SB2 common.math_util.explained_variance)."""
    var = torch.var(y, unbiased=False)
    return float("nan") if float(var) == 0.0 else float(1.0 - torch.var(y - y_pred, unbiased=False) / var)


def gae_returns(rewards, values, dones, last_values, last_dones, gamma, lam):
    """SB2 PPO2 Runner: GAE(gamma, lam) over [T, B] rollouts; dones[t] = obs[t] starts an episode.
    Returns advantages + values."""
    T = rewards.shape[0]
    adv = torch.empty_like(rewards)
    last = torch.zeros_like(rewards[0])
    for t in reversed(range(T)):
        if t == T - 1:
            nonterminal, next_values = 1.0 - last_dones, last_values
        else:
            nonterminal, next_values = 1.0 - dones[t + 1], values[t + 1]
        delta = rewards[t] + gamma * next_values * nonterminal - values[t]
        last = delta + gamma * lam * nonterminal * last
        adv[t] = last
    return adv + values


def ppo_loss(policy, obs, actions, returns, values, neglogp_old, clip, clip_vf, ent_coef, vf_coef):
    """SB2 PPO2's minibatch loss (ppo2.py `setup_model` / `_train_step`): advantages normalised
    over the minibatch, clipped surrogate, clipped value loss (clip_vf None: no clipping here --
    PPO2.learn passes the policy's clip range, as SB2 does), entropy bonus.  Returns the loss
    and the detached [pg_loss, vf_loss, entropy, approxkl, clipfrac]."""
    adv = returns - values
    adv = (adv - adv.mean()) / (adv.std(unbiased=False) + 1e-8)
    logits, v = policy(obs)
    nlp, ent = policy.neglogp_entropy(logits, actions)
    entropy = ent.mean()
    if clip_vf is None:
        vf_loss = 0.5 * ((v - returns) ** 2).mean()
    else:
        v_clip = values + torch.clamp(v - values, -clip_vf, clip_vf)
        vf_loss = 0.5 * torch.maximum((v - returns) ** 2, (v_clip - returns) ** 2).mean()
    ratio = torch.exp(neglogp_old - nlp)
    pg_loss = torch.maximum(-adv * ratio, -adv * torch.clamp(ratio, 1.0 - clip, 1.0 + clip)).mean()
    loss = pg_loss - entropy * ent_coef + vf_loss * vf_coef
    with torch.no_grad():
        approxkl = 0.5 * ((nlp - neglogp_old) ** 2).mean()
        clipfrac = ((ratio - 1.0).abs() > clip).float().mean()
        parts = torch.stack([pg_loss.detach(), vf_loss.detach(), entropy.detach(), approxkl, clipfrac])
    return loss, parts


class PPO2:
    """PPO2(policy, env, ...) with SB2's constructor arguments and learn()/predict()/save()/load().

    policy: "MlpPolicy" / "CustomPolicy" (the notebook's net_arch), a net_arch list, or an
    ActorCritic instance.  env: a FutbolVecEnv (torch tensors on the GPU) or anything with the
    same reset() / step() / num_envs / action_space / observation_space surface."""

    def __init__(self, policy, env, gamma=0.99, n_steps=128, ent_coef=0.01, learning_rate=2.5e-4, vf_coef=0.5,
                 max_grad_norm=0.5, lam=0.95, nminibatches=4, noptepochs=4, cliprange=0.2, cliprange_vf=None,
                 verbose=0, seed=None, device=None):
        from .vec_env import SB3VecEnv
        self.env = env.venv if isinstance(env, SB3VecEnv) else env  # the numpy adapter -> its torch env
        self.gamma, self.lam = float(gamma), float(lam)
        self.n_steps, self.nminibatches, self.noptepochs = int(n_steps), int(nminibatches), int(noptepochs)
        self.ent_coef, self.vf_coef, self.max_grad_norm = float(ent_coef), float(vf_coef), float(max_grad_norm)
        self.learning_rate, self.cliprange, self.cliprange_vf = learning_rate, cliprange, cliprange_vf
        self.verbose = int(verbose)
        self.n_envs = int(self.env.num_envs)
        self.n_batch = self.n_envs * self.n_steps
        if self.n_batch % self.nminibatches:
            raise ValueError("n_envs * n_steps (%d) must be a multiple of nminibatches (%d)"
                             % (self.n_batch, self.nminibatches))
        dev = device if device is not None else getattr(self.env, "device", "cpu")
        self.device = torch.device(dev)
        self.generator = torch.Generator(device=self.device)
        self.generator.manual_seed(0 if seed is None else int(seed))
        self.seed = seed
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
        self.optimizer = torch.optim.Adam(self.policy.parameters(), lr=1e-3, eps=1e-5)
        self.num_timesteps = 0
        self._obs = None
        self.ep_info_buf = []  # (mean return, episodes) of every rollout that finished episodes
        self.logs = []

    # ------------------------------------------------------------------ rollout
    def _ensure_started(self):
        if self._obs is None:
            self._obs = self.env.reset().float().clone()
            self._dones = torch.zeros(self.n_envs, dtype=torch.float32, device=self.device)
            self._ep_ret = torch.zeros(self.n_envs, dtype=torch.float64, device=self.device)

    @torch.no_grad()
    def _rollout(self, callback):
        T, B, dev = self.n_steps, self.n_envs, self.device
        obs_buf = torch.empty((T,) + tuple(self._obs.shape), dtype=torch.float32, device=dev)
        act_buf = torch.empty((T, B, len(self.policy.nvec)), dtype=torch.int64, device=dev)
        val_buf = torch.empty((T, B), dtype=torch.float32, device=dev)
        nlp_buf = torch.empty((T, B), dtype=torch.float32, device=dev)
        rew_buf = torch.empty((T, B), dtype=torch.float32, device=dev)
        done_buf = torch.empty((T, B), dtype=torch.float32, device=dev)
        fin = torch.zeros(2, dtype=torch.float64, device=dev)  # finished episodes: return sum, count
        for t in range(T):
            obs_buf[t].copy_(self._obs)
            done_buf[t].copy_(self._dones)
            logits, value = self.policy(self._obs)
            a = self.policy.sample(logits, generator=self.generator)
            nlp, _ = self.policy.neglogp_entropy(logits, a)
            act_buf[t], val_buf[t], nlp_buf[t] = a, value, nlp
            obs, rew, done, _ = self.env.step(a.to(torch.uint8))
            self._obs.copy_(obs)
            rew_buf[t].copy_(rew)
            db = done.bool()
            self._dones.copy_(db.float())
            # Monitor-style episode returns, accumulated on the device (fp64 like the env)
            self._ep_ret += rew.double()
            fin[0] += torch.where(db, self._ep_ret, torch.zeros_like(self._ep_ret)).sum()
            fin[1] += db.double().sum()
            self._ep_ret.masked_fill_(db, 0.0)
            self.num_timesteps += B
            if callback is not None and callback.on_step(self) is False:
                return None
        _, last_values = self.policy(self._obs)
        ret = gae_returns(rew_buf, val_buf, done_buf, last_values, self._dones, self.gamma, self.lam)

        def flat(x):
            return x.reshape((T * B,) + tuple(x.shape[2:]))
        return flat(obs_buf), flat(ret), flat(act_buf), flat(val_buf), flat(nlp_buf), fin

    # ------------------------------------------------------------------ update
    def _train(self, batch, lr, clip, clip_vf):
        obs, returns, actions, values, neglogp_old = batch
        for g in self.optimizer.param_groups:
            g["lr"] = lr
        mb = self.n_batch // self.nminibatches
        stats = []
        for _ in range(self.noptepochs):
            perm = torch.randperm(self.n_batch, device=self.device, generator=self.generator)
            for s in range(0, self.n_batch, mb):
                idx = perm[s:s + mb]
                loss, parts = ppo_loss(self.policy, obs[idx], actions[idx], returns[idx], values[idx],
                                       neglogp_old[idx], clip, clip_vf, self.ent_coef, self.vf_coef)
                self.optimizer.zero_grad(set_to_none=True)
                loss.backward()
                torch.nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
                self.optimizer.step()
                stats.append(parts)
        return torch.stack(stats).mean(0)

    def learn(self, total_timesteps, callback=None, log_interval=1, reset_num_timesteps=True):
        if reset_num_timesteps:
            self.num_timesteps = 0
        lr_fn, clip_fn = _schedule(self.learning_rate), _schedule(self.cliprange)
        if self.cliprange_vf is None:
            clip_vf_fn = clip_fn  # SB2: None -> the policy's clip range
        elif not callable(self.cliprange_vf) and float(self.cliprange_vf) < 0:
            clip_vf_fn = None  # original PPO: no value clipping
        else:
            clip_vf_fn = _schedule(self.cliprange_vf)
        self._ensure_started()
        n_updates = int(total_timesteps) // self.n_batch
        if callback is not None and hasattr(callback, "init_callback"):
            callback.init_callback(self)
        t_start = time.time()
        for update in range(1, n_updates + 1):
            frac = 1.0 - (update - 1.0) / n_updates
            lr, clip = float(lr_fn(frac)), float(clip_fn(frac))
            clip_vf = None if clip_vf_fn is None else float(clip_vf_fn(frac))
            t0 = time.time()
            out = self._rollout(callback)
            if out is None:
                break
            obs, ret, act, val, nlp, fin = out
            st = self._train((obs, ret, act, val, nlp), lr, clip, clip_vf)
            if update % log_interval == 0 or update == 1:
                pg, vf, ent, kl, cf = (float(x) for x in st.cpu())
                fsum, fcnt = (float(x) for x in fin.cpu())
                if fcnt > 0:
                    self.ep_info_buf.append((fsum / fcnt, fcnt))
                rec = {"nupdates": update, "total_timesteps": self.num_timesteps,
                       "fps": int(self.n_batch / max(time.time() - t0, 1e-9)),
                       "explained_variance": explained_variance(val, ret),
                       "policy_loss": pg, "value_loss": vf, "policy_entropy": ent, "approxkl": kl,
                       "clipfrac": cf, "ep_reward_mean": self.ep_info_buf[-1][0] if self.ep_info_buf else None,
                       "time_elapsed": time.time() - t_start}
                self.logs.append(rec)
                if self.verbose:
                    print(json.dumps(rec), flush=True)
        return self

    # ------------------------------------------------------------------ SB2 helpers
    @torch.no_grad()
    def predict(self, observation, deterministic=False):
        """(actions, None) like SB2's predict; numpy in -> numpy out, tensors stay tensors."""
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
        """Parameters + hyperparameters, loadable with torch.load(weights_only=True)."""
        hyper = {k: getattr(self, k) for k in ("gamma", "lam", "n_steps", "nminibatches", "noptepochs", "ent_coef",
                                              "vf_coef", "max_grad_norm")}
        for k in ("learning_rate", "cliprange", "cliprange_vf"):
            v = getattr(self, k)
            if v is None or not callable(v):
                hyper[k] = v
        torch.save({"state_dict": {k: v.detach().cpu() for k, v in self.policy.state_dict().items()},
                    "obs_dim": self.policy.obs_dim, "nvec": self.policy.nvec,
                    "net_arch": json.dumps(self.policy.net_arch), "hyper": json.dumps(hyper),
                    "num_timesteps": self.num_timesteps}, path)

    @staticmethod
    def load_policy(path, device="cpu"):
        d = torch.load(path, map_location="cpu", weights_only=True)
        pol = ActorCritic(d["obs_dim"], d["nvec"], json.loads(d["net_arch"]))
        pol.load_state_dict(d["state_dict"])
        return pol.to(device)

    @classmethod
    def load(cls, path, env, device=None, **kwargs):
        d = torch.load(path, map_location="cpu", weights_only=True)
        hyper = json.loads(d["hyper"])
        hyper.update(kwargs)
        from .vec_env import SB3VecEnv
        dev = device if device is not None else getattr(env.venv if isinstance(env, SB3VecEnv) else env, "device",
                                                        "cpu")
        model = cls(cls.load_policy(path, dev), env, device=dev, **hyper)
        model.num_timesteps = int(d["num_timesteps"])
        return model
