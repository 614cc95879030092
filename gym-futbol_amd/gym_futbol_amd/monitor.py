"""Monitor / EvalCallback-compatible logging for the GPU envs.

The reference's notebook wraps its env in stable-baselines 2 `Monitor(env, log_dir)` and trains
with `EvalCallback(eval_env, best_model_save_path='./logs/', log_path='./logs/',
eval_freq=1000, n_eval_episodes=5, deterministic=True)` (colab_notebook.ipynb:800-823); the
results it shipped are `gym_futbol/envs_v1/2v2/logs/evaluations.npz` and `best_model.zip`.

* `VecMonitor` writes `<dir>/monitor.csv` in SB2's Monitor format -- a first line
  `#{"t_start": ..., "env_id": ...}`, the header `r,l,t`, one row per finished episode (return,
  length, seconds since t_start) -- for all B envs of a FutbolVecEnv.  Episode returns and
  lengths accumulate on the device and finished episodes are appended to a device buffer by a
  scatter (no host synchronisation per step); rows reach the file every `flush_every` steps.
* `EvalCallback` mirrors SB2's: every `eval_freq` calls (= vectorised steps) it evaluates the
  model's policy deterministically on `eval_env` (`evaluation.evaluate_policy`: n_eval_episodes
  first episodes played in parallel), appends to `<log_path>/evaluations.npz` with SB2's keys
  and shapes (timesteps int64 [n]; results float32 [n, n_eval_episodes, 1] -- the trailing 1
  is the reward shape of SB2's one-env VecEnv; ep_lengths int64 [n, n_eval_episodes]), and saves
  the best model to `<best_model_save_path>/best_model.pt`.
"""
import json
import math
import os
import time

import numpy as np
import torch

from .evaluation import evaluate_policy


class VecMonitor:
    EXT = "monitor.csv"

    def __init__(self, venv, filename=None, env_id=None, flush_every=100):
        self.venv = venv
        self.num_envs = venv.num_envs
        self.device = venv.device
        self.observation_space, self.action_space = venv.observation_space, venv.action_space
        self.flush_every = max(1, int(flush_every))
        B, dev = self.num_envs, self.device
        ep_len = max(1, int(getattr(venv, "episode_steps", 1)))
        self.cap = B * int(math.ceil(self.flush_every / ep_len))  # episodes that can end between flushes
        self._r = torch.zeros(B, dtype=torch.float64, device=dev)
        self._l = torch.zeros(B, dtype=torch.int64, device=dev)
        self._fin_r = torch.zeros(self.cap + 1, dtype=torch.float64, device=dev)  # slot cap = discard
        self._fin_l = torch.zeros(self.cap + 1, dtype=torch.int64, device=dev)
        self._fin_s = torch.zeros(self.cap + 1, dtype=torch.int64, device=dev)
        self._fin_n = torch.zeros((), dtype=torch.int64, device=dev)
        self._step_times = []  # host time of every step since the last flush
        self._time_base = 0    # absolute index of the step _step_times[0] belongs to
        self._steps = 0
        self.t_start = time.time()
        self.episode_rewards, self.episode_lengths, self.episode_times = [], [], []
        self.file = None
        if filename is not None:
            path = filename if filename.endswith(self.EXT) else (
                os.path.join(filename, self.EXT) if os.path.isdir(filename) else filename + "." + self.EXT)
            self.file = open(path, "wt")
            self.file.write("#%s\n" % json.dumps({"t_start": self.t_start, "env_id": env_id}))
            self.file.write("r,l,t\n")
            self.file.flush()

    def reset(self, mask=None):
        obs = self.venv.reset(mask)
        if mask is None:
            self._r.zero_()
            self._l.zero_()
        else:
            m = torch.as_tensor(mask, device=self.device).bool()
            self._r.masked_fill_(m, 0.0)
            self._l.masked_fill_(m, 0)
        return obs

    def step(self, actions):
        obs, rew, done, info = self.venv.step(actions)
        d = done.bool()
        self._r += rew.double()
        self._l += 1
        pos = self._fin_n + torch.cumsum(d.long(), 0) - 1
        idx = torch.where(d, pos.clamp(max=self.cap), torch.full_like(pos, self.cap))
        self._fin_r.scatter_(0, idx, self._r)
        self._fin_l.scatter_(0, idx, self._l)
        self._fin_s.scatter_(0, idx, torch.full_like(idx, self._steps))
        self._fin_n += d.long().sum()
        self._r.masked_fill_(d, 0.0)
        self._l.masked_fill_(d, 0)
        self._step_times.append(time.time() - self.t_start)
        self._steps += 1
        if self._steps % self.flush_every == 0:
            self.flush()
        return obs, rew, done, info

    def flush(self):
        """Move the finished episodes from the device buffer to the lists / the CSV file."""
        n = int(self._fin_n)
        if n > self.cap:
            raise RuntimeError("VecMonitor buffer overflow: %d episodes ended between flushes (capacity %d)"
                               % (n, self.cap))
        if n:
            r = self._fin_r[:n].cpu().numpy()
            l_ = self._fin_l[:n].cpu().numpy()
            s = self._fin_s[:n].cpu().numpy()
            t = [round(self._step_times[int(k) - self._time_base], 6) for k in s]
            self.episode_rewards += [float(x) for x in r]
            self.episode_lengths += [int(x) for x in l_]
            self.episode_times += t
            if self.file is not None:
                for x, y, z in zip(r, l_, t):
                    self.file.write("%s,%d,%s\n" % (round(float(x), 6), int(y), z))
                self.file.flush()
            self._fin_n.zero_()
        self._step_times = []
        self._time_base = self._steps

    def get_episode_rewards(self):
        self.flush()
        return list(self.episode_rewards)

    def get_episode_lengths(self):
        self.flush()
        return list(self.episode_lengths)

    def close(self):
        self.flush()
        if self.file is not None:
            self.file.close()
            self.file = None

    def __getattr__(self, name):  # everything else (episode_steps, action_dim, ...) from the env
        if name == "venv":
            raise AttributeError(name)
        return getattr(self.venv, name)


def load_results(path):
    """Rows of a monitor.csv (SB2 `bench.monitor.load_results` for one file) as a pandas DataFrame."""
    import pandas as pd
    fn = path if path.endswith(VecMonitor.EXT) else os.path.join(path, VecMonitor.EXT)
    with open(fn) as f:
        header = json.loads(f.readline()[1:])
        df = pd.read_csv(f)
    df["t"] += header["t_start"]
    return df


class EvalCallback:
    """SB2 `EvalCallback(eval_env, callback_on_new_best=None, n_eval_episodes=5, eval_freq=10000,
    log_path=None, best_model_save_path=None, deterministic=True, render=False, verbose=1)`."""

    def __init__(self, eval_env, callback_on_new_best=None, n_eval_episodes=5, eval_freq=10000, log_path=None,
                 best_model_save_path=None, deterministic=True, render=False, verbose=1):
        self.eval_env = eval_env
        self.callback_on_new_best = callback_on_new_best
        self.n_eval_episodes = int(n_eval_episodes)
        self.eval_freq = int(eval_freq)
        self.deterministic = deterministic
        self.verbose = verbose
        self.best_mean_reward = -np.inf
        self.last_mean_reward = -np.inf
        self.n_calls = 0
        self.model = None
        self.log_path = None if log_path is None else os.path.join(log_path, "evaluations")
        self.best_model_save_path = best_model_save_path
        self.evaluations_timesteps, self.evaluations_results, self.evaluations_length = [], [], []

    def init_callback(self, model):
        self.model = model
        for p in (self.best_model_save_path, None if self.log_path is None else os.path.dirname(self.log_path)):
            if p:
                os.makedirs(p, exist_ok=True)

    def on_step(self, model=None):
        if model is not None:
            self.model = model
        self.n_calls += 1
        if self.eval_freq > 0 and self.n_calls % self.eval_freq == 0:
            self.evaluate()
        return True

    def evaluate(self):
        mean, std, returns, lengths = evaluate_policy(self.eval_env, self.model.policy,
                                                      n_eval_episodes=self.n_eval_episodes,
                                                      deterministic=self.deterministic)
        self.evaluations_timesteps.append(int(self.model.num_timesteps))
        self.evaluations_results.append(np.asarray(returns, np.float32)[:, None])
        self.evaluations_length.append(np.asarray(lengths, np.int64))
        if self.log_path is not None:
            np.savez(self.log_path, timesteps=np.asarray(self.evaluations_timesteps, np.int64),
                     results=np.stack(self.evaluations_results), ep_lengths=np.stack(self.evaluations_length))
        self.last_mean_reward = mean
        if self.verbose:
            print("Eval num_timesteps=%d, episode_reward=%.2f +/- %.2f" % (self.model.num_timesteps, mean, std))
        if mean > self.best_mean_reward:
            self.best_mean_reward = mean
            if self.best_model_save_path is not None:
                self.model.save(os.path.join(self.best_model_save_path, "best_model.pt"))
            if self.callback_on_new_best is not None:
                self.callback_on_new_best.on_step(self.model)
        return mean, std
