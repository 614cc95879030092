"""`evaluate_policy` on B GPU envs at once.

stable-baselines 2 `common.evaluation.evaluate_policy(model, env, n_eval_episodes=10,
deterministic=True)` (used by the reference notebook, colab_notebook.ipynb) resets one
env, plays `n_eval_episodes` episodes one after the other and returns the mean and
standard deviation of the episode returns.  Here every env of a `FutbolVecEnv` plays
its FIRST episode in parallel (the envs are independent, so B episodes = B samples of
the same distribution) and the same statistics are returned, plus the raw returns.
"""
import numpy as np
import torch


@torch.no_grad()
def evaluate_policy(venv, policy, n_eval_episodes=None, deterministic=True, max_steps=100000):
    B = venv.num_envs
    n = B if n_eval_episodes is None else int(n_eval_episodes)
    if n > B:
        raise ValueError("n_eval_episodes (%d) > num_envs (%d): use more envs" % (n, B))
    obs = venv.reset()
    ret = torch.zeros(B, dtype=torch.float64, device=venv.device)
    finished = torch.zeros(B, dtype=torch.bool, device=venv.device)
    final = torch.zeros(B, dtype=torch.float64, device=venv.device)
    lengths = torch.zeros(B, dtype=torch.int64, device=venv.device)
    act = torch.empty((B, venv.action_dim), dtype=torch.uint8, device=venv.device)
    for t in range(max_steps):
        policy.act(obs, deterministic=deterministic, out=act)
        obs, rew, done, _ = venv.step(act)
        live = ~finished
        ret += torch.where(live, rew.double(), torch.zeros_like(ret))
        lengths += live.long()
        newly = done & live
        final = torch.where(newly, ret, final)
        finished |= done
        if t % 50 == 49 and bool(finished.all()):
            break
    if not bool(finished[:n].all()):
        raise RuntimeError("episodes did not finish within max_steps")
    r = final[:n].cpu().numpy()
    return float(r.mean()), float(r.std()), r, lengths[:n].cpu().numpy()
