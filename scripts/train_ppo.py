"""PPO2 training on the GPU env with the notebook's setup:
CustomPolicy net_arch, SB2 PPO2 defaults, VecMonitor CSV and EvalCallback evaluations.npz.

    python scripts/train_ppo.py [--envs 4096] [--timesteps 4e6] [--out gpurun_out/ppo]

Prints one JSON line per update and a summary (wall time, env-steps/s of the whole training
loop, the deterministic evaluation before/after vs the random policy)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]

import torch  # noqa: E402

import gym_futbol_amd as gf  # noqa: E402
from gym_futbol_amd.evaluation import evaluate_policy  # noqa: E402


class RandomPolicy:
    def act(self, obs, deterministic=True, out=None):
        return out.random_(0, 5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--timesteps", type=float, default=4e6)
    ap.add_argument("--eval-envs", type=int, default=1024)
    ap.add_argument("--out", default="gpurun_out/ppo")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    env = gf.VecMonitor(gf.make("Futbol2v2-v1", num_envs=a.envs, seed=a.seed), a.out, env_id="Futbol2v2-v1")
    eval_env = gf.make("Futbol2v2-v1", num_envs=a.eval_envs, seed=a.seed + 1000)
    model = gf.PPO2("CustomPolicy", env, verbose=1, seed=a.seed)
    m0, s0, _, _ = evaluate_policy(eval_env, model.policy)
    mr, sr, _, _ = evaluate_policy(eval_env, RandomPolicy())
    n_batch = model.n_batch
    cb = gf.EvalCallback(eval_env, n_eval_episodes=a.eval_envs, eval_freq=4 * model.n_steps, log_path=a.out,
                         best_model_save_path=a.out, verbose=1)
    torch.cuda.synchronize()
    t0 = time.time()
    model.learn(int(a.timesteps), callback=cb)
    torch.cuda.synchronize()
    wall = time.time() - t0
    m1, s1, _, _ = evaluate_policy(eval_env, model.policy)
    env.close()
    summary = {"envs": a.envs, "timesteps": model.num_timesteps, "updates": len(model.logs), "n_batch": n_batch,
               "wall_s": wall, "train_env_steps_per_s": model.num_timesteps / wall,
               "eval_untrained": [m0, s0], "eval_random_policy": [mr, sr], "eval_trained": [m1, s1],
               "eval_callback_best": cb.best_mean_reward, "monitor_episodes": len(env.episode_rewards),
               "monitor_mean_last_1000": sum(env.episode_rewards[-1000:]) / max(1, len(env.episode_rewards[-1000:])),
               "last_update": model.logs[-1] if model.logs else None}
    print(json.dumps(summary), flush=True)
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump({"summary": summary, "updates": model.logs}, f, indent=1)


if __name__ == "__main__":
    main()
