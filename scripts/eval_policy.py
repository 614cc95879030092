"""Evaluate the reference's trained 2v2 PPO2 policy (trained_model_2v2/model1) on the GPU env and
compare with the notebook's published evaluate_policy result (2027.02 +/- 1519.25 over 10 episodes).

    python scripts/eval_policy.py [--envs 65536] [--out profiles/r01/policy_eval.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

REF_MEAN, REF_STD, REF_N = 2027.02, 1519.25, 10  # colab_notebook.ipynb, model1, n_eval_episodes=10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import gym_futbol_amd as gf
    from gym_futbol_amd.evaluation import evaluate_policy
    from gym_futbol_amd.policy import SB2MlpPolicy
    dev = torch.device("cuda", 0)
    res = {"reference": {"mean": REF_MEAN, "std": REF_STD, "n": REF_N,
                         "source": "colab_notebook.ipynb: evaluate_policy(PPO2.load('trained_model_2v2/model1'), "
                                   "gym.make('Futbol2v2-v1'), n_eval_episodes=10)"}}
    venv = gf.make("Futbol2v2-v1", num_envs=a.envs, device=dev, seed=a.seed)
    pol = SB2MlpPolicy.from_npz(os.path.join(ROOT, "tests", "golden", "sb2_2v2_model1.npz"), [5] * 4, dev)
    t0 = time.perf_counter()
    m, s, r, lens = evaluate_policy(venv, pol)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    se = REF_STD / np.sqrt(REF_N)
    res["model1"] = {"mean": m, "std": s, "n": int(len(r)), "ep_len": int(lens.max()),
                     "z_vs_reference": (m - REF_MEAN) / np.sqrt(se ** 2 + (s / np.sqrt(len(r))) ** 2),
                     "seconds": dt, "env_steps_per_s_with_policy": float(lens.sum()) / dt}

    class Random:
        def act(self, obs, deterministic=True, out=None):
            return out.random_(0, 5)
    m2, s2, r2, _ = evaluate_policy(venv, Random())
    res["random_policy"] = {"mean": m2, "std": s2, "n": int(len(r2))}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
