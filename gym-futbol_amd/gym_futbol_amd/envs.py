"""`FutbolEnv` -- single-env facade with the reference's v0 API.

Mirrors gym_futbol/envs/futbol_env.py:132-983 (`FutbolEnv`): constructor
kwargs, `reset() -> obs (6, 5)`, `step(a) -> (obs, reward, done, {})` with the
hard-coded opponent (`random_opp=False`) or the random one, `action_space`
Discrete(16) / Tuple(Discrete(4), Discrete(4)).  Runs on the GPU (B = 1, fp64,
no auto-reset).  The reference returns its internal `self.obs` array (aliased,
SURVEY D.11); this facade returns a copy.
"""
import numpy as np
import torch

from .vec_env import FutbolVecEnv

# envs/ballowner.py, envs/action.py
AI_1, AI_2, OPP_1, OPP_2, NOONE = range(5)
RUN, INTERCEPT, SHOOT, ASSIST = range(4)


def v0_attrs_from_state(st, i):
    """The reference FutbolEnv's per-env attributes (envs/futbol_env.py: ball_owner, last_ball_owner,
    time -- accumulated 0.1 per step in fp64 --, ai_score, opp_score) of env i of a host state dict."""
    from .vec_env import _accumulated_time
    meta = int(st["meta"][i])
    B = st["meta"].shape[0]
    return {"ball_owner": meta & 7, "last_ball_owner": (meta >> 3) & 7,
            "time": _accumulated_time((meta >> 18) & 0x3FFF),
            "ai_score": int(st["score"][i]), "opp_score": int(st["score"][B + i])}


class FutbolEnv:
    def __init__(self, length=105, width=68, goal_size=10, game_time=40, player_speed=12, shoot_speed=20,
                 Debug=False, pressure_range=2, one_goal_end=False, action_as_int=True, only_reward_goal=False,
                 random_opp=True, device="cuda", seed=0, env_id=0):
        self.length, self.width, self.goal_size = length, width, goal_size
        self.game_time, self.player_speed, self.shoot_speed = game_time, player_speed, shoot_speed
        self.Debug, self.one_goal_end = Debug, one_goal_end
        self.action_as_int, self.only_reward_goal, self.random_opp = action_as_int, only_reward_goal, random_opp
        self._venv = FutbolVecEnv("v0", 1, device=device, seed=seed, env_id_base=env_id, dtype=torch.float64,
                                  auto_reset=False, length=length, width=width, goal_size=goal_size,
                                  game_time=game_time, player_speed=player_speed, shoot_speed=shoot_speed,
                                  one_goal_end=one_goal_end, action_as_int=action_as_int,
                                  only_reward_goal=only_reward_goal, random_opp=random_opp)
        self.action_space = self._venv.action_space
        self.observation_space = self._venv.observation_space
        self.obs = self._obs_from_state()

    def _obs_from_state(self):
        s = self._venv.get_state()
        o = np.zeros((6, 5), np.float64)
        o[:5] = s["row"].reshape(5, 5, -1)[:, :, 0]
        meta = int(s["meta"][0])
        if (meta >> 7) & 1:
            owner = meta & 7
            o[5, owner if owner <= 3 else 4] = 10
        return o

    def reset(self):
        self.obs = self._venv.reset()[0].cpu().numpy().copy()
        return self.obs

    def step(self, ai_action_type):
        if self.action_as_int:
            a = int(ai_action_type)
            if not 0 <= a <= 15:
                raise ValueError("action %r outside Discrete(16)" % (ai_action_type,))
            t = torch.tensor([[a]], dtype=torch.uint8)
        else:
            a0, a1 = (int(x) for x in ai_action_type)
            if not (0 <= a0 <= 3 and 0 <= a1 <= 3):
                raise ValueError("action %r outside Tuple(Discrete(4), Discrete(4))" % (ai_action_type,))
            t = torch.tensor([[a0, a1]], dtype=torch.uint8)
        obs, rew, done, _ = self._venv.step(t)
        self.obs = obs[0].cpu().numpy().copy()
        return self.obs, float(rew[0].item()), bool(done[0].item()), {}

    @property
    def ball_owner(self):
        return v0_attrs_from_state(self._venv.get_state(), 0)["ball_owner"]

    @property
    def last_ball_owner(self):
        return v0_attrs_from_state(self._venv.get_state(), 0)["last_ball_owner"]

    @property
    def time(self):
        return v0_attrs_from_state(self._venv.get_state(), 0)["time"]

    @property
    def ai_score(self):
        return v0_attrs_from_state(self._venv.get_state(), 0)["ai_score"]

    @property
    def opp_score(self):
        return v0_attrs_from_state(self._venv.get_state(), 0)["opp_score"]

    def render(self, mode="human", close=False):
        import matplotlib.pyplot as plt
        _, ax = plt.subplots()
        ax.set_xlim(0, self.length)
        ax.set_ylim(0, self.width)
        o = self.obs
        for r, c in ((0, "red"), (1, "red"), (2, "blue"), (3, "blue")):
            ax.plot(o[r, 0], o[r, 1], color=c, marker="o", markersize=12)
        ax.plot(o[4, 0], o[4, 1], color="green", marker="o", markersize=8)
        return ax

    def close(self):
        self._venv.close()
