"""`Futbol` -- single-env facade with the reference's envs_v1 API.

Mirrors gym_futbol/envs_v1/futbol_env.py:62-515 (`Futbol`): same constructor
kwargs, `reset()`, `step(left_player_action) -> (obs, reward, done, {})`,
`random_action()`, `action_space`, `observation_space`, and the attributes the
reference's notebook reads (`width`, `height`, `number_of_player`,
`current_time`, `ball_owner_side`, and `space` for its drawing cells'
`env.space.debug_draw(pymunk.matplotlib_util.DrawOptions(ax))`).  The step runs on the GPU (a B = 1
context, fp64 outputs, no auto-reset: like the reference, `done` stays True if
one keeps stepping).  For throughput use FutbolVecEnv / make(..., num_envs=B).
"""
import numpy as np
import torch

from .vec_env import FutbolVecEnv

WIDTH, HEIGHT, TOTAL_TIME = 105, 68, 30


class Futbol:
    def __init__(self, width=WIDTH, height=HEIGHT, total_time=TOTAL_TIME, debug=False, number_of_player=5,
                 device="cuda", seed=0, env_id=0):
        self.width = width
        self.height = height
        self.total_time = total_time
        self.debug = debug
        self.number_of_player = number_of_player
        self._venv = FutbolVecEnv("v1", 1, device=device, seed=seed, env_id_base=env_id, dtype=torch.float64,
                                  auto_reset=False, number_of_player=number_of_player, width=width, height=height,
                                  total_time=total_time)
        self.action_space = self._venv.action_space
        self.observation_space = self._venv.observation_space
        # the constructor already ran reset() (envs_v1/futbol_env.py:127)
        self.observation = observation_from_state(self._venv.get_state(), number_of_player)

    def reset(self):
        obs = self._venv.reset()
        self.observation = obs[0].cpu().numpy().copy()
        return self.observation

    def random_action(self):
        return self.action_space.sample()

    def step(self, left_player_action):
        a = np.asarray(left_player_action, dtype=np.int64).reshape(1, -1)
        if a.shape[1] != 2 * self.number_of_player or (a < 0).any() or (a > 4).any():
            raise ValueError("invalid action %r for MultiDiscrete([5, 5] * %d)" % (left_player_action,
                                                                                 self.number_of_player))
        obs, rew, done, _ = self._venv.step(torch.as_tensor(a, dtype=torch.uint8))
        self.observation = obs[0].cpu().numpy().copy()
        return self.observation, float(rew[0].item()), bool(done[0].item()), {}

    # -- attributes of the reference env --------------------------------------
    @property
    def current_time(self):
        """futbol_env.py:478 accumulates 0.1 per step in fp64 (memoised sums, vec_env._accumulated_time).
        Like the reference it keeps counting past the episode end when stepping on without reset."""
        return self._venv.env_attr("current_time")[0]

    @property
    def ball_owner_side(self):
        return self._venv.env_attr("ball_owner_side")[0]

    def body_states(self):
        """(positions [Nb,2], velocities [Nb,2]) of A0.., B0.., ball."""
        s = self._venv.get_state()
        return np.stack([s["px"], s["py"]], 1), np.stack([s["vx"], s["vy"]], 1)

    @property
    def space(self):
        """Stand-in for the reference's pymunk Space (futbol_env.py:75) as far as the notebook uses it:
        `space.debug_draw(options)` (colab_notebook.ipynb:289,616) draws the field into `options.ax`
        (pymunk.matplotlib_util.DrawOptions keeps its Axes there).  There is no pymunk Space here: the
        physics is the GPU kernel."""
        return FieldSpace(self.width, self.height, self.number_of_player, lambda: self.body_states()[0])

    def render(self, ax=None):
        """Matplotlib drawing of the field (replaces pymunk's debug_draw, futbol_env.py:236-243)."""
        import matplotlib.pyplot as plt
        p, _ = self.body_states()
        pad = 5
        if ax is None:
            ax = plt.axes(xlim=(0 - pad, self.width + pad), ylim=(0 - pad, self.height + pad))
        ax.set_aspect("equal")
        draw_field(ax, self.width, self.height, p, self.number_of_player)
        return ax

    def close(self):
        self._venv.close()


class FieldSpace:
    """`Futbol.space`: the part of pymunk's Space API the reference's notebook calls.  `positions` returns
    the current body positions [Nb, 2] (A0.., B0.., ball)."""

    def __init__(self, width, height, n, positions):
        self.width, self.height, self.number_of_player = width, height, n
        self._positions = positions

    def debug_draw(self, options):
        """pymunk Space.debug_draw (futbol_env.py:236-243 via the notebook): draw into options.ax, or into
        `options` itself when it is a matplotlib Axes."""
        ax = getattr(options, "ax", options)
        if not hasattr(ax, "add_patch"):
            raise TypeError("debug_draw needs pymunk.matplotlib_util.DrawOptions(ax) or an Axes, got %r" % (options,))
        return draw_field(ax, self.width, self.height, np.asarray(self._positions()), self.number_of_player)


def field_segments(width, height, goal_size=20):
    """The 12 static segments of _setup_walls (futbol_env.py:182-234): 6 walls, then the 6
    goal-box segments behind each goal mouth ([(x0, y0), (x1, y1)], radius 1 each)."""
    w, h, g = width, height, goal_size
    lo, hi = h / 2 - g / 2, h / 2 + g / 2
    walls = [((0, 0), (0, lo)), ((0, hi), (0, h)), ((0, h), (w, h)),
             ((w, 0), (w, lo)), ((w, hi), (w, h)), ((0, 0), (w, 0))]
    goals = [((-2, lo), (-2, hi)), ((-2, lo), (0, lo)), ((-2, hi), (0, hi)),
             ((w + 2, lo), (w + 2, hi)), ((w, lo), (w + 2, lo)), ((w, hi), (w + 2, hi))]
    return walls + goals


def draw_field(ax, width, height, positions, n):
    """Matplotlib equivalent of pymunk's space.debug_draw (futbol_env.py:236-243): the 12 segments
    (walls black, goal boxes grey, drawn with the segments' radius 1), the 2N players (radius 1.5,
    left red / right blue like Team's colour ramps, team.py:34-50) and the ball (radius 1)."""
    from matplotlib.patches import Circle
    for s, ((x0, y0), (x1, y1)) in enumerate(field_segments(width, height)):
        ax.plot([x0, x1], [y0, y1], "-", color="k" if s < 6 else "0.5", lw=2, solid_capstyle="round")
    for k in range(2 * n + 1):
        color = "g" if k == 2 * n else ("r" if k < n else "b")
        ax.add_patch(Circle(tuple(positions[k]), 1.0 if k == 2 * n else 1.5, color=color))
    return ax


def observation_from_state(state, n, env=0):
    """_get_observation (futbol_env.py:154-180) of env `env` from a host state dict."""
    nb = 2 * n + 1
    B = state["meta"].shape[0]
    px, py, vx, vy = (state[k].reshape(nb, B)[:, env] for k in ("px", "py", "vx", "vy"))
    o = [(px[-1] - 52.5) / 52.5, (py[-1] - 34.0) / 34.0, (vx[-1] - 0.0) / 25.0, (vy[-1] - 0.0) / 25.0]
    for k in range(2 * n):
        o += [(px[k] - 52.5) / 55.5, (py[k] - 34.0) / 34.0, (vx[k] - 0.0) / 10.0, (vy[k] - 0.0) / 10.0]
    return np.array(o, dtype=np.float64)
