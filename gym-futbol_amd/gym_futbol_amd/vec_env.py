"""FutbolVecEnv: B independent gym-futbol envs resident on one GPU.

Torch-native, zero-copy: `reset()` / `step(actions)` take and return torch
tensors on the env's device; every call is one kernel launch on the current
HIP stream (graph-capturable, no host sync).  `as_sb3()` wraps it in the
stable-baselines VecEnv interface (numpy in/out, infos with
`terminal_observation`), which is what the reference's notebook drives through
DummyVecEnv (colab_notebook.ipynb:818-823).

Semantics per env are those of the reference's `step()`:
  v1 envs_v1/futbol_env.py:427-483 (opponent = random_action(), in-kernel)
  v0 envs/futbol_env.py:628-717     (hard-coded or random opponent, in-kernel)
plus DummyVecEnv's auto-reset: on done, `info["terminal_observation"]` holds the
episode's last obs and the returned obs is the reset obs.
"""
import ctypes as C

import numpy as np
import torch

from . import _native as nat
from . import spaces as sp

_DT = {"f8": np.float64, "u8": np.uint64, "u4": np.uint32, "u2": np.uint16, "u1": np.uint8}
# v1 body state is stored as (x, y) pairs per body and env (csrc/futbol_state.hpp): the state dict
# keeps the reference-shaped names (cpBody p / v / v_bias components), one [Nb * B] array each
_PAIR_FIELDS = {"pxy": ("px", "py"), "vxy": ("vx", "vy"), "bxy": ("bx", "by")}
# v0 rows / views are stored as consecutive pairs [n/2][B][2]: the state dict holds the [n][B] arrays
_GROUP_FIELDS = {"row2": ("row", 25), "view2": ("view", 8)}


def _stream_ptr(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class FutbolVecEnv:
    """Vectorised env.  kind: "v1" (envs_v1.Futbol) or "v0" (envs.FutbolEnv).

    v1 kwargs: number_of_player, width, height, total_time.
    v0 kwargs: length, width, goal_size, game_time, player_speed, shoot_speed,
               one_goal_end, action_as_int, only_reward_goal, random_opp.
    """

    def __init__(self, kind="v1", num_envs=1, device="cuda", seed=0, env_id_base=0, dtype=torch.float32,
                 auto_reset=True, **kwargs):
        if not torch.cuda.is_available():
            raise nat.NativeError("FutbolVecEnv needs a ROCm GPU (torch.cuda.is_available() is False); "
                                  "there is no CPU fallback")
        self.kind = kind
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        env_kind = nat.ENV_V1 if kind == "v1" else nat.ENV_V0
        n = int(kwargs.pop("number_of_player", 2)) if kind == "v1" else 2
        cfg = nat.default_config(env_kind, n)
        cfg.out_dtype = nat.F64 if dtype == torch.float64 else nat.F32
        cfg.auto_reset = 1 if auto_reset else 0
        v1_keys = {"width": "width", "height": "height", "total_time": "total_time"}
        v0_keys = {"length": "length0", "width": "width0", "goal_size": "goal_size0", "game_time": "game_time0",
                   "player_speed": "player_speed0", "shoot_speed": "shoot_speed0",
                   "one_goal_end": "one_goal_end0", "action_as_int": "action_as_int0",
                   "only_reward_goal": "only_reward_goal0", "random_opp": "random_opp0"}
        keys = v1_keys if kind == "v1" else v0_keys
        for k, v in kwargs.items():
            if k not in keys:
                raise TypeError("unexpected keyword argument %r for %s" % (k, kind))
            setattr(cfg, keys[k], type(getattr(cfg, keys[k]))(v) if not isinstance(v, bool) else int(v))
        self.number_of_player = n
        self.seed_value = int(seed)
        self.env_id_base = int(env_id_base)
        with torch.cuda.device(self.device):
            self.ctx = nat.Context(cfg, self.device.index, seed, env_id_base, num_envs)
        self.num_envs = self.ctx.num_envs
        self.obs_dim = self.ctx.obs_dim
        self.action_dim = self.ctx.action_dim
        self.dtype = dtype
        self.episode_steps = self.ctx.episode_steps
        B, dev = self.num_envs, self.device
        self.obs_shape = (self.obs_dim,) if kind == "v1" else (6, 5)
        self._obs = torch.zeros((B,) + self.obs_shape, dtype=dtype, device=dev)
        self._term = torch.zeros((B,) + self.obs_shape, dtype=dtype, device=dev)
        self._rew = torch.zeros(B, dtype=dtype, device=dev)
        self._done = torch.zeros(B, dtype=torch.uint8, device=dev)
        self._act = torch.zeros((B, self.action_dim), dtype=torch.uint8, device=dev)
        self._stats = torch.zeros(3, dtype=torch.float64, device=dev)
        if kind == "v1":
            self.action_space = sp.v1_action_space(n)
            self.observation_space = sp.v1_observation_space(n)
        else:
            self.action_space = sp.v0_action_space(bool(cfg.action_as_int0))
            self.observation_space = sp.v0_observation_space(cfg.length0, cfg.width0, cfg.player_speed0,
                                                             cfg.shoot_speed0)
        self._pending = None

    # ---------------------------------------------------------------- core
    def _actions_u8(self, actions):
        a = torch.as_tensor(actions, device=self.device)
        a = a.reshape(self.num_envs, self.action_dim)
        if a.dtype != torch.uint8:
            if bool((a < 0).any()):
                raise ValueError("negative action")
            a = a.to(torch.uint8)
        return a.contiguous()

    def reset(self, mask=None):
        """reset() every env (or those with mask[i] != 0); returns obs [B, ...] (device tensor)."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_reset(self.ctx.h, None if m is None else m.data_ptr(),
                                              self._obs.data_ptr(), _stream_ptr(self.device)), self.ctx.h)
        return self._obs

    def step(self, actions):
        """step(actions [B, action_dim]) -> (obs, reward, done(bool), info) as device tensors.

        The returned tensors are the env's own buffers and are overwritten by the
        next call (clone them to keep them).  info["terminal_observation"] is valid
        for the rows where done is True."""
        a = actions if (isinstance(actions, torch.Tensor) and actions.dtype == torch.uint8
                        and actions.is_contiguous() and actions.device == self.device) else self._actions_u8(actions)
        self.step_raw(a)
        return self._obs, self._rew, self._done.bool(), {"terminal_observation": self._term}

    def step_raw(self, actions_u8):
        """Launch one step; results land in self._obs/_rew/_done/_term.  No allocation, no sync."""
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_step(self.ctx.h, actions_u8.data_ptr(), self._obs.data_ptr(),
                                             self._rew.data_ptr(), self._done.data_ptr(), self._term.data_ptr(),
                                             _stream_ptr(self.device)), self.ctx.h)

    def rollout(self, actions, out=None):
        """Open-loop rollout: K consecutive steps in one launch for actions [K, B, action_dim] (uint8,
        device) chosen without looking at the observations.  Returns (obs [K, B, ...], reward [K, B],
        done [K, B] (uint8), terminal_obs [K, B, ...]); slice k is what the k-th step() returns.
        out: a tuple of such buffers to reuse (no allocation, graph-capturable)."""
        K = int(actions.shape[0])
        if actions.dtype != torch.uint8 or not actions.is_contiguous() or actions.device != self.device \
                or tuple(actions.shape[1:]) != (self.num_envs, self.action_dim):
            raise ValueError("rollout actions must be a contiguous uint8 [K, B, action_dim] tensor on the env's device")
        if out is None:
            out = (torch.empty((K, self.num_envs) + self.obs_shape, dtype=self.dtype, device=self.device),
                   torch.empty((K, self.num_envs), dtype=self.dtype, device=self.device),
                   torch.empty((K, self.num_envs), dtype=torch.uint8, device=self.device),
                   torch.empty((K, self.num_envs) + self.obs_shape, dtype=self.dtype, device=self.device))
        else:
            self._check_rollout_out(out, K)
        obs, rew, done, term = out
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_rollout(self.ctx.h, actions.data_ptr(), K, obs.data_ptr(), rew.data_ptr(),
                                                done.data_ptr(), term.data_ptr(), _stream_ptr(self.device)),
                      self.ctx.h)
        return out

    def _check_rollout_out(self, out, K):
        """The kernel writes K full slices into each caller buffer through raw pointers: dtype, shape,
        device and contiguity must be exactly what it assumes, or it would write past the allocation."""
        if not isinstance(out, (tuple, list)) or len(out) != 4:
            raise ValueError("rollout out must be a tuple (obs, reward, done, terminal_obs)")
        want = (((K, self.num_envs) + tuple(self.obs_shape), self.dtype), ((K, self.num_envs), self.dtype),
                ((K, self.num_envs), torch.uint8), ((K, self.num_envs) + tuple(self.obs_shape), self.dtype))
        for name, b, (shape, dt) in zip(("obs", "reward", "done", "terminal_obs"), out, want):
            if not isinstance(b, torch.Tensor) or b.dtype != dt or tuple(b.shape) != shape \
                    or not b.is_contiguous() or b.device != self.device:
                raise ValueError("rollout out[%s] must be a contiguous %s tensor of shape %s on %s, got %s"
                                 % (name, dt, shape, self.device,
                                    "%s %s %s contiguous=%s" % (b.dtype, tuple(b.shape), b.device, b.is_contiguous())
                                    if isinstance(b, torch.Tensor) else type(b).__name__))

    def random_actions(self, step, seed=1234, out=None):
        """Synthetic policy (iid uniform actions, Philox tag-1 stream), written on device."""
        out = self._act if out is None else out
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_fill_actions(self.ctx.h, int(seed), int(step), out.data_ptr(),
                                                     _stream_ptr(self.device)), self.ctx.h)
        return out

    def random_actions_steps(self, nsteps, step, seed=1234, out=None):
        """Synthetic actions of `nsteps` consecutive steps in one launch: [nsteps, B, action_dim]."""
        if out is None:
            out = torch.empty((nsteps, self.num_envs, self.action_dim), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_fill_actions_steps(self.ctx.h, int(seed), int(step), int(nsteps),
                                                           out.data_ptr(), _stream_ptr(self.device)), self.ctx.h)
        return out

    def episode_stats(self, clear=False):
        """Device f64[3] = [sum of finished-episode returns, #episodes, #env-steps] since last clear."""
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_episode_stats(self.ctx.h, self._stats.data_ptr(), int(clear),
                                                      _stream_ptr(self.device)), self.ctx.h)
        return self._stats

    def invalid_actions(self):
        v = C.c_uint64()
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_invalid_actions(self.ctx.h, C.byref(v), _stream_ptr(self.device)),
                      self.ctx.h)
        return v.value

    def kernel_timing(self, start):
        """start=True: time the following step launches with dispatch-stamped HIP events;
        start=False: stop and return (total kernel ms, number of timed launches)."""
        tot, cnt = C.c_double(), C.c_int64()
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_kernel_timing(self.ctx.h, 1 if start else 0, C.byref(tot), C.byref(cnt)),
                      self.ctx.h)
        return tot.value, cnt.value

    # ------------------------------------------------------------ state I/O
    def get_state(self):
        """Host copy of the SoA state: {field: numpy array} (see csrc/futbol_state.hpp)."""
        buf = np.zeros(self.ctx.state_bytes, dtype=np.uint8)
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_get_state(self.ctx.h, buf.ctypes.data, 1, _stream_ptr(self.device)),
                      self.ctx.h)
        out = {}
        for name, off, t, cnt in self.ctx.fields:
            dt = np.dtype(_DT[t])
            a = buf[off:off + dt.itemsize * cnt].view(dt)
            if name in _PAIR_FIELDS:  # (x, y) pairs in HBM: returned as the two [Nb * B] arrays
                x, y = _PAIR_FIELDS[name]
                out[x], out[y] = a[0::2].copy(), a[1::2].copy()
            elif name in _GROUP_FIELDS:
                key, n = _GROUP_FIELDS[name]
                B = self.num_envs
                out[key] = a.reshape(-1, B, 2).transpose(0, 2, 1).reshape(-1, B)[:n].reshape(-1).copy()
            else:
                out[name] = a.copy()
        return out

    def set_state(self, state):
        buf = np.zeros(self.ctx.state_bytes, dtype=np.uint8)
        for name, off, t, cnt in self.ctx.fields:
            dt = np.dtype(_DT[t])
            if name in _PAIR_FIELDS:
                x, y = _PAIR_FIELDS[name]
                ax = np.ascontiguousarray(state[x], dtype=dt).reshape(-1)
                ay = np.ascontiguousarray(state[y], dtype=dt).reshape(-1)
                if 2 * ax.size != cnt or 2 * ay.size != cnt:
                    raise ValueError("fields %s/%s: expected %d elements each, got %d/%d" % (x, y, cnt // 2, ax.size, ay.size))
                a = np.empty(cnt, dtype=dt)
                a[0::2], a[1::2] = ax, ay
            elif name in _GROUP_FIELDS:
                key, n = _GROUP_FIELDS[name]
                B = self.num_envs
                v = np.ascontiguousarray(state[key], dtype=dt).reshape(-1)
                if v.size != n * B:
                    raise ValueError("field %s: expected %d elements, got %d" % (key, n * B, v.size))
                full = np.zeros((cnt // B, B), dtype=dt)
                full[:n] = v.reshape(n, B)
                a = full.reshape(-1, 2, B).transpose(0, 2, 1).reshape(-1)
            else:
                a = np.ascontiguousarray(state[name], dtype=dt).reshape(-1)
                if a.size != cnt:
                    raise ValueError("field %s: expected %d elements, got %d" % (name, cnt, a.size))
            buf[off:off + dt.itemsize * cnt] = a.view(np.uint8)
        with torch.cuda.device(self.device):
            nat.check(nat.load().futbol_set_state(self.ctx.h, buf.ctypes.data, 1, _stream_ptr(self.device)),
                      self.ctx.h)

    def close(self):
        if getattr(self, "ctx", None) is not None:
            self.ctx.close()
            self.ctx = None

    # ------------------------------------------------ VecEnv-style plumbing
    def step_async(self, actions):
        self._pending = actions

    def step_wait(self):
        a, self._pending = self._pending, None
        return self.step(a)

    def seed(self, seed=None):
        """Re-seed every env (DummyVecEnv.seed: env i gets seed + i; here one context seed keys every
        env's Philox stream by its global id).  The randomness is counter-based, so re-seeding builds
        a new context with the same configuration: like the reference's constructor it ends in
        reset(), so call reset() before stepping.  seed=None keeps the current seed."""
        if seed is not None and int(seed) != self.seed_value:
            # the new context first: if it cannot be created the env keeps its live one.  (A hipGraph
            # captured before seed() still points at the old context's state and must be re-captured.)
            with torch.cuda.device(self.device):
                ctx = nat.Context(self.ctx.cfg, self.device.index, int(seed), self.env_id_base, self.num_envs)
            old, self.ctx = self.ctx, ctx
            old.close()
            self.seed_value = int(seed)
        return [self.seed_value + i for i in range(self.num_envs)]

    # per-env attributes of the reference envs, read from the device state
    def env_attr(self, name):
        """Per-env values of a reference attribute: v1 `current_time`, `ball_owner_side`; v0 `time`,
        `ball_owner`, `last_ball_owner`, `ai_score`, `opp_score`.  None if `name` is not per-env."""
        st = None
        if self.kind == "v1" and name in ("current_time", "ball_owner_side"):
            st = self.get_state()
            meta = st["meta"].astype(np.uint64)
            if name == "ball_owner_side":
                return ["left" if int(m & np.uint64(7)) == 0 else "right" for m in meta]
            return [_accumulated_time(int((m >> np.uint64(18)) & np.uint64(0x3FFF))) for m in meta]
        if self.kind == "v0" and name in ("time", "ball_owner", "last_ball_owner", "ai_score", "opp_score"):
            from .envs import v0_attrs_from_state
            st = self.get_state()
            return [v0_attrs_from_state(st, i)[name] for i in range(self.num_envs)]
        return None

    def as_sb3(self):
        return SB3VecEnv(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _accumulated_time(steps):
    """current_time after `steps` steps: the reference accumulates 0.1 in fp64
    (envs_v1/futbol_env.py:478); memoised running sums, no per-call loop."""
    while len(_TIMES) <= steps:
        _TIMES.append(_TIMES[-1] + 0.1)
    return _TIMES[steps]


_TIMES = [0.0]


try:  # pragma: no cover - stable-baselines3 is not installed in this image
    from stable_baselines3.common.vec_env import VecEnv as _SB3Base  # type: ignore
except Exception:  # noqa: BLE001
    _SB3Base = object


class SB3VecEnv(_SB3Base):
    """stable-baselines VecEnv interface over a FutbolVecEnv (numpy in/out).

    Rewards are float32 and obs are cast to the observation space dtype, as
    DummyVecEnv does; infos carry `terminal_observation` for done envs and a
    Monitor-style `episode` = {"r": return, "l": length}."""

    def __init__(self, venv):
        self.venv = venv
        self.num_envs = venv.num_envs
        self.observation_space = venv.observation_space
        self.action_space = venv.action_space
        self.metadata = {"render.modes": []}
        self._actions = None
        self._ep_ret = np.zeros(self.num_envs, np.float64)
        self._ep_len = np.zeros(self.num_envs, np.int64)

    def reset(self):
        self._ep_ret[:] = 0
        self._ep_len[:] = 0
        return self.venv.reset().cpu().numpy().astype(self.observation_space.dtype)

    def step_async(self, actions):
        self._actions = np.asarray(actions)

    def step_wait(self):
        obs, rew, done, info = self.venv.step(self._actions)
        obs_np = obs.cpu().numpy().astype(self.observation_space.dtype)
        rew_host = rew.cpu().numpy()  # one device-to-host copy of the rewards
        rew_np = rew_host.astype(np.float32)
        done_np = done.cpu().numpy()
        infos = [{} for _ in range(self.num_envs)]
        self._ep_ret += rew_host.astype(np.float64)
        self._ep_len += 1
        if done_np.any():
            term = info["terminal_observation"].cpu().numpy().astype(self.observation_space.dtype)
            for i in np.nonzero(done_np)[0]:
                infos[i]["terminal_observation"] = term[i]
                infos[i]["episode"] = {"r": float(self._ep_ret[i]), "l": int(self._ep_len[i])}
                self._ep_ret[i] = 0
                self._ep_len[i] = 0
        return obs_np, rew_np, done_np, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def seed(self, seed=None):
        """Re-seeds the envs (a new context, see FutbolVecEnv.seed); the next reset() starts from it."""
        out = self.venv.seed(seed)
        self._ep_ret[:] = 0
        self._ep_len[:] = 0
        return out

    def get_attr(self, attr_name, indices=None):
        """Per-env reference attributes (current_time, ball_owner_side; v0 time, scores, owners) are
        read per env; the others are configuration shared by every env of the vector."""
        idx = list(self._idx(indices))
        per_env = self.venv.env_attr(attr_name)
        if per_env is not None:
            return [per_env[i] for i in idx]
        return [getattr(self.venv, attr_name)] * len(idx)

    def set_attr(self, attr_name, value, indices=None):
        """Attributes are shared by every env of the context: setting one for a subset of the envs
        cannot be represented and raises."""
        if not self._all(indices):
            raise NotImplementedError("set_attr(%r) on a subset of the envs: the attributes of a FutbolVecEnv "
                                      "are shared by all its envs" % attr_name)
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        """Per-env methods of the reference env: `reset` (masked reset of the selected envs; returns their
        observations) and `random_action` (one sample per env).  Any other method acts on the whole
        vector at once, so it is only accepted for all envs and called once."""
        idx = list(self._idx(indices))
        if method_name == "reset":
            mask = np.zeros(self.num_envs, np.uint8)
            mask[idx] = 1
            obs = self.venv.reset(mask).cpu().numpy().astype(self.observation_space.dtype)
            self._ep_ret[idx] = 0
            self._ep_len[idx] = 0
            return [obs[i] for i in idx]
        if method_name == "random_action":
            return [self.venv.action_space.sample() for _ in idx]
        if not self._all(indices):
            raise NotImplementedError("env_method(%r) on a subset of the envs: only reset and random_action are "
                                      "per-env methods of a FutbolVecEnv" % method_name)
        return [getattr(self.venv, method_name)(*args, **kwargs)] * len(idx)

    def _all(self, indices):
        return indices is None or sorted(set(self._idx(indices))) == list(range(self.num_envs))

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._idx(indices))

    def get_images(self):
        return []

    def _idx(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices
