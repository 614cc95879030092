"""ctypes front-end of the C oracle -- TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  Builds oracle/_build/*.so with `make` on first use if they are missing.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MAXN = 10
MAXB = 2 * MAXN + 1
NSEG = 12
MAXP = MAXB * NSEG + MAXB * (MAXB - 1) // 2


class OrcV1(C.Structure):
    _fields_ = [("N", C.c_int32), ("Nb", C.c_int32), ("P", C.c_int32),
                ("width", C.c_double), ("height", C.c_double), ("total_time", C.c_double),
                ("seed", C.c_uint64), ("env_id", C.c_uint32),
                ("px", C.c_double * MAXB), ("py", C.c_double * MAXB),
                ("vx", C.c_double * MAXB), ("vy", C.c_double * MAXB),
                ("bx", C.c_double * MAXB), ("by", C.c_double * MAXB),
                ("current_time", C.c_double), ("owner", C.c_int32), ("event", C.c_uint32),
                ("stamp", C.c_uint32), ("curr_dt", C.c_double),
                ("arb_exists", C.c_int32 * MAXP), ("arb_stamp", C.c_uint32 * MAXP),
                ("arb_state", C.c_int32 * MAXP), ("arb_inlist", C.c_int32 * MAXP),
                ("arb_jn", C.c_double * MAXP), ("n_out", C.c_uint32), ("n_goal", C.c_uint32),
                ("last_out_wall", C.c_int32), ("last_out_pick", C.c_int32)]


class OrcV0(C.Structure):
    _fields_ = [("length", C.c_double), ("width", C.c_double), ("goal_size", C.c_double),
                ("game_time", C.c_double), ("player_speed", C.c_double), ("shoot_speed", C.c_double),
                ("one_goal_end", C.c_int32), ("only_reward_goal", C.c_int32), ("random_opp", C.c_int32),
                ("seed", C.c_uint64), ("env_id", C.c_uint32),
                ("obs", (C.c_double * 5) * 6), ("ball_owner", C.c_int32), ("last_ball_owner", C.c_int32),
                ("time", C.c_double), ("ai_score", C.c_int32), ("opp_score", C.c_int32),
                ("views_live", C.c_int32), ("ai_view", (C.c_double * 2) * 2),
                ("opp_view_frozen", (C.c_double * 2) * 2), ("pending_done", C.c_int32),
                ("event", C.c_uint32)]


_libs = {}


def lib(portable=False):
    name = "liboracle_portable.so" if portable else "liboracle.so"
    if name in _libs:
        return _libs[name]
    # FUTBOL_ORACLE_SANITIZE=1: the ASan + UBSan builds of `make sanitize` (tests/conftest.py)
    san = os.environ.get("FUTBOL_ORACLE_SANITIZE") == "1"
    path = os.path.join(HERE, "_build", "san" if san else "", name)
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", HERE] + (["sanitize"] if san else []))
    L = C.CDLL(path)
    dp = np.ctypeslib.ndpointer(np.float64, flags="C")
    ip = np.ctypeslib.ndpointer(np.int32, flags="C")
    up = np.ctypeslib.ndpointer(np.uint8, flags="C")
    L.orc_v1_init.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_double, C.c_uint64, C.c_uint32]
    L.orc_v1_reset.argtypes = [C.c_void_p, C.c_void_p]
    L.orc_v1_step.argtypes = [C.c_void_p, ip, dp, C.POINTER(C.c_double)]
    L.orc_v1_step.restype = C.c_int
    L.orc_v1_observe.argtypes = [C.c_void_p, dp]
    L.orc_v1_space_step.argtypes = [C.c_void_p, C.c_double]
    L.orc_v1_vec_step.argtypes = [C.c_void_p, C.c_int, ip, dp, dp, up, C.c_void_p, C.c_int]
    L.orc_v1_run.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.POINTER(C.c_double)]
    L.orc_v1_run.restype = C.c_int
    L.orc_v1_vec_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
    L.orc_v1_vec_run.restype = C.c_longlong
    L.orc_v0_vec_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
    L.orc_v0_vec_run.restype = C.c_longlong
    L.orc_libm_check.argtypes = [C.c_int64, C.c_double, C.c_double, C.c_uint64] + [C.POINTER(C.c_int64)] * 3
    L.orc_v0_init.argtypes = [C.c_void_p] + [C.c_double] * 6 + [C.c_int] * 3 + [C.c_uint64, C.c_uint32]
    L.orc_v0_reset.argtypes = [C.c_void_p, C.c_void_p]
    L.orc_v0_step.argtypes = [C.c_void_p, C.c_int32, C.c_int32, dp, C.POINTER(C.c_double)]
    L.orc_v0_step.restype = C.c_int
    L.orc_v0_vec_step.argtypes = [C.c_void_p, C.c_int, ip, dp, dp, up, C.c_void_p, C.c_int]
    L.orc_v1_set_sq_mask.argtypes = [C.c_int]
    L.orc_philox.argtypes = [C.POINTER(C.c_uint32)] * 3
    L.orc_draw_u01.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                               C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.orc_sizeof_v1.restype = C.c_int
    L.orc_sizeof_v0.restype = C.c_int
    assert L.orc_sizeof_v1() == C.sizeof(OrcV1), (L.orc_sizeof_v1(), C.sizeof(OrcV1))
    assert L.orc_sizeof_v0() == C.sizeof(OrcV0), (L.orc_sizeof_v0(), C.sizeof(OrcV0))
    _libs[name] = L
    return L


class V1Vec:
    """B independent envs_v1 envs with DummyVecEnv semantics (auto-reset)."""

    def __init__(self, B, N=2, seed=0, env_id_base=0, width=105.0, height=68.0, total_time=30.0,
                 portable=False):
        self.L = lib(portable)
        self.B, self.N = B, N
        self.envs = (OrcV1 * B)()
        for i in range(B):
            self.L.orc_v1_init(C.byref(self.envs[i]), N, width, height, total_time, seed, env_id_base + i)
        self.obs_dim = 4 * (2 * N + 1)

    def reset(self):
        obs = np.zeros((self.B, self.obs_dim), np.float64)
        for i in range(self.B):
            self.L.orc_v1_reset(C.byref(self.envs[i]), obs[i].ctypes.data)
        return obs

    def step(self, actions, nthreads=1):
        actions = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.B, 2 * self.N)
        obs = np.zeros((self.B, self.obs_dim), np.float64)
        rew = np.zeros(self.B, np.float64)
        done = np.zeros(self.B, np.uint8)
        term = np.zeros((self.B, self.obs_dim), np.float64)
        self.L.orc_v1_vec_step(C.byref(self.envs), self.B, actions, obs, rew, done, term.ctypes.data, nthreads)
        return obs, rew, done.astype(bool), term

    def run(self, nsteps, act_seed=1234, nthreads=1):
        """nsteps steps of every env in one C call (synthetic Philox actions, auto-reset), envs split
        over nthreads threads; returns (finished episodes, their return sum)."""
        ret = C.c_double()
        eps = self.L.orc_v1_vec_run(C.byref(self.envs), self.B, int(nsteps), act_seed, int(nthreads), C.byref(ret))
        return eps, ret.value


class V0Vec:
    """B independent v0 FutbolEnv envs with DummyVecEnv semantics."""

    def __init__(self, B, seed=0, env_id_base=0, random_opp=False, one_goal_end=False,
                 only_reward_goal=False, length=105.0, width=68.0, goal_size=10.0, game_time=40.0,
                 player_speed=12.0, shoot_speed=20.0, portable=False):
        self.L = lib(portable)
        self.B = B
        self.envs = (OrcV0 * B)()
        for i in range(B):
            self.L.orc_v0_init(C.byref(self.envs[i]), length, width, goal_size, game_time, player_speed,
                               shoot_speed, int(one_goal_end), int(only_reward_goal), int(random_opp),
                               seed, env_id_base + i)

    def reset(self):
        obs = np.zeros((self.B, 6, 5), np.float64)
        for i in range(self.B):
            self.L.orc_v0_reset(C.byref(self.envs[i]), obs[i].ctypes.data)
        return obs

    def step(self, actions, nthreads=1):
        actions = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.B)
        obs = np.zeros((self.B, 6, 5), np.float64)
        rew = np.zeros(self.B, np.float64)
        done = np.zeros(self.B, np.uint8)
        term = np.zeros((self.B, 6, 5), np.float64)
        self.L.orc_v0_vec_step(C.byref(self.envs), self.B, actions, obs.reshape(-1), rew, done,
                               term.ctypes.data, nthreads)
        return obs, rew, done.astype(bool), term

    def run(self, nsteps, act_seed=1234, nthreads=1):
        """nsteps steps of every env in one C call (synthetic Philox actions, auto-reset), envs split
        over nthreads threads; returns (finished episodes, the sum of every step's reward)."""
        ret = C.c_double()
        eps = self.L.orc_v0_vec_run(C.byref(self.envs), self.B, int(nsteps), act_seed, int(nthreads), C.byref(ret))
        return eps, ret.value


def philox(ctr, key, portable=False):
    L = lib(portable)
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    L.orc_philox(c, k, o)
    return tuple(o)
