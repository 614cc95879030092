"""ctypes binding of include/futbol.h (libfutbol_amd.so, built in-tree by build.py).

There is no CPU fallback: if the library is missing or no GPU is visible,
creating an env raises.  The library is loaded from this package directory
(never from site-packages), so the round-end checks see it as in-tree code.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfutbol_amd.so")
# diagnostic builds (bench.py --stamps) are selected by name, always from this directory
if os.environ.get("FUTBOL_LIB_VARIANT"):
    LIB_PATH = os.path.join(HERE, "libfutbol_amd_%s.so" % os.environ["FUTBOL_LIB_VARIANT"])

ENV_V0, ENV_V1 = 0, 1
F32, F64 = 0, 1
ABI_VERSION = 1
TYPE_CODES = {0: "f8", 1: "u8", 2: "u4", 3: "u2", 4: "u1"}


class NativeError(RuntimeError):
    pass


class FutbolConfig(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("env_kind", C.c_int32), ("out_dtype", C.c_int32),
                ("number_of_player", C.c_int32),
                ("width", C.c_double), ("height", C.c_double), ("total_time", C.c_double),
                ("length0", C.c_double), ("width0", C.c_double), ("goal_size0", C.c_double),
                ("game_time0", C.c_double), ("player_speed0", C.c_double), ("shoot_speed0", C.c_double),
                ("one_goal_end0", C.c_int32), ("action_as_int0", C.c_int32), ("only_reward_goal0", C.c_int32),
                ("random_opp0", C.c_int32), ("auto_reset", C.c_int32)]


# (name, restype, argtypes) for every symbol declared in include/futbol.h
SIGNATURES = [
    ("futbol_config_default", C.c_int, [C.c_int32, C.c_int32, C.POINTER(FutbolConfig)]),
    ("futbol_create", C.c_int, [C.POINTER(FutbolConfig), C.c_int32, C.c_uint64, C.c_uint64, C.c_int32,
                                C.POINTER(C.c_void_p)]),
    ("futbol_destroy", C.c_int, [C.c_void_p]),
    ("futbol_last_error", C.c_char_p, [C.c_void_p]),
    ("futbol_dims", C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("futbol_reset", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("futbol_step", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                              C.c_void_p]),
    ("futbol_rollout", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p]),
    ("futbol_fill_actions", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]),
    ("futbol_fill_actions_steps", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int32, C.c_void_p,
                                             C.c_void_p]),
    ("futbol_episode_stats", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    ("futbol_invalid_actions", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p]),
    ("futbol_state_bytes", C.c_int, [C.c_void_p, C.POINTER(C.c_size_t)]),
    ("futbol_state_field", C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                                     C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    ("futbol_get_state", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    ("futbol_set_state", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    ("futbol_episode_limit", C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    ("futbol_debug_stamps", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]),
    ("futbol_kernel_timing", C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    ("futbol_stream_copy", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("futbol_solver_layout", C.c_int, [C.c_int32, C.POINTER(C.c_int32), C.c_int32]),
]

_lib = None


def load():
    """Load libfutbol_amd.so (raises NativeError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError("libfutbol_amd.so not built: run `python gym-futbol_amd/build.py` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, ctx=None):
    if rc != 0:
        msg = load().futbol_last_error(ctx)
        raise NativeError("futbol native call failed (%d): %s" % (rc, msg.decode() if msg else ""))
    return rc


def default_config(env_kind, number_of_player=2):
    cfg = FutbolConfig()
    check(load().futbol_config_default(env_kind, number_of_player, C.byref(cfg)))
    return cfg


SOLVER_LAYOUT_KEYS = ("lds_slots", "reg_spill", "cache_preload", "cache_batch", "arbiters", "one_rows",
                      "components", "sq_batch")


def solver_layout(number_of_player):
    """The envs_v1 step kernel's solver layout for a team size, as compiled into the loaded library
    (futbol_solver_layout; host-only, no GPU needed)."""
    out = (C.c_int32 * len(SOLVER_LAYOUT_KEYS))()
    check(load().futbol_solver_layout(number_of_player, out, len(SOLVER_LAYOUT_KEYS)))
    return dict(zip(SOLVER_LAYOUT_KEYS, (int(v) for v in out)))


class Context:
    """Owns one FutbolCtx (B envs on one GPU)."""

    def __init__(self, cfg, device, seed, env_id_base, num_envs):
        lib = load()
        h = C.c_void_p()
        check(lib.futbol_create(C.byref(cfg), int(device), int(seed) & (2**64 - 1), int(env_id_base),
                                int(num_envs), C.byref(h)))
        self.h = h
        self.cfg = cfg
        od, ad, n = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib.futbol_dims(h, C.byref(od), C.byref(ad), C.byref(n)), h)
        self.obs_dim, self.action_dim, self.num_envs = od.value, ad.value, n.value
        k = C.c_int32()
        check(lib.futbol_episode_limit(h, C.byref(k)), h)
        self.episode_steps = k.value
        nb = C.c_size_t()
        check(lib.futbol_state_bytes(h, C.byref(nb)), h)
        self.state_bytes = nb.value
        self.fields = []
        i = 0
        while True:
            name, off, tc, cnt = C.c_char_p(), C.c_size_t(), C.c_int32(), C.c_int64()
            if lib.futbol_state_field(h, i, C.byref(name), C.byref(off), C.byref(tc), C.byref(cnt)) != 0:
                break
            self.fields.append((name.value.decode(), off.value, TYPE_CODES[tc.value], cnt.value))
            i += 1

    def close(self):
        if getattr(self, "h", None):
            load().futbol_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
