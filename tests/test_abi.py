"""The C ABI boundary (include/futbol.h) without a GPU: the in-tree library
loads, exports every declared symbol, the Python binding covers them all, and
the calls that need no device behave (defaults, error paths).  No kernel runs."""
import ctypes as C
import os
import re

import pytest

from helpers import ROOT

HEADER = os.path.join(ROOT, "include", "futbol.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(futbol_[a-z_0-9]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def nat():
    from gym_futbol_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return _native


def test_library_is_in_tree(nat):
    assert os.path.dirname(nat.LIB_PATH) == os.path.join(ROOT, "gym-futbol_amd", "gym_futbol_amd")


def test_every_declared_symbol_is_exported(nat):
    lib = nat.load()
    names = declared_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name


def test_binding_covers_the_header(nat):
    assert sorted(n for n, _, _ in nat.SIGNATURES) == declared_functions()


def test_config_struct_matches_header(nat):
    # FutbolConfig: 4 int32, 3 double, 6 double, 5 int32 (+ padding) -- keep ctypes in sync
    assert C.sizeof(nat.FutbolConfig) == 4 * 4 + 9 * 8 + 5 * 4 + 4


def test_config_defaults(nat):
    v1 = nat.default_config(nat.ENV_V1, 2)
    assert (v1.width, v1.height, v1.total_time, v1.number_of_player) == (105, 68, 30, 2)
    assert v1.abi_version == nat.ABI_VERSION and v1.auto_reset == 1 and v1.out_dtype == nat.F32
    v0 = nat.default_config(nat.ENV_V0, 0)
    assert (v0.length0, v0.width0, v0.goal_size0, v0.game_time0, v0.player_speed0, v0.shoot_speed0) == \
        (105, 68, 10, 40, 12, 20)
    assert (v0.random_opp0, v0.action_as_int0, v0.one_goal_end0, v0.only_reward_goal0) == (1, 1, 0, 0)
    assert nat.load().futbol_config_default(7, 2, C.byref(nat.FutbolConfig())) != 0


def test_create_rejects_bad_arguments_without_touching_a_device(nat):
    lib = nat.load()
    cfg = nat.default_config(nat.ENV_V1, 2)
    h = C.c_void_p()
    assert lib.futbol_create(C.byref(cfg), 0, 0, 0, 0, C.byref(h)) == -1          # num_envs = 0
    assert b"num_envs" in lib.futbol_last_error(None)
    for bad_n in (0, 11):                                                         # team.py:52-112: 1..10
        cfg.number_of_player = bad_n
        assert lib.futbol_create(C.byref(cfg), 0, 0, 0, 8, C.byref(h)) == -4      # unsupported N
    cfg = nat.default_config(nat.ENV_V1, 2)
    cfg.abi_version = 99
    assert lib.futbol_create(C.byref(cfg), 0, 0, 0, 8, C.byref(h)) == -1
    cfg = nat.default_config(nat.ENV_V1, 2)
    assert lib.futbol_create(C.byref(cfg), 0, 0, 2**32 - 4, 8, C.byref(h)) == -1  # env ids > 32 bits
    cfg = nat.default_config(nat.ENV_V1, 10)                                      # 32-bit per-env offsets
    assert lib.futbol_create(C.byref(cfg), 0, 0, 0, 60_000_000, C.byref(h)) == -1
    assert b"32-bit" in lib.futbol_last_error(None)
    assert lib.futbol_step(None, None, None, None, None, None, None) == -1


def test_solver_layout_query(nat):
    """futbol_solver_layout reports each team size's compiled record / cache layout (host-only): the
    crowded-state parity test reads its slot counts from here, so they cannot drift from the build."""
    lib = nat.load()
    for n in range(1, 11):
        lay = nat.solver_layout(n)
        nb = 2 * n + 1
        assert lay["arbiters"] == nb * 12 + nb * (nb - 1) // 2
        assert 2 <= lay["lds_slots"] <= 8 and 0 <= lay["reg_spill"] <= 8
        assert 1 <= lay["cache_preload"] <= lay["arbiters"] and lay["cache_batch"] >= 1
        assert lay["one_rows"] in (0, 1) and lay["components"] == (1 if nb <= 8 else 0)
    out = (C.c_int32 * 8)()
    assert lib.futbol_solver_layout(0, out, 8) == -1 and lib.futbol_solver_layout(11, out, 8) == -1
    assert lib.futbol_solver_layout(2, None, 8) == -1 and lib.futbol_solver_layout(2, out, 0) == -1
