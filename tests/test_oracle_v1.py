"""Known-answer tests pinning the envs_v1 oracle.

The reference's v1 step needs pymunk (Chipmunk2D), which is absent and not
installable here, so parity with real pymunk is UNPINNED; these hand-derived
KATs pin the oracle's restatement of envs_v1/futbol_env.py + Chipmunk 7's
cpSpaceStep instead.  Expected values are computed in Python with the same
IEEE double operations the reference performs (Python floats are doubles).
"""
import ctypes as C
import math

import numpy as np
import pytest

from helpers import O

L = O.lib()
W, H = 105.0, 68.0


def fresh(n=2, seed=0):
    e = O.OrcV1()
    L.orc_v1_init(C.byref(e), n, W, H, 30.0, seed, 0)
    return e


def quiet(e, n):
    """Zero every velocity / v_bias and forget cached arbiters."""
    for k in range(2 * n + 1):
        e.vx[k] = e.vy[k] = e.bx[k] = e.by[k] = 0.0
    for p in range(e.P):
        e.arb_exists[p] = 0
        e.arb_inlist[p] = 0


def step(e, n, left):
    obs = np.zeros(4 * (2 * n + 1))
    r = C.c_double()
    d = L.orc_v1_step(C.byref(e), np.asarray(left, np.int32), obs, C.byref(r))
    return obs, r.value, bool(d)


@pytest.mark.parametrize("n", list(range(1, 11)))
def test_k1_formation_obs(n):
    """team.py:52-112 formation, futbol_env.py:154-180 normalisation."""
    e = fresh(n)
    obs = np.zeros(4 * (2 * n + 1))
    L.orc_v1_observe(C.byref(e), obs)
    exp = [0.0, 0.0, 0.0, 0.0]
    for side in (0, 1):
        for k in range(n):
            if n <= 3:
                x, y = (W * 0.25 if side == 0 else W * 0.75), (H / (n + 1)) * (k + 1)
            elif n <= 6:
                if k < 3:
                    x, y = ((W * 1) / 6 if side == 0 else (W * 5) / 6), (H / 4) * (k + 1)
                else:
                    x, y = ((W * 2) / 6 if side == 0 else (W * 4) / 6), (H / (n - 3 + 1)) * (k - 2)
            else:
                if k < 4:
                    x, y = ((W * 1) / 8 if side == 0 else (W * 7) / 8), (H / 5) * (k + 1)
                elif k < 7:
                    x, y = ((W * 2) / 8 if side == 0 else (W * 6) / 8), (H / 4) * (k - 3)
                else:
                    x, y = ((W * 3) / 8 if side == 0 else (W * 5) / 8), (H / (n - 7 + 1)) * (k - 6)
            exp += [(x - 52.5) / 55.5, (y - 34.0) / 34.0, 0.0, 0.0]
    assert np.array_equal(obs, np.array(exp))
    if n == 2:  # SURVEY 8c K1 literal
        assert np.allclose(obs, [0, 0, 0, 0, -0.472973, -0.333333, 0, 0, -0.472973, 0.333333, 0, 0,
                                 0.472973, -0.333333, 0, 0, 0.472973, 0.333333, 0, 0], atol=1e-6)


def test_k2_isolated_player_impulse():
    """RIGHT + noop: impulse 20 * m_inv -> dv = 1; position integrates the
    pre-damping velocity, then v *= 0.95**0.1 (cpSpaceStep order)."""
    e = fresh(2)
    quiet(e, 2)
    x0, y0 = e.px[0], e.py[0]
    step(e, 2, [2, 0, 0, 0])
    assert e.px[0] == x0 + 1.0 * 0.1 and e.py[0] == y0
    assert e.vx[0] == 0.9948838031081763 == 1.0 * 0.95 ** 0.1
    assert e.vy[0] == 0.0


def test_k3_clamp_after_position_integration():
    """limit_velocity clamps the stored velocity only; the position of this
    step used the unclamped one."""
    e = fresh(2)
    quiet(e, 2)
    e.vx[0] = 12.0
    x0 = e.px[0]
    step(e, 2, [0, 0, 0, 0])
    assert e.px[0] == x0 + 12.0 * 0.1
    v = 12.0 * 0.95 ** 0.1
    l = math.sqrt(v ** 2 + 0.0 ** 2)
    assert e.vx[0] == v * (10 / l) and abs(e.vx[0] - 10.0) < 1e-14


def _place(e, k, x, y):
    e.px[k], e.py[k] = x, y


def test_k4_shoot_and_pass_impulses():
    n = 2
    # shoot: ball touching A0, ball at rest -> |v_ball| = 120 * m_inv = 12 toward (105, 34)
    e = fresh(n)
    quiet(e, n)
    _place(e, 4, 50.0, 34.0)
    _place(e, 0, 47.6, 34.0)
    bx0 = e.px[4]
    step(e, n, [0, 2, 0, 0])
    fx = 120 * 55.0 / 55.0
    vx = 0.0 / 2 + fx * (1 / 10)
    assert e.px[4] == bx0 + vx * 0.1
    assert e.vx[4] == vx * 0.95 ** 0.1 and e.vy[4] == 0.0
    assert e.owner == 0
    # pass with arrow UP: the only teammate above A0 is A1 -> force 100 toward it, v_ball /= 10
    e = fresh(n)
    quiet(e, n)
    _place(e, 0, 40.0, 20.0)
    _place(e, 4, 40.0, 22.4)
    _place(e, 1, 40.0, 60.0)
    e.vx[4] = 3.0
    step(e, n, [1, 4, 0, 0])
    dy = 60.0 - 22.4
    vy = 0.0 / 10 + (100 * dy / math.sqrt(0.0 ** 2 + dy ** 2)) * (1 / 10)
    assert e.vy[4] == vy * 0.95 ** 0.1
    assert e.vx[4] == (3.0 / 10) * 0.95 ** 0.1


@pytest.mark.parametrize("w,ball,bexp,pexp", [
    (0, (0.5, 10.0), (4.0, 10.0), (1.5, 10.0)),
    (1, (0.5, 50.0), (4.0, 50.0), (1.5, 50.0)),
    (2, (50.0, 67.5), (50.0, 64.0), (50.0, 66.5)),
    (3, (104.5, 10.0), (101.0, 10.0), (103.5, 10.0)),
    (4, (104.5, 50.0), (101.0, 50.0), (103.5, 50.0)),
    (5, (50.0, 0.5), (50.0, 4.0), (50.0, 1.5)),
])
@pytest.mark.parametrize("owner", [0, 1])
def test_k5_out_of_bounds(w, ball, bexp, pexp, owner):
    """check_and_fix_out_bounds (futbol_env.py:247-287), before physics."""
    n = 2
    e = fresh(n)
    quiet(e, n)
    _place(e, 4, *ball)
    e.vx[4] = 7.0
    e.owner = owner
    obs, r, d = step(e, n, [0, 0, 0, 0])
    assert (e.px[4], e.py[4]) == bexp and (e.vx[4], e.vy[4]) == (0.0, 0.0)
    assert e.owner == 1 - owner and r == 0.0
    team = range(n) if owner == 1 else range(n, 2 * n)
    # the picked player was put 1 inward of the old ball position with v = 0, then the
    # physics step may push it off the wall it overlaps: it stays within 1 of the spot
    assert any(abs(e.px[k] - pexp[0]) < 1.0 and abs(e.py[k] - pexp[1]) < 1.0 for k in team)


def test_k6_goal_sign_and_restart():
    """ball_contact_goal + bx > width - 2 -> +1000, formation restart (v_bias carried, D.2)."""
    n = 2
    for x, vx, sign in ((105.5, 5.0, 1), (-0.5, -5.0, -1)):
        e = fresh(n)
        quiet(e, n)
        _place(e, 4, x, 34.0)
        e.vx[4] = vx
        obs, r, d = step(e, n, [0, 0, 0, 0])
        assert (r > 900) if sign > 0 else (r < -900)
        ref = np.zeros(4 * (2 * n + 1))
        L.orc_v1_observe(C.byref(fresh(n)), ref)
        assert np.allclose(obs, ref, atol=1e-3)
        assert e.curr_dt == 0.0001


def test_k7_episode_length():
    e = fresh(2)
    obs = np.zeros(20)
    for t in range(1, 301):
        _, _, d = step(e, 2, [0, 0, 0, 0])
        assert d == (t == 300), t
    assert e.current_time == 30.000000000000156


def test_k8_head_on_collision():
    """Ball hits a resting player: after the 10-iteration sequential-impulse solve
    the relative normal velocity is -bounce (e = 0.2*0.2 on the PRE-damping approach
    speed), momentum is conserved, and the v_bias pair resolves the bias velocity."""
    n = 2
    e = fresh(n)
    quiet(e, n)
    _place(e, 0, 50.0, 34.0)
    _place(e, 4, 52.4, 34.0)
    e.vx[4] = -5.0
    e.curr_dt = 0.1
    L.orc_v1_space_step(C.byref(e), 0.1)
    bounce = (-5.0 - 0.0) * (0.2 * 0.2)
    vrn = e.vx[4] - e.vx[0]
    assert abs(vrn + bounce) < 1e-12
    assert abs((20 * e.vx[0] + 10 * e.vx[4]) - 10 * (-5.0 * 0.95 ** 0.1)) < 1e-12
    dist = (52.4 - 0.5) - 50.0 - 2.5
    bias = -(1 - (0.9 ** 60) ** 0.1) * min(0.0, dist + 0.1) / 0.1
    assert abs((e.bx[4] - e.bx[0]) - bias) < 1e-5  # collisionBias uses 0.9f (float) in Chipmunk
    assert abs(20 * e.bx[0] + 10 * e.bx[4]) < 1e-12


def test_k9_arbiter_persistence_and_warm_start():
    """collisionPersistence = 3 and the NORMAL / CACHED distinction."""
    n = 2
    e = fresh(n)
    quiet(e, n)
    _place(e, 0, 50.0, 34.0)
    _place(e, 4, 52.2, 34.0)
    e.curr_dt = 0.1
    L.orc_v1_space_step(C.byref(e), 0.1)
    pair = 5 * 12 + (0 * 5 - 0 + (4 - 0 - 1))  # circle pair (0, 4)
    assert e.arb_exists[pair] and e.arb_stamp[pair] == e.stamp and e.arb_jn[pair] >= 0.0
    # separate the bodies: the arbiter ages 1, 2, then is dropped on the 3rd untouched step
    _place(e, 4, 80.0, 60.0)
    for age in (1, 2):
        quiet_v = (e.vx[0], e.vx[4])
        L.orc_v1_space_step(C.byref(e), 0.1)
        assert e.arb_exists[pair] and e.stamp - e.arb_stamp[pair] == age and e.arb_state[pair] == 2
    L.orc_v1_space_step(C.byref(e), 0.1)
    assert not e.arb_exists[pair]
    # a player pressed into wall 0 for two steps: the second touch is NORMAL (warm
    # started with jnAcc * dt/prev_dt); with the cache cleared it is FIRST_COLLISION
    seg_pair = 0 * 12 + 0
    base = fresh(n)
    quiet(base, n)
    _place(base, 0, 1.2, 10.0)
    base.vx[0] = -5.0
    base.curr_dt = 0.1
    L.orc_v1_space_step(C.byref(base), 0.1)
    assert base.arb_exists[seg_pair] and base.arb_jn[seg_pair] > 0.0
    a, b = O.OrcV1(), O.OrcV1()
    C.memmove(C.byref(a), C.byref(base), C.sizeof(base))
    C.memmove(C.byref(b), C.byref(base), C.sizeof(base))
    b.arb_exists[seg_pair] = 0
    for x in (a, b):
        x.vx[0] = -5.0
        L.orc_v1_space_step(C.byref(x), 0.1)
    assert a.arb_state[seg_pair] == 1 and b.arb_state[seg_pair] == 0  # NORMAL vs FIRST_COLLISION
    assert a.arb_jn[seg_pair] > 0.0 and b.arb_jn[seg_pair] > 0.0
    # both converge to the same impulse (single contact), through different rounding paths
    assert abs(a.arb_jn[seg_pair] - b.arb_jn[seg_pair]) < 1e-9 * abs(a.arb_jn[seg_pair])
    assert abs(a.vx[0] - b.vx[0]) < 1e-9
