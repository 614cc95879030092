"""envs_v1 `x*x` (the kernels, the portable oracle) vs libm `pow(x, 2)` (the reference's Python `**2`,
the faithful oracle) over a whole workload: both oracle builds step the same envs with the same
synthetic actions (Philox tag 1, seed 1234: the bench's left-team stream) and every step is compared.
TEST INFRASTRUCTURE (tests/test_oracle_modes.py, scripts/v1_sq_divergence.py).

Reference call sites of `**2`: get_vec (envs_v1/futbol_env.py:56-59), _ball_to_team_distance_arr
(:485-491) and pymunk 5's Vec2d.length inside limit_velocity (ball.py:49-56, player.py:45-52)."""
import time

import numpy as np

from helpers import O


def divergence(n, B, T, seed=0, nthreads=8, act_seed=1234, b_mask=None):
    """Step B envs (N = n) T steps in the faithful build and in the portable one (b_mask None) -- or in
    the faithful build with x*x at the call sites of b_mask (orc_v1_set_sq_mask) -- and compare."""
    a = O.V1Vec(B, N=n, seed=seed, portable=False)
    b = O.V1Vec(B, N=n, seed=seed, portable=b_mask is None)
    L = O.lib(False)

    def mask(m):
        if b_mask is not None:
            L.orc_v1_set_sq_mask(m)
    oa, ob = a.reset(), b.reset()
    assert np.array_equal(oa, ob)
    sa, sb = np.ctypeslib.as_array(a.envs), np.ctypeslib.as_array(b.envs)
    rng = np.random.default_rng(act_seed)
    bit_first = np.full(B, -1, np.int64)      # first step with any bit of obs / reward different
    obs_first = np.full(B, -1, np.int64)      # first step with any bit of obs different
    disc = {k: np.zeros(B, bool) for k in ("done", "goal", "owner", "out_of_bounds", "rng_events", "reward_sign")}
    max_obs = max_rew = 0.0
    max_pos = max_vel = 0.0
    t0 = time.perf_counter()
    for t in range(T):
        act = rng.integers(0, 5, (B, 2 * n), dtype=np.int32)
        mask(0)
        oa, ra, da, _ = a.step(act, nthreads=nthreads)
        mask(b_mask)
        ob, rb, db, _ = b.step(act, nthreads=nthreads)
        mask(0)
        dob = np.abs(oa - ob)
        drw = np.abs(ra - rb)
        max_obs = max(max_obs, float(dob.max()))
        max_rew = max(max_rew, float(drw.max()))
        # obs layout: per body (x, y, vx, vy)
        max_pos = max(max_pos, float(dob.reshape(B, -1, 4)[:, :, :2].max()))
        max_vel = max(max_vel, float(dob.reshape(B, -1, 4)[:, :, 2:].max()))
        obit = (oa.view(np.uint64) != ob.view(np.uint64)).any(1)
        anybit = obit | (ra.view(np.uint64) != rb.view(np.uint64))
        bit_first[(bit_first < 0) & anybit] = t
        obs_first[(obs_first < 0) & obit] = t
        disc["done"] |= da != db
        disc["goal"] |= sa["n_goal"] != sb["n_goal"]
        disc["owner"] |= sa["owner"] != sb["owner"]
        disc["out_of_bounds"] |= sa["n_out"] != sb["n_out"]
        disc["rng_events"] |= sa["event"] != sb["event"]
        disc["reward_sign"] |= np.sign(ra) != np.sign(rb)
    anyd = np.zeros(B, bool)
    for v in disc.values():
        anyd |= v
    return {"N": n, "envs": B, "steps": T, "seed": seed,
            "compared": "faithful vs portable" if b_mask is None else "faithful vs faithful with x*x at sites %d" % b_mask, "actions": "numpy default_rng(%d) integers [0, 5)" % act_seed,
            "seconds": time.perf_counter() - t0,
            "envs_any_bit_different": int((bit_first >= 0).sum()),
            "envs_obs_bit_different": int((obs_first >= 0).sum()),
            "median_first_bit_step": float(np.median(bit_first[bit_first >= 0])) if (bit_first >= 0).any() else None,
            "max_abs_obs_diff": max_obs, "max_abs_pos_diff": max_pos, "max_abs_vel_diff": max_vel,
            "max_abs_reward_diff": max_rew,
            "envs_discrete_diff": {k: int(v.sum()) for k, v in disc.items()},
            "envs_any_discrete_diff": int(anyd.sum()),
            "goals": int(sa["n_goal"].sum()), "out_of_bounds": int(sa["n_out"].sum())}
