"""envs_v1 kernel vs the CPU oracle, on the GPU.

The kernel is compared BIT-FOR-BIT with oracle/liboracle_portable.so (the
oracle with the kernels' arithmetic: glibc's pow(x, 2) restated for the squares
that feed the state, x*x only for the reward's; see oracle/oracle_math.h):
obs, reward, done, every body's p / v / v_bias and the arbiter cache, at every
step of free-running rollouts with auto-reset, and on teacher-forced crowded
states that exercise multi-contact solves, cached-impulse warm starts and the
LDS->global contact spill.  North-star bar: bit-exact scoring/termination and
<= 1e-5 on positions/velocities -- met here with 0 difference.
"""
import numpy as np
import pytest
import torch

from helpers import (O, npairs, v1_dense_cache, v1_oracle_bodies, v1_oracle_dense_cache, v1_oracle_to_state,
                     v1_state_to_oracle)

pytestmark = pytest.mark.gpu


def _venv(n, B, seed, dtype=torch.float64, base=0):
    from gym_futbol_amd import FutbolVecEnv
    return FutbolVecEnv("v1", B, seed=seed, env_id_base=base, dtype=dtype, number_of_player=n)


def _compare_state(venv, ora, n, B, tag):
    st = venv.get_state()
    ob = v1_oracle_bodies(ora.envs, n, B)
    for f in ("px", "py", "vx", "vy", "bx", "by"):
        d = np.abs(st[f] - ob[f]).max()
        # bitwise: also the sign of zero
        assert np.array_equal(st[f].view(np.uint64), ob[f].view(np.uint64)), "%s: %s differs (max %g)" % (tag, f, d)
    ex, age, jn = v1_dense_cache(st, n, B)
    ex2, age2, jn2 = v1_oracle_dense_cache(ora.envs, n, B)
    assert np.array_equal(ex, ex2), tag + ": arbiter cache membership"
    assert np.array_equal(age[ex], age2[ex2]), tag + ": arbiter ages"
    assert np.array_equal(jn[ex], jn2[ex2]), tag + ": cached jnAcc"
    meta = st["meta"].astype(np.uint64)
    owner = (meta & np.uint64(7)).astype(np.int64)
    assert np.array_equal(owner, np.array([ora.envs[i].owner for i in range(B)])), tag + ": ball_owner_side"
    ev = (meta >> np.uint64(32)).astype(np.int64)
    assert np.array_equal(ev, np.array([ora.envs[i].event for i in range(B)])), tag + ": rng event"


def _layout(n):
    """LDS record slots, register-held spill records and preloaded cache entries of the team size's
    step kernel, read from the loaded library itself (futbol_solver_layout) -- hand-copied tables here
    drifted from the shipped values once (round 4)"""
    from gym_futbol_amd._native import solver_layout
    return solver_layout(n)


@pytest.mark.parametrize("n,B,T", [(2, 1024, 620), (5, 256, 320), (10, 64, 320), (1, 128, 310), (3, 128, 310),
                                   (4, 128, 310), (6, 64, 305), (7, 64, 305), (8, 64, 305), (9, 64, 305),
                                   (2, 200, 310), (5, 70, 305)])  # ragged: the last block has idle lanes
def test_free_running_rollout_bit_exact(n, B, T):
    seed = 7 + n
    venv = _venv(n, B, seed)
    ora = O.V1Vec(B, N=n, seed=seed, portable=True)
    _compare_state(venv, ora, n, B, "after create")
    o_gpu = venv.reset().cpu().numpy()
    o_cpu = ora.reset()
    assert np.array_equal(o_gpu, o_cpu)
    goals = dones = contacts = 0
    for t in range(T):
        a = venv.random_actions(t, seed=1234)
        a_np = a.cpu().numpy().astype(np.int32)
        obs, rew, done, info = venv.step(a)
        o2, r2, d2, term2 = ora.step(a_np)
        o1, r1, d1 = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        assert np.array_equal(d1, d2), "done differs at step %d" % t
        assert np.array_equal(r1.view(np.uint64), r2.view(np.uint64)), "reward differs at step %d: max %g" % (t, np.abs(r1 - r2).max())
        assert np.array_equal(o1.view(np.uint64), o2.view(np.uint64)), "obs differs at step %d: max %g" % (t, np.abs(o1 - o2).max())
        if d1.any():
            assert np.array_equal(info["terminal_observation"].cpu().numpy()[d1].view(np.uint64),
                                  term2[d1].view(np.uint64))
        goals += int((np.abs(r1) > 500).sum())
        dones += int(d1.sum())
        if t % 97 == 0:
            _compare_state(venv, ora, n, B, "step %d" % t)
            contacts += int((v1_dense_cache(venv.get_state(), n, B)[0]).sum())
    _compare_state(venv, ora, n, B, "end")
    # coverage: the rollout must have exercised goals, episode ends and contacts
    assert dones >= B * (T // 300)
    assert goals > 0 and contacts > 0
    venv.close()


def _crowded_states(n, B, seed):
    """Oracle envs in random crowded configurations: bodies overlapping each other
    and the walls / goal boxes, random v, v_bias and random cached arbiters."""
    rng = np.random.default_rng(seed)
    lay = _layout(n)
    ora = O.V1Vec(B, N=n, seed=seed, portable=True)
    nb = 2 * n + 1
    P = nb * 12 + nb * (nb - 1) // 2
    for i in range(B):
        e = ora.envs[i]
        mode = i % 4
        for k in range(nb):
            if mode == 0:  # cluster in the middle
                x, y = 52.5 + rng.normal(0, 1.2), 34 + rng.normal(0, 1.2)
            elif mode == 1:  # piled in a corner / goal mouth
                x, y = rng.choice([0.3, 104.7]) + rng.normal(0, 1.0), rng.choice([1.0, 24.0, 44.0, 67.0]) + rng.normal(0, 1.0)
            elif mode == 2:  # around the left goal box
                x, y = -1.0 + rng.normal(0, 1.0), 34 + rng.normal(0, 8)
            else:  # anywhere
                x, y = rng.uniform(-3, 108), rng.uniform(-3, 71)
            e.px[k], e.py[k] = x, y
            e.vx[k], e.vy[k] = rng.normal(0, 6, 2)
            e.bx[k], e.by[k] = rng.normal(0, 1, 2) * (rng.random() < 0.5)
        e.stamp = 50
        e.curr_dt = [0.1, 0.0001][int(rng.random() < 0.2)]
        e.current_time = 0.0
        # up to 3x (the kernel's register-preloaded entries + one batched read) cached arbiters, sized
        # from the loaded library's own layout (futbol_solver_layout), so that the lookups and the
        # in-place compaction past the preloaded entries run on the first step
        ckn = lay["cache_preload"] + lay["cache_batch"]
        for p in rng.choice(P, size=int(rng.integers(0, min(P, 3 * ckn) + 1)), replace=False):
            p = int(p)
            age = int(rng.integers(0, 3))
            e.arb_exists[p] = 1
            e.arb_stamp[p] = e.stamp - age
            e.arb_state[p] = 1 if age == 0 else 2
            e.arb_inlist[p] = 1 if age == 0 else 0
            e.arb_jn[p] = abs(rng.normal(0, 5))
        e.owner = int(rng.integers(0, 2))
        e.event = int(rng.integers(0, 1000))
    return ora


def _components(e, n):
    """connected components of an oracle env's contact graph (its arbiters in this step's list):
    records sharing a dynamic body are connected; segments belong to the static body"""
    nb = 2 * n + 1
    parent = list(range(nb))

    def find(x):
        while parent[x] != x:
            x = parent[x]
        return x
    pairs = [(i, j) for i in range(nb) for j in range(i + 1, nb)]
    bodies = set()
    for p in range(npairs(n)):
        if not e.arb_inlist[p]:
            continue
        if p < nb * 12:
            bodies.add(p // 12)
        else:
            i, j = pairs[p - nb * 12]
            bodies.update((i, j))
            parent[find(i)] = find(j)
    return len({find(b) for b in bodies})


@pytest.mark.parametrize("n,B", [(2, 2048), (5, 512), (10, 128), (3, 512), (1, 256), (4, 256), (8, 128),
                                 (6, 128), (7, 128), (9, 128)])
def test_teacher_forced_crowded_states(n, B):
    seed = 100 + n
    lay = _layout(n)
    ora = _crowded_states(n, B, seed)
    venv = _venv(n, B, seed)
    st = v1_oracle_to_state(ora.envs, n, B)
    venv.set_state(st)
    # the oracle must see exactly the state the kernel got (stamps are relative)
    v1_state_to_oracle(venv.get_state(), ora.envs, n, B)
    ex0, _, _ = v1_dense_cache(venv.get_state(), n, B)
    assert ex0.sum(1).max() > lay["cache_preload"] + lay["cache_batch"], \
        "some env must hold more cache entries than are preloaded, past one batched read"
    # contact records per env: past the LDS slots the solve holds the first spill records in
    # registers and re-reads the rest from the global spill area in every sweep -- every one of
    # these paths must run (the counts are the library's own, futbol_solver_layout)
    lds_slots, reg_spill = lay["lds_slots"], lay["reg_spill"]
    most = comps = 0
    per_env = np.zeros(B, np.int64)
    for t in range(3):
        a = venv.random_actions(900 + t, seed=4321)
        obs, rew, done, _ = venv.step(a)
        o2, r2, d2, _ = ora.step(a.cpu().numpy().astype(np.int32))
        cnt = np.array([int(np.sum(np.asarray(e.arb_inlist))) for e in ora.envs])
        per_env = np.maximum(per_env, cnt)
        most = max(most, int(cnt.max()))
        if n <= 3:  # the per-component split solve (Nb <= 8) must see multi-component envs
            comps = max(comps, max(_components(e, n) for e in ora.envs))
        assert np.array_equal(done.cpu().numpy(), d2)
        assert np.array_equal(rew.cpu().numpy(), r2), "step %d reward max diff %g" % (
            t, np.abs(rew.cpu().numpy() - r2).max())
        assert np.array_equal(obs.cpu().numpy(), o2), "step %d obs max diff %g" % (
            t, np.abs(obs.cpu().numpy() - o2).max())
        _compare_state(venv, ora, n, B, "crowded step %d" % t)
    ex, _, _ = v1_dense_cache(venv.get_state(), n, B)
    if n > 1:  # 1v1 (3 bodies) never holds more than its 8 LDS slots in practice
        assert ex.sum(1).max() > 8, "crowded states must overflow the LDS contact slots"
        assert most > lds_slots + reg_spill, "some env must have records past the register-held spill slots"
        if reg_spill:  # an env whose spill records all fit the register-held ones, too
            assert ((per_env > lds_slots) & (per_env <= lds_slots + reg_spill)).any(), \
                "some env must spill into the register-held records only"
    else:
        assert most >= lds_slots - 2, "some 1v1 env must come close to filling its LDS slots"
    assert n > 3 or comps >= 2, "some env must have a contact graph of two or more components"
    venv.close()


@pytest.mark.parametrize("n,B", [(2, 512), (5, 128), (10, 64), (1, 128), (3, 128), (4, 64), (7, 64)])
def test_float32_outputs_are_the_cast_of_float64(n, B):
    """The float-output kernel instances (the default of make()) against the double ones."""
    a64, a32 = _venv(n, B, 3, torch.float64), _venv(n, B, 3, torch.float32)
    o64, o32 = a64.reset(), a32.reset()
    assert torch.equal(o64.float(), o32)
    for t in range(310):
        act = a64.random_actions(t)
        r64 = a64.step(act)
        r32 = a32.step(act)
        assert torch.equal(r64[0].float(), r32[0]) and torch.equal(r64[1].float(), r32[1])
        assert torch.equal(r64[2], r32[2])


def test_sharding_invariance():
    """An env's trajectory depends only on its global id, not on the shard it lives in."""
    n, B = 2, 256
    full = _venv(n, B, 11)
    lo = _venv(n, B // 2, 11, base=0)
    hi = _venv(n, B // 2, 11, base=B // 2)
    f0 = full.reset()
    assert torch.equal(f0, torch.cat([lo.reset(), hi.reset()]))
    for t in range(320):
        a = full.random_actions(t)
        of, rf, df, _ = full.step(a)
        ol, rl, dl, _ = lo.step(a[: B // 2].contiguous())
        oh, rh, dh, _ = hi.step(a[B // 2:].contiguous())
        assert torch.equal(of, torch.cat([ol, oh])) and torch.equal(rf, torch.cat([rl, rh]))
        assert torch.equal(df, torch.cat([dl, dh]))


def _rollout_equal(venv, ora, n, B, T, tag):
    assert np.array_equal(venv.reset().cpu().numpy(), ora.reset())
    for t in range(T):
        a = venv.random_actions(t, seed=77)
        obs, rew, done, info = venv.step(a)
        o2, r2, d2, term2 = ora.step(a.cpu().numpy().astype(np.int32))
        assert np.array_equal(done.cpu().numpy(), d2), (tag, t)
        assert np.array_equal(rew.cpu().numpy().view(np.uint64), r2.view(np.uint64)), (tag, t)
        assert np.array_equal(obs.cpu().numpy().view(np.uint64), o2.view(np.uint64)), (tag, t)
    _compare_state(venv, ora, n, B, tag)


@pytest.mark.parametrize("n", [2, 5])
def test_generic_geometry_kernel(n, monkeypatch):
    """The runtime-geometry instance (forced with FUTBOL_GENERIC=1) on the default field."""
    monkeypatch.setenv("FUTBOL_GENERIC", "1")
    B = 256
    venv = _venv(n, B, seed=41)
    _rollout_equal(venv, O.V1Vec(B, N=n, seed=41, portable=True), n, B, 320, "generic")
    venv.close()


def test_custom_field_size():
    """A non-default width/height (Futbol(width=90, height=60)) selects the generic instance."""
    from gym_futbol_amd import FutbolVecEnv
    B, n = 256, 2
    venv = FutbolVecEnv("v1", B, seed=3, dtype=torch.float64, number_of_player=n, width=90, height=60)
    _rollout_equal(venv, O.V1Vec(B, N=n, seed=3, width=90.0, height=60.0, portable=True), n, B, 320, "90x60")
    venv.close()


@pytest.mark.parametrize("n,B", [(2, 512), (5, 256), (3, 512), (1, 256), (6, 128)])
def test_goal_restart_micro_step(n, B):
    """A goal's restart micro-step (space.step(1e-4) from formation) runs the per-lane no-contact
    path: teacher-forced states with the ball about to cross the right goal line (or the left
    one), random v_bias and random cached arbiters of every age, compared with the oracle
    right after the goal step (arbiter ages and compaction included) and for a few steps more."""
    seed = 300 + n
    ora = _crowded_states(n, B, seed)
    rng = np.random.default_rng(seed + 1)
    nb = 2 * n + 1
    for i in range(B):
        e = ora.envs[i]
        right = i % 2 == 0
        e.px[nb - 1], e.py[nb - 1] = (103.8 if right else 1.2), 34 + rng.uniform(-6, 6)
        e.vx[nb - 1], e.vy[nb - 1] = (18.0 if right else -18.0), 0.0
        for k in range(nb - 1):  # players out of the way of the ball
            e.px[k], e.py[k] = rng.uniform(20, 85), rng.uniform(5, 63)
    venv = _venv(n, B, seed)
    venv.set_state(v1_oracle_to_state(ora.envs, n, B))
    v1_state_to_oracle(venv.get_state(), ora.envs, n, B)
    a = torch.zeros((B, 2 * n), dtype=torch.uint8, device=venv.device)  # left team: noop
    for t in range(4):
        obs, rew, done, _ = venv.step(a)
        o2, r2, d2, _ = ora.step(a.cpu().numpy().astype(np.int32))
        r1 = rew.cpu().numpy()
        if t == 0:
            assert (np.abs(r1) > 500).mean() > 0.9, "most envs must score on the first step"
        assert np.array_equal(r1.view(np.uint64), r2.view(np.uint64))
        assert np.array_equal(obs.cpu().numpy().view(np.uint64), o2.view(np.uint64))
        _compare_state(venv, ora, n, B, "goal step %d" % t)
    venv.close()


@pytest.mark.parametrize("n,B", [(2, 512), (5, 128)])
def test_reset_with_large_v_bias(n, B):
    """reset() keeps v_bias; with |v_bias| beyond the no-contact bound of the
    formation micro-step (half of the envs, ~1e5) the bodies move by ~10 in space.step(1e-4)
    and may collide, so those lanes take the full cpSpaceStep: both paths vs the oracle."""
    seed = 500 + n
    ora = _crowded_states(n, B, seed)
    rng = np.random.default_rng(seed)
    nb = 2 * n + 1
    for i in range(B):
        e = ora.envs[i]
        s = 1e5 if i % 2 else 5.0
        for k in range(nb):
            e.bx[k], e.by[k] = rng.normal(0, s, 2)
    venv = _venv(n, B, seed)
    venv.set_state(v1_oracle_to_state(ora.envs, n, B))
    v1_state_to_oracle(venv.get_state(), ora.envs, n, B)
    o1 = venv.reset().cpu().numpy()
    o2 = ora.reset()
    assert np.array_equal(o1.view(np.uint64), o2.view(np.uint64))
    _compare_state(venv, ora, n, B, "reset")
    assert np.abs(o1[1::2, :2]).max() > 0.05, "the large-v_bias envs must have moved off formation"
    for t in range(3):
        a = venv.random_actions(t, seed=99)
        obs, rew, done, _ = venv.step(a)
        o2, r2, d2, _ = ora.step(a.cpu().numpy().astype(np.int32))
        assert np.array_equal(obs.cpu().numpy().view(np.uint64), o2.view(np.uint64))
        assert np.array_equal(rew.cpu().numpy().view(np.uint64), r2.view(np.uint64))
        _compare_state(venv, ora, n, B, "after reset step %d" % t)
    venv.close()


def _out_of_bounds_states(n, B, seed):
    """Oracle envs with the ball touching one of the six wall segments (envs_v1/futbol_env.py:247-287:
    walls 0/1 left, 2 top, 3/4 right, 5 bottom; every 8th env in a corner, where two walls hit and the
    first in order wins), every player at least 4 from the ball (no touch: the action phase leaves the
    ball where it is), random owner and RNG event, so that the restart's random.choice picks every
    player of both teams"""
    rng = np.random.default_rng(seed)
    ora = O.V1Vec(B, N=n, seed=seed, portable=True)
    nb = 2 * n + 1
    ball = nb - 1
    corners = [(0.5, 0.5), (0.5, 67.5), (104.5, 0.5), (104.5, 67.5)]
    for i in range(B):
        e = ora.envs[i]
        w = i % 6
        if i % 8 == 7:
            bx, by = corners[(i // 8) % 4]
        elif w in (0, 3):
            bx, by = (0.5 if w == 0 else 104.5) + rng.uniform(-0.4, 0.4), rng.uniform(2, 22)
        elif w in (1, 4):
            bx, by = (0.5 if w == 1 else 104.5) + rng.uniform(-0.4, 0.4), rng.uniform(46, 66)
        else:
            bx, by = rng.uniform(5, 100), (67.5 if w == 2 else 0.5) + rng.uniform(-0.4, 0.4)
        e.px[ball], e.py[ball] = bx, by
        e.vx[ball], e.vy[ball] = rng.normal(0, 3, 2)
        for k in range(nb - 1):
            while True:
                x, y = rng.uniform(4, 101), rng.uniform(4, 64)
                if (x - bx) ** 2 + (y - by) ** 2 > 16:
                    break
            e.px[k], e.py[k] = x, y
            e.vx[k], e.vy[k] = rng.normal(0, 3, 2)
            e.bx[k] = e.by[k] = 0.0
        e.stamp = 50
        e.curr_dt = 0.1
        e.owner = int(rng.integers(0, 2))
        e.event = int(rng.integers(0, 1 << 20))
    return ora


@pytest.mark.parametrize("rollout", [0, 1])
@pytest.mark.parametrize("generic", [0, 1])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("n", [9, 10])
def test_out_of_bounds_every_pick(n, dtype, generic, rollout, monkeypatch):
    """Every leaf of the out-of-bounds restart (check_and_fix_out_bounds, envs_v1/futbol_env.py:256-287:
    the new owner team's random.choice places player `pick` at the ball + (+-1, 0) / (0, +-1)) on every
    compiled step-kernel instance of N = 9 and 10 (f64 / f32 outputs x default / runtime geometry x
    step / rollout): the kernels compute that player's new position in each leaf of a switch over
    `pick`, where the ISA listing shows register copies that are never read.
    Teacher-forced states put the ball on each wall; the oracle reports the wall and the pick of each
    env, and every (wall, pick) pair of both teams must occur; obs / reward / done and the full state
    are compared bit for bit after the restart step and two more."""
    monkeypatch.setenv("FUTBOL_GENERIC", "1" if generic else "0")
    B = 2048
    seed = 700 + n
    ora = _out_of_bounds_states(n, B, seed)
    venv = _venv(n, B, seed, dtype)
    venv.set_state(v1_oracle_to_state(ora.envs, n, B))
    v1_state_to_oracle(venv.get_state(), ora.envs, n, B)
    a = torch.zeros((3, B, 2 * n), dtype=torch.uint8, device=venv.device)  # left team: noop
    a[1:] = venv.random_actions_steps(2, 1, seed=55)
    a_np = a.cpu().numpy().astype(np.int32)
    if rollout:
        obs, rew, done, _ = venv.rollout(a)
        outs = [(obs[t].cpu().numpy(), rew[t].cpu().numpy(), done[t].cpu().numpy()) for t in range(3)]
    else:
        outs = []
        for t in range(3):
            o, r, d, _ = venv.step(a[t])
            outs.append((o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy()))
    seen = set()
    cast = np.float32 if dtype == torch.float32 else np.float64
    ut = np.uint32 if dtype == torch.float32 else np.uint64
    for t in range(3):
        o2, r2, d2, _ = ora.step(a_np[t])
        if t == 0:
            for e in ora.envs:
                assert e.last_out_wall >= 0, "every env must restart from out of bounds on the first step"
                seen.add((int(e.last_out_wall), int(e.last_out_pick)))
        o1, r1, d1 = outs[t]
        assert np.array_equal(d1.astype(bool), d2), "done, step %d" % t
        assert np.array_equal(r1.view(ut), r2.astype(cast).view(ut)), "reward, step %d" % t
        bad = ~(o1.view(ut) == o2.astype(cast).view(ut)).all(axis=1)
        assert not bad.any(), "obs of env %d at step %d (wall %d)" % (int(np.flatnonzero(bad)[0]), t,
                                                                        ora.envs[int(np.flatnonzero(bad)[0])].last_out_wall)
    _compare_state(venv, ora, n, B, "out of bounds, 3 steps")
    missing = {(w, p) for w in range(6) for p in range(2 * n)} - seen
    assert not missing, "uncovered (wall, pick) leaves: %s" % sorted(missing)[:10]
    venv.close()
