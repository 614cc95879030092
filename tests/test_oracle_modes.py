"""Faithful (libm pow / sin / cos, = CPython) vs portable (= the kernels) oracle builds.

v0: the portable build computes the reference's `x**2` and math.sin / math.cos with the glibc
restatements (tests/test_glibc_sincos.py pins them against the host libm), so the two builds must
agree BIT FOR BIT on whole rollouts -- the kernels' bit-exact parity with the portable build is a
bit-exact parity with the reference's own arithmetic (and tests/test_oracle_v0.py checks it against
1 024-env reference fingerprints).

envs_v1: the kernels (and the portable build) compute glibc's pow(x, 2) where the reference's `**2`
feeds the state (_process_action's get_vec, pymunk's Vec2d.length in limit_velocity) and x*x only in
the reward's squares, so the two builds' observations (every position and velocity) are bit-identical
and only the rewards' last bits may differ.  (Round 3 squared with x*x everywhere: at 8 192 5v5 envs
x 600 steps one env then flipped its ball owner and an out-of-bounds restart, traced to
_process_action's get_vec with tests/sq_divergence.py's per-site mask.)

(Before round 3 the faithful build was not faithful: gcc turned pow(x, 2.0) into x*x and fused
sin(x), cos(x) into glibc's sincos(); -fno-builtin-pow/-sin/-cos/-sincos now keep libm's calls.)"""
import os

import numpy as np
import pytest

from helpers import O
from sq_divergence import divergence


# default: 8 192 envs x 600 steps (two whole episodes); FUTBOL_FULL_WORKLOAD=1: the C2 / C5 workload,
# 65 536 envs x 600 steps (scripts/v1_sq_divergence.py records that run in profiles/)
_FULL = os.environ.get("FUTBOL_FULL_WORKLOAD") == "1"


@pytest.mark.slow
@pytest.mark.parametrize("n", list(range(1, 11)))
def test_v1_faithful_vs_portable(n):
    """every team size (round 5; rounds 4: N = 2, 5): 8 192 envs x 600 steps for N <= 5, 2 048 for the
    larger teams (CPU time); the C2 / C5-sized run of every N, 65 536 x 600, is
    profiles/r05/v1_sq_divergence_all.json (scripts/v1_sq_divergence.py): 0 observation bits, 0
    discrete differences for each"""
    r = divergence(n, 65536 if _FULL else (8192 if n <= 5 else 2048), 600, seed=0)
    # the reward's x*x squares do show (some rewards differ in their last bits: the comparison sees
    # a difference at all), but no observation bit, no discrete outcome
    assert r["envs_any_bit_different"] > 0, r
    assert r["envs_obs_bit_different"] == 0 and r["max_abs_obs_diff"] == 0.0, r
    assert r["envs_any_discrete_diff"] == 0, r
    assert r["max_abs_reward_diff"] <= 1e-9, r


@pytest.mark.slow
def test_v1_xx_at_process_action_flips_an_outcome():
    """Why the state sites are exact: x*x in _process_action's get_vec alone (faithful build, per-site
    mask) reaches a discrete outcome on this sample (an owner flip and an out-of-bounds restart)."""
    r = divergence(5, 8192, 600, seed=0, b_mask=1)
    assert r["envs_any_discrete_diff"] >= 1, r


@pytest.mark.parametrize("random_opp", [False, True])
def test_v0_faithful_vs_portable(random_opp):
    """v0's only libm calls are screw_vec's math.sin / math.cos and get_vec's `**2`."""
    B = 1024
    a = O.V0Vec(B, seed=3, random_opp=random_opp, portable=False)
    b = O.V0Vec(B, seed=3, random_opp=random_opp, portable=True)
    assert np.array_equal(a.reset(), b.reset())
    rng = np.random.default_rng(2)
    for t in range(820):
        act = rng.integers(0, 16, B)
        oa, ra, da, _ = a.step(act, nthreads=4)
        ob, rb, db, _ = b.step(act, nthreads=4)
        assert np.array_equal(da, db), t
        assert np.array_equal(ra.view(np.uint64), rb.view(np.uint64)), t
        assert np.array_equal(oa.view(np.uint64), ob.view(np.uint64)), t
