"""The v0 oracle pinned against the REFERENCE's own outputs.

tests/golden/v0_*.npz were produced by running gym_futbol/envs/futbol_env.py
(the reference) with its RNG calls replaced by the Philox tape
(tests/golden/gen_v0_golden.py).  The faithful oracle build must reproduce
every obs/reward/done bit-for-bit; the portable build (the kernels'
arithmetic) within 1e-9 with identical discrete outputs.
"""
import os

import numpy as np
import pytest

from helpers import O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ["v0_hardcoded_opp.npz", "v0_random_opp.npz"]


def _replay(g, portable):
    E, T = g["actions"].shape
    v = O.V0Vec(E, seed=int(g["seed"]), random_opp=bool(g["random_opp"]), portable=portable)
    yield 0, v.reset(), None, None, None
    for t in range(T):
        o, r, d, term = v.step(g["actions"][:, t])
        yield t, o, r, d, term


@pytest.mark.parametrize("fname", FIXTURES)
def test_faithful_oracle_bit_exact_vs_reference(fname):
    g = np.load(os.path.join(GOLDEN, fname))
    it = _replay(g, portable=False)
    _, o0, _, _, _ = next(it)
    assert np.array_equal(o0, g["obs0"])
    for t, o, r, d, term in it:
        assert np.array_equal(d, g["done"][:, t].astype(bool)), t
        assert np.array_equal(r, g["reward"][:, t]), t
        assert np.array_equal(o, g["obs"][:, t]), t
        if d.any():
            assert np.array_equal(term[d], g["terminal_obs"][:, t][d])


@pytest.mark.parametrize("fname", FIXTURES)
def test_portable_oracle_close_to_reference(fname):
    g = np.load(os.path.join(GOLDEN, fname))
    it = _replay(g, portable=True)
    next(it)
    for t, o, r, d, term in it:
        assert np.array_equal(d, g["done"][:, t].astype(bool)), t
        assert np.array_equal(o[:, 5], g["obs"][:, t, 5]), t  # owner row: discrete
        assert np.allclose(o, g["obs"][:, t], rtol=0, atol=1e-9), t
        assert np.allclose(r, g["reward"][:, t], rtol=0, atol=1e-9), t


@pytest.mark.parametrize("fname", FIXTURES)
def test_fixture_coverage(fname):
    """The golden rollouts exercise episode ends, goals both ways, shots and owner changes."""
    g = np.load(os.path.join(GOLDEN, fname))
    assert g["done"].sum() >= g["actions"].shape[0]
    assert (g["reward"] > 900).any() or (g["reward"] < -900).any()
    assert (g["obs"][:, :, 4, 4] >= 4).any()          # ball speed of a shot
    owners = g["obs"][:, :, 5].argmax(-1)
    assert len(np.unique(owners)) == 5
    assert (np.diff(np.nonzero(g["done"][0])[0]) == 401).all()  # K7: 401 steps per v0 episode


def test_v0_flags_and_tuple_actions_run():
    """one_goal_end / only_reward_goal / random_opp paths of the oracle (no reference fixture:
    the registered id uses the defaults)."""
    for kw in ({"one_goal_end": True}, {"only_reward_goal": True}, {"random_opp": True}):
        v = O.V0Vec(64, seed=1, **kw)
        v.reset()
        rng = np.random.default_rng(0)
        for _ in range(450):
            o, r, d, _ = v.step(rng.integers(0, 16, 64))
        if "only_reward_goal" in kw:
            assert set(np.unique(r)) <= {0.0, 1000.0, -1000.0}
