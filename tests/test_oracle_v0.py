"""The v0 oracle pinned against the REFERENCE's own outputs.

tests/golden/v0_*.npz were produced by running gym_futbol/envs/futbol_env.py
(the reference) with its RNG calls replaced by the Philox tape
(tests/golden/gen_v0_golden.py): 6 + 4 envs with every observation, and
1 024 envs x 900 steps per opponent mode as fingerprints (exact rewards, dones,
ball owner and 32-bit digests of every observation, tests/golden_digest.py).
Both oracle builds -- faithful (libm) and portable (the kernels' arithmetic:
the glibc sin / cos / pow(x, 2) restatements) -- must reproduce every output
bit for bit; the scale test reports each env's first divergent step.
"""
import os

import numpy as np
import pytest

from golden_digest import obs_digest
from helpers import O
from rng_tape import synthetic_actions_vec

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ["v0_hardcoded_opp.npz", "v0_random_opp.npz"]


def load_golden(fname):
    """all arrays decompressed once (an NpzFile decompresses a member on every access)"""
    with np.load(os.path.join(GOLDEN, fname)) as z:
        return {k: z[k] for k in z.files}


def _replay(g, portable):
    E, T = g["actions"].shape
    v = O.V0Vec(E, seed=int(g["seed"]), random_opp=bool(g["random_opp"]), portable=portable)
    yield 0, v.reset(), None, None, None
    for t in range(T):
        o, r, d, term = v.step(g["actions"][:, t])
        yield t, o, r, d, term


@pytest.mark.parametrize("fname", FIXTURES)
def test_faithful_oracle_bit_exact_vs_reference(fname):
    g = load_golden(fname)
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
def test_portable_oracle_bit_exact_vs_reference(fname):
    g = load_golden(fname)
    it = _replay(g, portable=True)
    next(it)
    for t, o, r, d, term in it:
        assert np.array_equal(d, g["done"][:, t].astype(bool)), t
        assert np.array_equal(r.view(np.uint64), g["reward"][:, t].view(np.uint64)), t
        assert np.array_equal(o.view(np.uint64), g["obs"][:, t].view(np.uint64)), t


SCALE = ["v0_scale_hardcoded_opp.npz", "v0_scale_random_opp.npz"]


def first_divergence(g, step_fn):
    """Replays a scale fingerprint set through step_fn(actions [E]) -> (obs [E,6,5], reward, done,
    terminal_obs); returns each env's first step whose outputs are not bit-identical (-1: none)."""
    E, T = g["reward"].shape
    first = np.full(E, -1)
    envs = np.arange(E)
    for t in range(T):
        a = synthetic_actions_vec(int(g["act_seed"]), envs, t, 0, 16)
        o, r, d, term = step_fn(a)
        bad = (obs_digest(o.reshape(E, 30)) != g["obs_digest"][:, t])
        bad |= r.view(np.uint64) != g["reward"][:, t].view(np.uint64)
        bad |= d != g["done"][:, t].astype(bool)
        bad |= np.argmax(o[:, 5], axis=-1) != g["owner"][:, t]
        if d.any():
            bad |= d & (obs_digest(term.reshape(E, 30)) != g["term_digest"][:, t])
        first[(first < 0) & bad] = t
    return first


def report(first, tag):
    div = np.nonzero(first >= 0)[0]
    return "%s: %d of %d envs diverge from the reference; (env, first step): %s" % (
        tag, len(div), len(first), list(zip(div[:20].tolist(), first[div[:20]].tolist())))


@pytest.mark.parametrize("portable", [False, True])
@pytest.mark.parametrize("fname", SCALE)
def test_oracle_vs_reference_at_scale(fname, portable):
    """1 024 envs x 900 steps (two whole 401-step episodes and more) of the reference, per mode."""
    g = load_golden(fname)
    E = g["reward"].shape[0]
    v = O.V0Vec(E, seed=int(g["seed"]), random_opp=bool(g["random_opp"]), portable=portable)
    assert np.array_equal(v.reset(), g["obs0"])
    first = first_divergence(g, lambda a: v.step(a.astype(np.int32), nthreads=4))
    assert (first < 0).all(), report(first, fname)


@pytest.mark.parametrize("fname", SCALE)
def test_scale_fixture_coverage(fname):
    g = load_golden(fname)
    E, T = g["reward"].shape
    assert E >= 1024 and T >= 900
    assert g["done"].sum() == E * (T // 401)
    assert (g["reward"] > 900).sum() > 100 and (g["reward"] < -900).sum() > 100
    assert len(np.unique(g["owner"])) == 5


@pytest.mark.parametrize("fname", FIXTURES)
def test_fixture_coverage(fname):
    """The golden rollouts exercise episode ends, goals both ways, shots and owner changes."""
    g = load_golden(fname)
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
