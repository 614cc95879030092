"""The gym-facing surface: registered ids, spaces, make(), loud failure without
a GPU (no CPU fallback)."""
import numpy as np
import pytest

import gym_futbol_amd as gf
from gym_futbol_amd import spaces as sp


def test_registered_ids_match_the_reference():
    # gym_futbol/__init__.py:3-28
    assert set(gf.ENV_SPECS) == {"Futbol-v0", "Futbol-extrahard-v0", "Futbol-v1", "Futbol2v2-v1", "Futbol5v5-v1"}
    assert gf.spec("Futbol-v1") == ("v1", {"number_of_player": 10})
    assert gf.spec("gym_futbol:Futbol2v2-v1") == ("v1", {"number_of_player": 2})
    assert gf.spec("Futbol5v5-v1") == ("v1", {"number_of_player": 5})
    assert gf.spec("Futbol-v0") == ("v0", {})
    with pytest.raises(AttributeError):
        gf.spec("Futbol-extrahard-v0")
    with pytest.raises(KeyError):
        gf.spec("Futbol3v3-v1")


@pytest.mark.parametrize("n,dim", [(2, 20), (5, 44), (10, 84)])
def test_v1_spaces(n, dim):
    a, o = sp.v1_action_space(n), sp.v1_observation_space(n)
    assert list(a.nvec) == [5, 5] * n and o.shape == (dim,) and o.dtype == np.float32
    assert (o.low == -1).all() and (o.high == 1).all()
    s = a.sample()
    assert s.shape == (2 * n,) and a.contains(s)


def test_v0_spaces():
    assert sp.v0_action_space(True).n == 16
    t = sp.v0_action_space(False)
    assert [s.n for s in t.spaces] == [4, 4] and t.contains(t.sample())
    o = sp.v0_observation_space()
    assert o.shape == (6, 5) and o.dtype == np.float64
    assert o.high[4, 4] == 20 and o.high[0, 4] == 12 and (o.high[5] == 10).all()


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    for env_id in ("Futbol2v2-v1", "Futbol-v0"):
        with pytest.raises(gf.NativeError):
            gf.make(env_id, num_envs=8)
        with pytest.raises(gf.NativeError):
            gf.make(env_id)
