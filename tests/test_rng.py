"""The RNG-tape contract: Philox4x32-10 known-answer
vectors (Random123's kat_vectors) for the Python tape and both oracle builds,
and identical draw conversions between the Python tape and the C oracle."""
import ctypes as C

import numpy as np
import pytest

from helpers import O
from rng_tape import Tape, philox4x32_10

KAT = [  # (counter, key, expected) -- Random123 kat_vectors, philox4x32_10
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,exp", KAT)
def test_philox_kat_python(ctr, key, exp):
    assert philox4x32_10(ctr, key) == exp


@pytest.mark.parametrize("portable", [False, True])
@pytest.mark.parametrize("ctr,key,exp", KAT)
def test_philox_kat_oracle(ctr, key, exp, portable):
    assert O.philox(ctr, key, portable) == exp


@pytest.mark.parametrize("portable", [False, True])
def test_draws_python_vs_oracle(portable):
    L = O.lib(portable)
    rng = np.random.default_rng(0)
    for _ in range(300):
        seed, env, ev, j = (int(rng.integers(0, 2**63)), int(rng.integers(0, 2**32)),
                            int(rng.integers(0, 2**32)), int(rng.integers(0, 64)))
        t = Tape(seed, env, ev)
        t.j = j
        u = t.random()
        t.j = j
        z = t.normal(0.0, 1.0)
        uc, zc = C.c_double(), C.c_double()
        L.orc_draw_u01(seed, env, ev, j, 0, C.byref(uc), C.byref(zc))
        assert u == uc.value and 0.0 <= u < 1.0
        assert z == zc.value   # the normal draw is specified with +,-,*,/-only log/cos


def test_conversions_are_unbiased_enough():
    t = Tape(7, 3, 11)
    k = np.array([t.choice_index(5) for _ in range(20000)])
    assert set(k) == {0, 1, 2, 3, 4}
    assert np.all(np.abs(np.bincount(k) / len(k) - 0.2) < 0.02)
    assert all(32 <= Tape(1, i, 0).randint(32.0, 36.0) <= 36 for i in range(200))


def test_tape_functions_are_accurate():
    """pm_log / pm_cos define the normal draw; they stay within a few ulp of libm."""
    import math
    from rng_tape import pm_cos, pm_log
    rng = np.random.default_rng(5)
    for x in rng.random(20000):
        assert abs(pm_log(1.0 - x) - math.log(1.0 - x)) <= 4e-16 * max(1.0, abs(math.log(1.0 - x)))
        a = 6.283185307179586 * x
        assert abs(pm_cos(a) - math.cos(a)) <= 4e-16
