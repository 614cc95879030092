"""Faithful (libm pow / sin / cos, = CPython) vs portable (= the kernels) oracle builds.

v0: the portable build computes the reference's `x**2` and math.sin / math.cos with the glibc
restatements (tests/test_glibc_sincos.py pins them against the host libm), so the two builds must
agree BIT FOR BIT on whole rollouts -- the kernels' bit-exact parity with the portable build is a
bit-exact parity with the reference's own arithmetic (and tests/test_oracle_v0.py checks it against
1 024-env reference fingerprints).

envs_v1: the kernels square with x*x where the reference's Python code writes `**2` (libm pow,
which differs from x*x on ~0.08% of arguments): a deliberate difference,
bounded here -- identical discrete outcomes, positions / velocities within the north star's 1e-5.

(Before round 3 the faithful build was not faithful: gcc turned pow(x, 2.0) into x*x and fused
sin(x), cos(x) into glibc's sincos(); -fno-builtin-pow/-sin/-cos/-sincos now keep libm's calls.)"""
import numpy as np
import pytest

from helpers import O


@pytest.mark.parametrize("n", [2, 5])
def test_v1_faithful_vs_portable(n):
    B = 256
    a = O.V1Vec(B, N=n, seed=5, portable=False)
    b = O.V1Vec(B, N=n, seed=5, portable=True)
    assert np.array_equal(a.reset(), b.reset())
    rng = np.random.default_rng(1)
    for t in range(320):
        act = rng.integers(0, 5, (B, 2 * n))
        oa, ra, da, _ = a.step(act)
        ob, rb, db, _ = b.step(act)
        assert np.array_equal(da, db)
        assert np.array_equal(np.abs(ra) > 500, np.abs(rb) > 500)  # goals identical
        assert np.abs(oa - ob).max() <= 1e-5 and np.abs(ra - rb).max() <= 1e-6


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
