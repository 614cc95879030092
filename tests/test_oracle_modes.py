"""Faithful (libm pow / sin / cos, = CPython) vs portable (x*x squares and the glibc sin/cos
restatement, = the kernels) oracle builds.  The two differ only in where the libm results come
from; tests/test_glibc_sincos.py pins the restatement against the host libm, so the builds must
agree BIT FOR BIT on whole rollouts -- which makes the kernels' bit-exact parity with the portable
build a bit-exact parity with the reference's own arithmetic.

(Before round 3 the portable build used correctly rounded sin/cos, and the faithful build's
sin(x), cos(x) pair was fused by gcc into glibc's sincos(); 1 env in ~4 000 diverged discretely.)"""
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
        assert np.array_equal(ra.view(np.uint64), rb.view(np.uint64))
        assert np.array_equal(oa.view(np.uint64), ob.view(np.uint64))


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
