"""The step kernels' division by a constant (`cdiv` in csrc/futbol_v1_impl.hpp: reciprocal multiply
+ one FMA correction) against the IEEE quotient x / c the reference computes, for every constant
divisor the kernels use with the default geometry -- obs normalisation (52.5, 55.5, 34, 25, 10),
the kick (2, 10), the contact bias (dt = 0.1 and the reset micro-step 1e-4) and the segments'
squared lengths (576, 11025, 400, 4) -- on random doubles and on quotients within a few ulps of
a rounding midpoint (oracle/cdiv_check.c; the GPU's fp64 FMA / multiply are the same IEEE ops)."""
import ctypes as C
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(os.path.dirname(HERE), "oracle", "_build", "liboracle.so")


@pytest.mark.parametrize("c", [52.5, 55.5, 34.0, 25.0, 10.0, 2.0, 0.1, 1e-4, 576.0, 11025.0, 400.0, 4.0])
def test_cdiv_equals_ieee_division(c):
    from oracle import oracle as O
    O.lib()  # builds oracle/_build on first use
    L = C.CDLL(LIB)
    L.orc_cdiv_check.argtypes = [C.c_double, C.c_longlong, C.c_uint64, C.c_int]
    L.orc_cdiv_check.restype = C.c_longlong
    assert L.orc_cdiv_check(c, 2_000_000, 12345, 40) == 0


def test_checker_detects_an_uncorrected_reciprocal():
    """Control: without the FMA correction, x * RN(1/c) differs from x / c on a sizeable fraction
    of inputs, and the same sampler sees it."""
    from oracle import oracle as O
    O.lib()
    L = C.CDLL(LIB)
    L.orc_mul_check.argtypes = [C.c_double, C.c_longlong, C.c_uint64, C.c_int]
    L.orc_mul_check.restype = C.c_longlong
    assert L.orc_mul_check(0.1, 100_000, 7, 40) > 1000
    assert L.orc_mul_check(55.5, 100_000, 7, 40) > 1000
