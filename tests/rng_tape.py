"""Pure-Python restatement of the RNG-tape contract.

TEST INFRASTRUCTURE.  Written independently of oracle/oracle_rng.h and of the
kernel's csrc/futbol_rng.hpp; all three are checked against Random123's
Philox4x32-10 known-answer vectors (tests/test_rng.py).

draw(seed, env_id, event, j, tag) -> 4 x u32 = Philox4x32-10(
    counter=(j, event, env_id, tag), key=(seed & 0xffffffff, seed >> 32))
"""
import math
import struct

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
    return c0, c1, c2, c3


def u53(a, b):
    return ((a >> 5) * 67108864.0 + (b >> 6)) * (1.0 / 9007199254740992.0)


def pm_log(x):
    """The tape's log (x > 0): atanh series on m in [sqrt(1/2), sqrt(2)), + - * / only.
    Python floats are IEEE doubles with correctly rounded + - * /, so this is the
    same double as oracle_math.h:orc_pm_log and csrc/futbol_math.hpp:pm_log."""
    bits = struct.unpack("<Q", struct.pack("<d", x))[0]
    e = ((bits >> 52) & 0x7FF) - 1023
    m = struct.unpack("<d", struct.pack("<Q", (bits & 0x000FFFFFFFFFFFFF) | 0x3FF0000000000000))[0]
    if m > 1.4142135623730951:
        m = m * 0.5
        e = e + 1
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    p = 1.0 / 25.0
    for d in (23.0, 21.0, 19.0, 17.0, 15.0, 13.0, 11.0, 9.0, 7.0, 5.0, 3.0):
        p = p * s2 + 1.0 / d
    lm = 2.0 * s + 2.0 * s * (s2 * p)
    de = float(e)
    return (de * 6.93147180369123816490e-01 + lm) + de * 1.90821492927058770002e-10


_SIN_F = (355687428096000.0, 1307674368000.0, 6227020800.0, 39916800.0, 362880.0, 5040.0, 120.0, 6.0)
_COS_F = (6402373705728000.0, 20922789888000.0, 87178291200.0, 479001600.0, 3628800.0, 40320.0, 720.0,
          24.0, 2.0)


def pm_cos(a):
    """The tape's cos: three-part pi/2 reduction, Taylor to r^18 (+ - * / only)."""
    kq = math.floor(a * 6.36619772367581382433e-01 + 0.5)
    kq = float(kq)
    r = ((a - kq * 1.57079632673412561417e+00) - kq * 6.07710050630396597660e-11) - kq * 2.02226624879595063154e-21
    r2 = r * r
    s = -1.0 / _SIN_F[0]
    for i, f in enumerate(_SIN_F[1:]):
        s = s * r2 + (1.0 / f if i % 2 == 0 else -1.0 / f)
    sr = r - r * (r2 * s)
    c = 1.0 / _COS_F[0]
    for i, f in enumerate(_COS_F[1:-1]):
        c = c * r2 + (-1.0 / f if i % 2 == 0 else 1.0 / f)
    c = c * r2 + 0.5
    cr = 1.0 - r2 * c
    return (cr, -sr, -cr, sr)[int(kq) & 3]


class Tape:
    """Program-order draws for one (seed, env_id, event)."""

    def __init__(self, seed, env_id, event, tag=0):
        self.seed, self.env_id, self.event, self.tag = seed, env_id, event, tag
        self.j = 0

    def block(self):
        out = philox4x32_10((self.j & MASK, self.event & MASK, self.env_id & MASK, self.tag),
                            (self.seed & MASK, (self.seed >> 32) & MASK))
        self.j += 1
        return out

    def random(self):
        x = self.block()
        return u53(x[0], x[1])

    def choice_index(self, n):
        k = int(math.floor(self.random() * n))
        return min(k, n - 1)

    def randint(self, a, b):
        a, b = int(a), int(b)
        return a + self.choice_index(b - a + 1)

    def uniform(self, a, b):
        u = self.random()
        return a + (b - a) * u

    def normal(self, mu, sigma):
        x = self.block()
        u1, u2 = u53(x[0], x[1]), u53(x[2], x[3])
        z = math.sqrt(-2.0 * pm_log(1.0 - u1)) * pm_cos(6.283185307179586 * u2)
        return mu + sigma * z


def synthetic_action(seed, env_id, step, j, n):
    """Synthetic 'left agent' (benchmark policy) action j of an env-step (tag 1): four actions
    per Philox block, action j = (w * n) >> 32 with w = word j % 4 of block j // 4."""
    x = philox4x32_10((j // 4, step & MASK, env_id & MASK, 1), (seed & MASK, (seed >> 32) & MASK))
    return (x[j % 4] * n) >> 32


def synthetic_actions_vec(seed, env_ids, step, j, n):
    """synthetic_action for an array of env ids at once (numpy, same Philox4x32-10 arithmetic)."""
    import numpy as np
    env_ids = np.asarray(env_ids, dtype=np.uint64)
    m = np.uint64(MASK)
    c0 = np.full(env_ids.shape, j // 4, np.uint64)
    c1 = np.full(env_ids.shape, step & MASK, np.uint64)
    c2 = env_ids & m
    c3 = np.full(env_ids.shape, 1, np.uint64)
    k0, k1 = seed & MASK, (seed >> 32) & MASK
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = np.uint64(M0) * c0
        p1 = np.uint64(M1) * c2
        c0, c1, c2, c3 = (((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)) & m, p1 & m,
                          ((p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)) & m, p0 & m)
    w = (c0, c1, c2, c3)[j % 4]
    return ((w * np.uint64(n)) >> np.uint64(32)).astype(np.int64)
