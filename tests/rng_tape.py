"""Pure-Python restatement of the RNG-tape contract.

TEST INFRASTRUCTURE.  Written independently of oracle/oracle_rng.h and of the
kernel's csrc/futbol_rng.hpp; all three are checked against Random123's
Philox4x32-10 known-answer vectors (tests/test_rng.py).

draw(seed, env_id, event, j, tag) -> 4 x u32 = Philox4x32-10(
    counter=(j, event, env_id, tag), key=(seed & 0xffffffff, seed >> 32))
"""
import math

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
        z = math.sqrt(-2.0 * math.log(1.0 - u1)) * math.cos(6.283185307179586 * u2)
        return mu + sigma * z


def synthetic_action(seed, env_id, step, j, n):
    """Synthetic 'left agent' action stream (tag 1): floor(U * n)."""
    t = Tape(seed, env_id, step, tag=1)
    t.j = j
    return t.choice_index(n)
