"""Compact fingerprints for the large golden sets (tests/golden/v0_scale_*.npz): a 32-bit digest of
the exact bit patterns of each step's observation, so that 1 024 envs x 900 steps of reference
output fit in a few MB and the GPU / oracle tests can still demand bit-identical observations and
report the first step at which an env departs from the reference.  TEST INFRASTRUCTURE."""
import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def obs_digest(obs):
    """obs [..., k] float64 -> uint32 [...]: splitmix64 of every element's bits, position-weighted
    sum, folded to 32 bits.  Equal digests <=> equal bits (up to 2^-32 collisions)."""
    a = np.ascontiguousarray(obs, dtype=np.float64)
    x = a.view(np.uint64).copy()
    x ^= x >> np.uint64(30)
    x *= _M1
    x ^= x >> np.uint64(27)
    x *= _M2
    x ^= x >> np.uint64(31)
    w = (np.arange(a.shape[-1], dtype=np.uint64) * np.uint64(2) + np.uint64(1)) * _G
    h = (x * w).sum(axis=-1, dtype=np.uint64)
    return ((h ^ (h >> np.uint64(32))) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
