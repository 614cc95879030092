"""Test helpers: state conversion between the oracle (oracle/, Chipmunk-style
dense arbiter table) and the kernels' SoA state (csrc/futbol_state.hpp).
TEST INFRASTRUCTURE."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gym-futbol_amd"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import oracle as O  # noqa: E402

NSEG = 12


def npairs(n):
    nb = 2 * n + 1
    return nb * NSEG + nb * (nb - 1) // 2


def time_to_steps(t):
    k, acc = 0, 0.0
    while acc != t:
        acc += 0.1
        k += 1
        if k > 20000:
            raise ValueError("time %r is not a multiple-of-0.1 accumulation" % t)
    return k


def dtcode(dt):
    return {0.0: 0, 0.0001: 1, 0.1: 2}[dt]


def v1_oracle_to_state(envs, n, B):
    """OrcV1[B] -> kernel state dict (ep_ret / stats zero)."""
    nb, P = 2 * n + 1, npairs(n)
    st = {k: np.zeros(nb * B) for k in ("px", "py", "vx", "vy", "bx", "by")}
    st["meta"] = np.zeros(B, np.uint64)
    st["ep_ret"] = np.zeros(B)
    st["ckey"] = np.zeros(P * B, np.uint16)
    st["cjn"] = np.zeros(P * B)
    st["stat_ret"] = np.zeros(B)
    st["stat_cnt"] = np.zeros(B, np.uint32)
    for i in range(B):
        e = envs[i]
        for k in range(nb):
            for f in ("px", "py", "vx", "vy", "bx", "by"):
                st[f][k * B + i] = getattr(e, f)[k]
        c = 0
        for p in range(P):
            if e.arb_exists[p]:
                age = e.stamp - e.arb_stamp[p]
                assert 0 <= age <= 2
                st["ckey"][c * B + i] = p | (age << 12)
                st["cjn"][c * B + i] = e.arb_jn[p]
                c += 1
        meta = (e.owner & 7) | (dtcode(e.curr_dt) << 6) | (c << 8) | (time_to_steps(e.current_time) << 18) \
            | (int(e.event) << 32)
        st["meta"][i] = np.uint64(meta)
    return st


def v1_state_to_oracle(st, envs, n, B):
    """kernel state -> OrcV1[B] (in place; config fields must already be set)."""
    nb, P = 2 * n + 1, npairs(n)
    for i in range(B):
        e = envs[i]
        for k in range(nb):
            for f in ("px", "py", "vx", "vy", "bx", "by"):
                getattr(e, f)[k] = st[f][k * B + i]
        m = int(st["meta"][i])
        e.owner = m & 7
        e.curr_dt = [0.0, 0.0001, 0.1][(m >> 6) & 3]
        steps = (m >> 18) & 0x3FFF
        t = 0.0
        for _ in range(steps):
            t += 0.1
        e.current_time = t
        e.event = m >> 32
        e.stamp = 1000
        for p in range(P):
            e.arb_exists[p] = 0
            e.arb_inlist[p] = 0
        for c in range((m >> 8) & 0x3FF):
            key = int(st["ckey"][c * B + i])
            p, age = key & 0x3FF, key >> 12
            e.arb_exists[p] = 1
            e.arb_stamp[p] = e.stamp - age
            e.arb_state[p] = 1 if age == 0 else 2  # NORMAL / CACHED
            e.arb_inlist[p] = 1 if age == 0 else 0
            e.arb_jn[p] = st["cjn"][c * B + i]


def v1_dense_cache(st, n, B):
    """kernel state -> (exists[B,P], age[B,P], jn[B,P])"""
    P = npairs(n)
    ex = np.zeros((B, P), bool)
    age = np.zeros((B, P), np.int64)
    jn = np.zeros((B, P))
    nc = (st["meta"].astype(np.uint64) >> np.uint64(8)) & np.uint64(0x3FF)
    for i in range(B):
        for c in range(int(nc[i])):
            key = int(st["ckey"][c * B + i])
            p = key & 0x3FF
            ex[i, p] = True
            age[i, p] = key >> 12
            jn[i, p] = st["cjn"][c * B + i]
    return ex, age, jn


def v1_oracle_dense_cache(envs, n, B):
    P = npairs(n)
    ex = np.zeros((B, P), bool)
    age = np.zeros((B, P), np.int64)
    jn = np.zeros((B, P))
    for i in range(B):
        e = envs[i]
        for p in range(P):
            if e.arb_exists[p]:
                ex[i, p] = True
                age[i, p] = e.stamp - e.arb_stamp[p]
                jn[i, p] = e.arb_jn[p]
    return ex, age, jn


def v1_oracle_bodies(envs, n, B):
    nb = 2 * n + 1
    out = {}
    for f in ("px", "py", "vx", "vy", "bx", "by"):
        a = np.zeros((nb, B))
        for i in range(B):
            a[:, i] = np.frombuffer(getattr(envs[i], f), dtype=np.float64)[:nb]
        out[f] = a.reshape(-1)
    return out


def v0_oracle_views(envs, B):
    """oracle -> kernel 'view' field [8][B] (frozen Easy_Agent views)."""
    v = np.zeros((8, B))
    for i in range(B):
        e = envs[i]
        for a in range(2):
            v[2 * a, i], v[2 * a + 1, i] = e.ai_view[a][0], e.ai_view[a][1]
        for a in range(2):
            v[2 * (a + 2), i], v[2 * (a + 2) + 1, i] = e.opp_view_frozen[a][0], e.opp_view_frozen[a][1]
    return v
