"""Generate v0 golden vectors by running THE REFERENCE itself (this container only).

    python tests/golden/gen_v0_golden.py          # writes tests/golden/v0_*.npz
    python tests/golden/gen_v0_golden.py --scale  # only the 1 024-env fingerprint sets (v0_scale_*.npz)

The reference (`/root/reference/gym_futbol/envs/futbol_env.py`, `easy_agent.py`)
is imported behind a throw-away `gym` stand-in written to a temp directory
outside the repo (gym 0.17.1 is not installed; only `gym.Env`, `gym.spaces`
and `gym.envs.registration.register` are touched by the v0 path).  Every
stochastic call of the reference -- `random.random/randint/uniform` and
`np.random.normal` -- is monkey-patched to read the RNG tape of
tests/rng_tape.py (Philox4x32-10) in program order;
`random.choice/choices/randrange/getrandbits` and the other numpy samplers are
made to raise, proving the tape captures all randomness.

Driven with VecEnv semantics: construct (event 0), reset() (event 1), then
step(a) with a = synthetic Philox action (tag 1) and reset() on done.
Only inputs/outputs are saved (actions, obs, reward, done): data, not source.
Skips itself when /root/reference is absent (e.g. on the GPU box).
"""
import os
import random
import sys
import tempfile
import textwrap

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from rng_tape import Tape, synthetic_action  # noqa: E402

REFERENCE = "/root/reference"

GYM_STUB = {
    "gym/__init__.py": """
        from . import spaces, error, utils
        class Env(object):
            pass
    """,
    "gym/error.py": "",
    "gym/utils/__init__.py": "from . import seeding\n",
    "gym/utils/seeding.py": "",
    "gym/spaces/__init__.py": """
        import numpy as np
        class Discrete(object):
            def __init__(self, n): self.n = n
        class Box(object):
            def __init__(self, low=None, high=None, shape=None, dtype=np.float32):
                self.low, self.high, self.dtype = low, high, dtype
        class Tuple(object):
            def __init__(self, spaces): self.spaces = spaces
        class MultiDiscrete(object):
            def __init__(self, nvec): self.nvec = np.asarray(nvec)
    """,
    "gym/envs/__init__.py": "",
    "gym/envs/registration.py": """
        def register(**kw):
            pass
    """,
}


class TapeDriver:
    def __init__(self, seed):
        self.seed = seed
        self.tape = None
        self.draws = 0

    def begin(self, env_id, event):
        self.tape = Tape(self.seed, env_id, event, tag=0)

    # patched functions ------------------------------------------------------
    def random(self):
        self.draws += 1
        return self.tape.random()

    def randint(self, a, b):
        self.draws += 1
        return self.tape.randint(a, b)

    def uniform(self, a, b):
        self.draws += 1
        return self.tape.uniform(a, b)

    def normal(self, loc=0.0, scale=1.0, size=None):
        self.draws += 1
        v = self.tape.normal(loc, scale)
        return v if size is None else np.full(size, v)


def _forbidden(name):
    def f(*a, **k):
        raise RuntimeError("reference called un-taped RNG function %s" % name)
    return f


def install_stub():
    d = tempfile.mkdtemp(prefix="gymstub_")
    for rel, body in GYM_STUB.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(textwrap.dedent(body))
    return d


def run(random_opp, n_envs, n_steps, seed, act_seed, env0=0):
    import gym_futbol.envs.futbol_env as fe  # noqa: the reference

    drv = TapeDriver(seed)
    random.random, random.randint, random.uniform = drv.random, drv.randint, drv.uniform
    for name in ("choice", "choices", "randrange", "getrandbits", "shuffle", "sample", "gauss"):
        setattr(random, name, _forbidden(name))
    np.random.normal = drv.normal
    for name in ("rand", "randn", "randint", "random", "random_sample", "uniform", "choice"):
        setattr(np.random, name, _forbidden("np.random." + name))

    acts = np.zeros((n_envs, n_steps), np.int32)
    obs = np.zeros((n_envs, n_steps, 6, 5), np.float64)
    term = np.zeros((n_envs, n_steps, 6, 5), np.float64)
    rew = np.zeros((n_envs, n_steps), np.float64)
    done = np.zeros((n_envs, n_steps), np.uint8)
    ndraw = np.zeros((n_envs, n_steps), np.int32)
    obs0 = np.zeros((n_envs, 6, 5), np.float64)
    for ei in range(n_envs):
        e = env0 + ei
        event = 0
        drv.begin(e, event); event += 1
        env = fe.FutbolEnv(random_opp=random_opp)
        drv.begin(e, event); event += 1
        obs0[ei] = env.reset()
        for t in range(n_steps):
            a = synthetic_action(act_seed, e, t, 0, 16)
            acts[ei, t] = a
            drv.begin(e, event); event += 1
            d0 = drv.draws
            o, r, d, _ = env.step(a)
            ndraw[ei, t] = drv.draws - d0
            obs[ei, t] = o
            rew[ei, t] = r
            done[ei, t] = d
            if d:
                term[ei, t] = o
                drv.begin(e, event); event += 1
                obs[ei, t] = env.reset()
    return dict(actions=acts, obs=obs, terminal_obs=term, reward=rew, done=done, draws=ndraw, obs0=obs0,
                seed=np.uint64(seed), act_seed=np.uint64(act_seed), random_opp=np.int32(random_opp))


def _run_chunk(args):
    """worker: envs [e0, e1) of one scale case (env ids are global: the tape is keyed by them)"""
    ro, e0, e1, T, seed, aseed = args
    stub = install_stub()
    sys.path[:0] = [stub, REFERENCE]
    import warnings
    warnings.simplefilter("ignore", DeprecationWarning)
    from golden_digest import obs_digest
    out = run(ro, e1 - e0, T, seed, aseed, env0=e0)
    return dict(reward=out["reward"], done=out["done"], draws=out["draws"].astype(np.uint8),
                obs_digest=obs_digest(out["obs"].reshape(e1 - e0, T, 30)),
                term_digest=np.where(out["done"] != 0, obs_digest(out["terminal_obs"].reshape(e1 - e0, T, 30)), 0)
                .astype(np.uint32),
                owner=np.argmax(out["obs"][:, :, 5, :], axis=-1).astype(np.uint8),
                obs0=out["obs0"])


def run_scale(ro, E, T, seed, aseed, workers):
    """E envs x T steps of the reference, as compact fingerprints (tests/golden_digest.py): exact
    rewards, dones, RNG draws per step, the ball owner and 32-bit digests of every observation."""
    from multiprocessing import Pool
    step = (E + workers - 1) // workers
    chunks = [(ro, e0, min(E, e0 + step), T, seed, aseed) for e0 in range(0, E, step)]
    with Pool(len(chunks)) as pool:
        parts = pool.map(_run_chunk, chunks)
    out = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    out.update(seed=np.uint64(seed), act_seed=np.uint64(aseed), random_opp=np.int32(ro))
    return out


SCALE_CASES = [("v0_scale_hardcoded_opp.npz", False, 1024, 900, 20240601, 1234),
               ("v0_scale_random_opp.npz", True, 1024, 900, 777, 99)]


def main():
    if not os.path.isdir(os.path.join(REFERENCE, "gym_futbol")):
        print("reference absent; skipping golden generation")
        return
    stub = install_stub()
    sys.path[:0] = [stub, REFERENCE]
    import warnings
    warnings.simplefilter("ignore", DeprecationWarning)  # randint(32.0, 36.0) on py3.10
    if "--scale" not in sys.argv:
        cases = [("v0_hardcoded_opp.npz", False, 6, 900, 20240601, 1234),
                 ("v0_random_opp.npz", True, 4, 500, 777, 99)]
        for fname, ro, E, T, seed, aseed in cases:
            out = run(ro, E, T, seed, aseed)
            np.savez_compressed(os.path.join(HERE, fname), **out)
            print(fname, "episodes done:", int(out["done"].sum()), "goals:",
                  int((np.abs(out["reward"]) >= 900).sum()), "draws/step mean:", float(out["draws"].mean()))
    if "--small" not in sys.argv:
        workers = min(8, os.cpu_count() or 1)
        for fname, ro, E, T, seed, aseed in SCALE_CASES:
            out = run_scale(ro, E, T, seed, aseed, workers)
            np.savez_compressed(os.path.join(HERE, fname), **out)
            print(fname, "envs", E, "steps", T, "episodes done:", int(out["done"].sum()), "goals:",
                  int((np.abs(out["reward"]) >= 900).sum()))


if __name__ == "__main__":
    main()
