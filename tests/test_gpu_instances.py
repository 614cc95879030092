"""Every compiled envs_v1 step-kernel instance against the oracle, on the GPU.

Each team size N = 1..10 is compiled into 8 step instances (csrc/futbol_v1_inst.hpp): output type
(f64 / f32) x field geometry (the default field with its constants as immediates, or the runtime
geometry of custom width / height, forced here with FUTBOL_GENERIC=1) x launch (one step per launch,
or the open-loop rollout of K steps per launch).  The instances compile the same source, but the
large ones run at the 512-register limit with spills, where code generation has failed before
("compiler": a wrong double-output instance while the float one of the same
source was right).  So every instance is run here: 64 envs x 60 steps from reset, obs / reward /
done bit for bit against the portable oracle (f32 outputs: the f32 cast of the oracle's f64 values).
"""
import numpy as np
import pytest
import torch

from helpers import O

pytestmark = pytest.mark.gpu

B, T = 64, 60


def _run(n, seed, acts, dtype, generic, rollout, monkeypatch):
    from gym_futbol_amd import FutbolVecEnv
    monkeypatch.setenv("FUTBOL_GENERIC", "1" if generic else "0")
    venv = FutbolVecEnv("v1", B, seed=seed, dtype=dtype, number_of_player=n)
    o0 = venv.reset().cpu().numpy()
    if rollout:
        obs, rew, done, _ = venv.rollout(acts)
        out = (obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool))
    else:
        os_, rs, ds = [], [], []
        for t in range(T):
            o, r, d, _ = venv.step(acts[t])
            os_.append(o.cpu().numpy())
            rs.append(r.cpu().numpy())
            ds.append(d.cpu().numpy().astype(bool))
        out = (np.stack(os_), np.stack(rs), np.stack(ds))
    venv.close()
    return o0, out


@pytest.mark.parametrize("n", list(range(1, 11)))
def test_every_step_instance(n, monkeypatch):
    seed = 31 + n
    from gym_futbol_amd import FutbolVecEnv
    gen = FutbolVecEnv("v1", B, seed=seed, number_of_player=n)
    acts = gen.random_actions_steps(T, 0, seed=5)
    gen.close()
    a_np = acts.cpu().numpy().astype(np.int32)
    ora = O.V1Vec(B, N=n, seed=seed, portable=True)
    ref0 = ora.reset()
    ro, rr, rd = [], [], []
    for t in range(T):
        o, r, d, _ = ora.step(a_np[t])
        ro.append(o)
        rr.append(r)
        rd.append(np.asarray(d, bool))
    ref = (np.stack(ro), np.stack(rr), np.stack(rd))
    assert ref[2].shape == (T, B)
    failures = []
    for dtype in (torch.float64, torch.float32):
        npdt = np.float64 if dtype == torch.float64 else np.float32
        want = (ref[0].astype(npdt), ref[1].astype(npdt), ref[2])
        for generic in (False, True):
            for rollout in (False, True):
                tag = "N=%d %s %s %s" % (n, "f64" if dtype == torch.float64 else "f32",
                                         "generic" if generic else "default-field", "rollout" if rollout else "step")
                o0, got = _run(n, seed, acts, dtype, generic, rollout, monkeypatch)
                assert np.array_equal(o0.view(np.uint8), ref0.astype(npdt).view(np.uint8)), tag + ": reset obs"
                for what, g, w in zip(("obs", "reward", "done"), got, want):
                    g = np.asarray(g).reshape(w.shape)
                    if what == "done":
                        diff = g != w
                    else:  # bitwise, including the sign of zero
                        diff = (g.view(np.uint8).reshape(g.shape + (-1,)) != w.view(np.uint8).reshape(w.shape + (-1,))).any(-1)
                    if diff.any():
                        where = np.argwhere(diff)
                        failures.append("%s: %s differs, first at %s (%d entries)" % (tag, what, where[0].tolist(), len(where)))
                        break
    assert not failures, "; ".join(failures)
