"""Every compiled envs_v1 step-kernel instance against the oracle, on the GPU.

Each team size N = 1..10 is compiled into 8 step instances (csrc/futbol_v1_inst.hpp): output type
(f64 / f32) x field geometry (the default field with its constants as immediates, or the runtime
geometry of custom width / height, forced here with FUTBOL_GENERIC=1) x launch (one step per launch,
or the open-loop rollout of K steps per launch).  The instances compile the same source, but the
large ones run at the 512-register limit with spills, where code generation has failed before
("compiler": a wrong double-output instance while the float one of the same
source was right).  So every instance is run here: 96 envs (a full and a ragged block of 64) x 310
steps from reset -- through the 300-step episode end, the auto-reset and its terminal observation --
obs / reward / done / terminal obs bit for bit against the portable oracle (f32 outputs: the f32
cast of the oracle's f64 values).  (Round 3 ran 64 envs x 60 steps, which never reached an episode
end.)
"""
import numpy as np
import pytest
import torch

from helpers import O

pytestmark = pytest.mark.gpu

B, T = 96, 310


def _run(n, seed, acts, dtype, generic, rollout, monkeypatch):
    from gym_futbol_amd import FutbolVecEnv
    monkeypatch.setenv("FUTBOL_GENERIC", "1" if generic else "0")
    venv = FutbolVecEnv("v1", B, seed=seed, dtype=dtype, number_of_player=n)
    o0 = venv.reset().cpu().numpy()
    if rollout:
        obs, rew, done, term = venv.rollout(acts)
    else:  # outputs gathered on the device, one copy at the end
        obs = torch.empty((T, B) + tuple(venv._obs.shape[1:]), dtype=dtype, device=venv.device)
        rew = torch.empty((T, B), dtype=dtype, device=venv.device)
        done = torch.empty((T, B), dtype=torch.uint8, device=venv.device)
        term = torch.zeros_like(obs)
        for t in range(T):
            o, r, d, info = venv.step(acts[t])
            obs[t] = o
            rew[t] = r
            done[t] = d.to(torch.uint8)
            term[t] = info["terminal_observation"]
    out = (obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy().astype(bool), term.cpu().numpy())
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
    ro, rr, rd, rt = [], [], [], []
    for t in range(T):
        o, r, d, term = ora.step(a_np[t])
        ro.append(o)
        rr.append(r)
        rd.append(np.asarray(d, bool))
        rt.append(term)
    ref = (np.stack(ro), np.stack(rr), np.stack(rd), np.stack(rt))
    assert ref[2].shape == (T, B) and ref[2].sum() == B  # every env ends its episode once
    failures = []
    for dtype in (torch.float64, torch.float32):
        npdt = np.float64 if dtype == torch.float64 else np.float32
        want = (ref[0].astype(npdt), ref[1].astype(npdt), ref[2], ref[3].astype(npdt))
        for generic in (False, True):
            for rollout in (False, True):
                tag = "N=%d %s %s %s" % (n, "f64" if dtype == torch.float64 else "f32",
                                         "generic" if generic else "default-field", "rollout" if rollout else "step")
                o0, got = _run(n, seed, acts, dtype, generic, rollout, monkeypatch)
                assert np.array_equal(o0.view(np.uint8), ref0.astype(npdt).view(np.uint8)), tag + ": reset obs"
                for what, g, w in zip(("obs", "reward", "done", "terminal obs"), got, want):
                    g = np.asarray(g).reshape(w.shape)
                    if what == "terminal obs":  # valid in the done rows only
                        g, w = g[ref[2]], w[ref[2]]
                    if what == "done":
                        diff = g != w
                    else:  # bitwise, including the sign of zero
                        diff = (g.view(np.uint8).reshape(g.shape + (-1,)) != w.view(np.uint8).reshape(w.shape + (-1,))).any(-1)
                    if diff.any():
                        where = np.argwhere(diff)
                        failures.append("%s: %s differs, first at %s (%d entries)" % (tag, what, where[0].tolist(), len(where)))
                        break
    assert not failures, "; ".join(failures)
