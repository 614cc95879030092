"""The N > 1 layout on CPU (gloo, world_size 2): env shards keyed by global env
id reproduce a single process running every env, episode statistics reduce
with one all_reduce, and the timed region is the max over ranks.  The env
physics here is the CPU oracle (test infrastructure) standing in for the
per-rank GPU step; the sharding / collective code is the product's
(gym_futbol_amd/distributed.py, used by bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from helpers import O

B_PER_RANK, WORLD = 24, 2
STEPS = {"v1": 330, "v0": 420}   # past one episode (300 / 401 steps)


def _actions(kind, gids, t, adim):
    nv = 5 if kind == "v1" else 16
    return ((gids[:, None] * 7 + t * 3 + np.arange(adim)[None, :] * 11) % nv).astype(np.int32)


def _run(kind, base, B, stats_out=None):
    if kind == "v1":
        env, adim = O.V1Vec(B, N=2, seed=17, env_id_base=base), 4
    else:
        env, adim = O.V0Vec(B, seed=17, env_id_base=base, random_opp=False), 1
    gids = base + np.arange(B)
    obs = [env.reset()]
    ret = np.zeros(B)
    stats = np.zeros(3)
    T = STEPS[kind]
    for t in range(T):
        a = _actions(kind, gids, t, adim)
        o, r, d, _ = env.step(a if kind == "v1" else a.reshape(-1))
        obs.append(o)
        ret += r
        stats[0] += ret[d].sum()
        stats[1] += d.sum()
        ret[d] = 0
    stats[2] = B * T
    return np.stack(obs, 1), stats


def _worker(rank, port, kind, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from gym_futbol_amd import distributed as D
    r = D.init(use_gpu=False)
    assert r.distributed and r.world == WORLD
    obs, stats = _run(kind, r.shard(B_PER_RANK), B_PER_RANK)
    st = D.reduce_episode_stats(torch.tensor(stats, dtype=torch.float64))
    slowest = D.max_over_ranks(1.0 + rank, r.device)
    gathered = [torch.zeros(obs.shape, dtype=torch.float64) for _ in range(WORLD)]
    torch.distributed.all_gather(gathered, torch.as_tensor(obs))
    D.barrier(r.device)
    if rank == 0:
        np.savez(os.path.join(outdir, "r0.npz"), obs=np.concatenate([g.numpy() for g in gathered], 0),
                 stats=st.numpy(), slowest=slowest)
    D.shutdown()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("kind", ["v1", "v0"])
def test_two_rank_shards_equal_one_process(kind, tmp_path):
    mp.spawn(_worker, args=(_free_port(), kind, str(tmp_path)), nprocs=WORLD, join=True)
    res = np.load(os.path.join(tmp_path, "r0.npz"))
    full_obs, full_stats = _run(kind, 0, B_PER_RANK * WORLD)
    assert np.array_equal(res["obs"], full_obs)
    assert res["stats"][1] == full_stats[1] and res["stats"][2] == full_stats[2] == WORLD * B_PER_RANK * STEPS[kind]
    assert np.isclose(res["stats"][0], full_stats[0], rtol=1e-12, atol=1e-9)
    assert full_stats[1] >= WORLD * B_PER_RANK        # every env finished an episode
    assert float(res["slowest"]) == 2.0


def test_shard_base_limits():
    from gym_futbol_amd.distributed import shard_base
    assert shard_base(3, 65536) == 196608
    with pytest.raises(ValueError):
        shard_base(65536, 65536)
