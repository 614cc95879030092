"""Multi-GPU layout: one process per GPU, env shards, one tiny collective.

The reference scales only by running more independent envs (stable-baselines
DummyVecEnv in one process, colab_notebook.ipynb:818-823); envs never exchange
data.  Here each rank owns a contiguous shard of GLOBAL env ids
[rank*B, rank*B + B) on its own GPU -- since every env's randomness is keyed by
its global id (RNG tape), the union of the shards is
bit-identical to one process running all world*B envs (weak scaling, no
data-path collective).  The only communication is the all_reduce(SUM) of the
3-double episode statistics [return sum, episodes, env-steps], and the
max-over-ranks of the timed region in bench.py.

Backend: "nccl" (= RCCL over xGMI on ROCm) when the tensors live on a GPU,
"gloo" for the CPU tests.  Rendezvous from the torchrun environment
(RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT).
"""
import os

import torch
import torch.distributed as dist


class Rank:
    """rank / world / local_rank of this process and its device."""

    def __init__(self, rank, world, local_rank, device):
        self.rank, self.world, self.local_rank, self.device = rank, world, local_rank, device

    @property
    def distributed(self):
        return self.world > 1

    def shard(self, envs_per_rank):
        """Global env-id base of this rank's shard."""
        return shard_base(self.rank, envs_per_rank)


def shard_base(rank, envs_per_rank):
    base = int(rank) * int(envs_per_rank)
    if base + int(envs_per_rank) > 2**32:
        raise ValueError("global env ids must fit in 32 bits (RNG tape counter word)")
    return base


def init(backend=None, use_gpu=True):
    """Join the process group described by the torchrun environment (no-op for world 1).

    use_gpu: bind LOCAL_RANK's GPU and default to RCCL; otherwise CPU + gloo."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if use_gpu:
        # rehearsal of the multi-rank path on a one-GPU box: FUTBOL_SHARE_DEVICE=1 puts every
        # local rank on device local_rank % device_count (with FUTBOL_DIST_BACKEND=gloo, since RCCL
        # refuses two ranks on one GPU)
        dev_idx = local % max(1, torch.cuda.device_count()) if os.environ.get("FUTBOL_SHARE_DEVICE") else local
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or os.environ.get("FUTBOL_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        if backend == "nccl":
            dist.init_process_group(backend, device_id=device)
        else:
            dist.init_process_group(backend)
    return Rank(rank, world, local, device)


def reduce_episode_stats(stats):
    """In-place all_reduce(SUM) of a [return sum, episodes, env-steps] f64 tensor; returns it."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats)
    return stats


def max_over_ranks(seconds, device):
    """The slowest rank's timed region (bench contract)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def distinct_devices(device):
    """Number of distinct physical devices the ranks run on (host name + device UUID / PCI id):
    a rehearsal that puts several ranks on one GPU reports 1, not world."""
    import socket
    if device.type == "cuda":
        p = torch.cuda.get_device_properties(device)
        ident = str(getattr(p, "uuid", "")) or "%s:%s" % (getattr(p, "pci_bus_id", ""), getattr(p, "pci_device_id", ""))
    else:
        ident = "cpu"
    key = "%s/%s/%d" % (socket.gethostname(), ident, device.index if device.index is not None else -1)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return 1
    keys = [None] * dist.get_world_size()
    dist.all_gather_object(keys, key)
    return len(set(keys))


def barrier(device):
    if dist.is_initialized() and dist.get_world_size() > 1:
        if device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
