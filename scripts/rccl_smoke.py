"""RCCL calls of the multi-GPU path, run once on hardware with a one-rank world (diagnostic).

The N > 1 bench / training path uses exactly these torch.distributed calls on the "nccl" (RCCL)
backend (gym_futbol_amd/distributed.py): init_process_group(device_id=...), barrier(device_ids=...),
all_reduce(SUM) of the [return sum, episodes, env-steps] f64 stats and all_reduce(MAX) of the timed
region.  On a one-GPU box RCCL refuses two ranks on one device, so this forms a world of one rank on
cuda:0 -- the same API calls, communicator set-up and collective kernels, without the xGMI traffic --
and checks the results.  The 2-rank path itself is covered by the gloo tests and
scripts/gpu_multirank.sh.

    python scripts/rccl_smoke.py
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.perf_counter()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    init_s = time.perf_counter() - t0
    dist.barrier(device_ids=[dev.index])
    stats = torch.tensor([123.5, 7.0, 65536.0 * 300], dtype=torch.float64, device=dev)
    dist.all_reduce(stats)  # SUM, as distributed.reduce_episode_stats
    t = torch.tensor([0.0123], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # as distributed.max_over_ranks
    torch.cuda.synchronize(dev)
    ok = stats.tolist() == [123.5, 7.0, 65536.0 * 300] and t.item() == 0.0123
    out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "device": str(dev),
           "init_process_group_s": round(init_s, 3), "barrier": "ok", "all_reduce_sum": stats.tolist(),
           "all_reduce_max": t.item(), "results_ok": ok, "torch": torch.__version__,
           "hip": getattr(torch.version, "hip", None)}
    dist.destroy_process_group()
    print(json.dumps(out))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
