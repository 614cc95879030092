"""Throughput benchmark of the vectorised Futbol env step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs B] [--players 2] [--kind v1|v0]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N

Workload (BASELINE.json configs[1]/[3]): B = 65 536 independent 2v2 envs_v1
matches per GPU, synthetic random left-team actions (Philox, generated on the
GPU by one fill launch for all K timed steps before the timed region starts:
the inputs are resident in HBM, and each step kernel reads its own step's
actions), opponent random actions drawn inside the step kernel,
DummyVecEnv auto-reset; every step writes obs/reward/done to HBM.  (Staggered
episode phases would be --stagger 1; by default all envs run in lockstep, as DummyVecEnv
runs them, and a timed region shorter than an episode sits mid-episode).  A "step" =
one env-step launch over all B envs.  N > 1: one process per
GPU, env shards with global env ids rank*B..; weak scaling; one RCCL
all_reduce(SUM) of [episode-return sum, episodes, env-steps] every 300 steps
(the only collective: the envs never exchange anything).

Prints ONE JSON line (rank 0).  `roofline` is the step kernel's algorithmic
HBM bytes (579 B per 2v2 env-step) / its average duration,
measured live with HIP events on the launch stream; `cpu_baseline` times the
oracle/ C restatement of the same step on the host (kind "port": the
reference's own v1 step needs pymunk, absent here).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-futbol_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env-steps/sec (whole node), 2v2 Futbol, batch=65536 envs, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
# reference v0 FutbolEnv.step() timed by the survey (not this box): envs_v1 cannot
# run here (pymunk absent), so these are the only numbers of the reference's own code
REF_V0_PYTHON = {"random_opp_env_steps_per_s_1core": 14188, "hardcoded_opp_env_steps_per_s_1core": 12372,
                 "hardcoded_opp_env_steps_per_s_8proc": 65746,
                 "where": "survey container, 8 cores 'Intel(R) Xeon(R) Processor', Python 3.10 / numpy 2.2 "
                          "(SURVEY.md 6), not the GPU box"}


def metric_of(kind, n, B):
    """BASELINE.json's metric for its own configs (C2/C4 2v2 is the headline); the other kinds get a
    label of their own so that a C3 / C5 line is never read as the 2v2 metric."""
    if kind == "v1" and n == 2 and B == 65536:
        return METRIC
    if kind == "v1":
        return "env-steps/sec (whole node), %dv%d Futbol, batch=%d envs, MI355X" % (n, n, B)
    return "env-steps/sec (whole node), 2v2 Futbol-v0 with the hard-coded opponent, batch=%d envs, MI355X" % B


def workload_of(kind, n, B, world):
    if kind == "v0":
        return "C3: %d envs/GPU v0 FutbolEnv(random_opp=False), hard-coded opponent on the GPU" % B
    tag = {2: "C4" if world > 1 else "C2", 5: "C5"}.get(n, "envs_v1 %dv%d (not a BASELINE config)" % (n, n))
    return "%s: %d envs/GPU envs_v1 %dv%d, synthetic random actions, auto-reset" % (tag, B, n, n)


def host_cpu():
    """CPU model and thread counts of this host (cpu_baseline context)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff}


def c1_baseline(n=2, steps=100000):
    """1 env, 1 thread, 100 000 steps, state seed 0, left actions from the synthetic
    Philox stream (seed 1234), auto-reset -- the oracle (C restatement) in a C loop: the reference's own
    envs_v1 step needs pymunk, absent here."""
    import ctypes as C
    from oracle import oracle as O
    L = O.lib()
    e = O.OrcV1()
    L.orc_v1_init(C.byref(e), n, 105.0, 68.0, 30.0, 0, 0)
    obs = np.zeros(4 * (2 * n + 1))
    L.orc_v1_reset(C.byref(e), obs.ctypes.data)
    ret = C.c_double()
    t0 = time.perf_counter()
    eps = L.orc_v1_run(C.byref(e), steps, 1234, C.byref(ret))
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port", "envs": 1, "steps": steps,
            "seconds": dt, "episodes": eps, "mean_return": ret.value / max(eps, 1),
            "sample": "C1: oracle/liboracle.so orc_v1_run, 1 env %dv%d, 1 thread, %d steps, seed 0, Philox(1234) "
                      "left actions, auto-reset" % (n, n, steps)}


def algo_bytes_per_env_step(kind, n, out_bytes):
    """state read+write + actions + obs/reward/done writes (contact cache excluded)."""
    if kind == "v1":
        nb = 2 * n + 1
        return 2 * (48 * nb + 5) + 2 * n + 4 * nb * out_bytes + out_bytes + 1
    return 2 * (25 * 8 + 14) + 1 + 30 * out_bytes + out_bytes + 1


def cpu_threads():
    """Every host core this process may run on (its affinity mask): SURVEY 8(d) times the restatement
    "on all host cores"."""
    if hasattr(os, "sched_getaffinity"):
        return max(1, len(os.sched_getaffinity(0)))
    return max(1, os.cpu_count() or 1)


def cpu_quota():
    """The CPU time this process's cgroup may use, in CPUs (cgroup v2 cpu.max or v1 cfs quota), or None
    when unlimited / unknown.  (The GPU box's affinity mask lists all 256 host CPUs, but its share is a
    quota: 256 threads there ran at 11.6 M env-steps/s against 26.5 M on 16.)"""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                return max(1, math.ceil(int(q) / int(per)))
            return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return max(1, math.ceil(q / per)) if q > 0 else None
    except (OSError, ValueError):
        return None


def omp_share():
    """OMP_NUM_THREADS when set (16 on the GPU box: its CPU share per GPU), else None."""
    try:
        t = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        return None
    return t if t > 0 else None


def cpu_baseline(kind, n, budget_s=8.0, B=65536):
    """The oracle (faithful build) on the same B-env workload: every env stepped by the C loop of
    orc_v1_run / orc_v0_vec_run (synthetic Philox actions, auto-reset, obs / reward written every step,
    no Python per step), envs split over OpenMP threads -- on all host cores (`value`, `cores`), on
    the OMP_NUM_THREADS share and on 1 thread.  Each figure is a ~budget_s run whose step count is
    extrapolated from a calibration run of at least 0.5 s."""
    from oracle import oracle as O
    if kind == "v1":
        ora = O.V1Vec(B, N=n, seed=0)
    else:
        ora = O.V0Vec(B, seed=0, random_opp=False)
    ora.reset()

    def timed(nthreads):
        steps = 1
        while True:  # calibration
            t0 = time.perf_counter()
            ora.run(steps, 1234, nthreads)
            dt = time.perf_counter() - t0
            if dt >= 0.5 or steps >= 1 << 20:
                break
            steps *= 2
        steps = max(1, int(steps * budget_s / dt))
        t0 = time.perf_counter()
        eps, _ = ora.run(steps, 1234, nthreads)
        dt = time.perf_counter() - t0
        return {"value": steps * B / dt, "threads": nthreads, "steps": steps, "seconds": dt, "episodes": eps}

    what = "envs_v1 %dv%d" % (n, n) if kind == "v1" else "v0 hard-coded-opponent"
    T = cpu_threads()
    allc = timed(T)
    share = omp_share()
    quota = cpu_quota()
    sh = timed(share) if share and share != T else None
    qt = timed(quota) if quota and quota not in (T, share) else None
    one = timed(1) if T > 1 else allc
    # the baseline is the host's best: every core of the affinity mask, or the cgroup's CPU quota / the
    # OMP_NUM_THREADS share when the mask lists more CPUs than the process may use (all reported)
    best = max([r for r in (allc, sh, qt) if r], key=lambda r: r["value"])
    out = {"value": best["value"], "unit": "env-steps/s", "cores": best["threads"], "kind": "port",
           "sample": "oracle/liboracle.so (C restatement of the %s step), %d envs x %d steps (%.1f s) on %d OpenMP "
                     "threads (the fastest of: all %d CPUs of the affinity mask, the OMP_NUM_THREADS share %s, the "
                     "cgroup quota %s); each thread steps its own envs in a C loop (synthetic Philox actions, "
                     "auto-reset)" % (what, B, best["steps"], best["seconds"], best["threads"], T, share, quota),
           "all_cores": allc, "omp_share": sh, "cgroup_quota_cpus": quota, "quota_run": qt, "single_thread": one,
           "single_thread_value": one["value"], "host": host_cpu(), "reference_v0_python": REF_V0_PYTHON}
    if kind == "v1" and n == 2:
        out["c1"] = c1_baseline(n)
    return out


def rollout_companion(args):
    """The same workload stepped by open-loop rollout launches (futbol_rollout, 100 steps per launch:
    the synthetic actions do not depend on the observations, so a launch can run many steps and its
    blocks never wait for each other between steps), measured by a child bench.py run.  Reported
    beside `value`, which stays the one-launch-per-step (lockstep, DummyVecEnv) rate."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--envs", str(args.envs), "--players", str(args.players), "--kind", args.kind, "--rollout", "100",
           "--no-cpu-baseline", "--no-rollout-line", "--stagger", str(args.stagger)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        ln = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
        d = json.loads(ln)
    except Exception as e:  # noqa: BLE001 - report, never fail the main line
        return {"error": repr(e)[:300]}
    r = d["roofline"]
    return {"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"], "steps_per_launch": 100,
            "kernel_ms_per_step": r["kernel_ms"], "achieved": r["achieved"], "frac": r["frac"],
            "launch": d["config"]["launch"], "command": " ".join(["bench.py"] + cmd[2:])}


def copy_ceiling(dev, mib=1024, reps=10):
    """Measured HBM stream-copy ceiling (SURVEY 8(d) Roofline): futbol_stream_copy of a `mib` MiB
    buffer (16 B per lane), HIP events on the launch stream; GB/s = 2 x bytes / time."""
    from gym_futbol_amd import _native as nat
    nbytes = mib << 20
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(dev)
    lib = nat.load()
    for _ in range(2):
        nat.check(lib.futbol_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, stream.cuda_stream))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        nat.check(lib.futbol_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, stream.cuda_stream))
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    ok = bool(torch.equal(src[:4096], dst[:4096]))
    del src, dst
    return {"gbs": 2 * nbytes / (ms * 1e-3) / 1e9, "bytes_copied": nbytes, "ms_per_copy": ms, "verified": ok,
            "method": "futbol_stream_copy (16 B/lane, 4 loads in flight per lane), %d MiB, %d reps, HIP events"
                      % (mib, reps)}


def pmc_traffic(kind, n, B):
    """HBM bytes per step-kernel launch from the committed rocprofv3 --pmc pass of this
    same configuration (scripts/gpu_profile.sh -> scripts/pmc_traffic.py ->
    profiles/<round>/traffic.json), or (None, None) when no matching entry exists."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")), reverse=True):
        try:
            with open(path) as f:
                entries = json.load(f)
        except (OSError, ValueError):
            continue
        for e in entries:
            if e.get("kind") == kind and e.get("players", n) == n and e.get("envs") == B:
                return e["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


STAMP_SLOTS = ["load state", "actions + opponent RNG", "process_action + out-of-bounds", "phase glue",
               "collide: contacts + records (work list)", "cache lookups + integrate v", "solve: items, warm start, 10 sweeps",
               "arbiter cache update", "reward / goal / time", "goal reset + auto-reset phases", "obs + store"]
STAMP_STRIDE = 32  # u64 slots per wave (futbol_kernels.hpp kStampStride)
SUB_SLOTS = {16: "integrate p", 17: "collide: stage rows", 18: "collide: hit tests (segments, pairs)",
             19: "solve: publish rows / records / work list", 20: "process_action: exact squares (batch)",
             21: "process_action: player loop", 22: "cache lookups past the preloaded entries"}
# (slot 2 is then the out-of-bounds test + segment-table store, slot 5 integrate v + clamp)


def stamps_report(venv, one_step, args):
    """Per-phase s_memtime breakdown of the step kernel (diagnostic build)."""
    import ctypes as C
    from gym_futbol_amd import _native as nat
    nblk = (venv.num_envs + 63) // 64
    buf = np.zeros((nblk + 1) * STAMP_STRIDE, np.uint64)
    nat.check(nat.load().futbol_debug_stamps(venv.ctx.h, buf.ctypes.data, buf.size, 1), venv.ctx.h)
    steps = args.steps
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    nat.check(nat.load().futbol_debug_stamps(venv.ctx.h, buf.ctypes.data, buf.size, 0), venv.ctx.h)
    epw = 64
    per = buf[:nblk * STAMP_STRIDE].reshape(nblk, STAMP_STRIDE).astype(np.float64).sum(0) / (nblk * steps * (64 // epw))
    tot = per[:11].sum() + sum(per[k] for k in SUB_SLOTS)
    rep = {"diagnostic": "stamps", "envs_per_wave": epw, "steps": steps, "ms_per_step_wall": wall / steps * 1e3,
           "cycles_per_wave_step_total": tot,
           "phases": dict([(STAMP_SLOTS[i], {"cycles": per[i], "share": per[i] / tot}) for i in range(11)] +
                          [(SUB_SLOTS[k], {"cycles": per[k], "share": per[k] / tot}) for k in SUB_SLOTS]),
           "solver_records_per_wave_step": per[15],
           "segment_candidate_iterations_per_wave_step": per[24], "segment_contact_iterations_per_wave_step": per[25],
           # FUTBOL_STAT slots (space_step phase 0): contact work-list hits per wave-step, the fraction of
           # wave-steps whose hits overflow the work-list table (every lane computes its own contacts),
           # with a lane past the preloaded cache entries, with spill records; out-of-bounds, goals
           "worklist_hits_per_wave_step": per[26], "worklist_overflow_wave_frac": per[27],
           "cache_past_preload_wave_frac": per[28], "spill_wave_frac": per[29],
           "out_of_bounds_per_wave_step": per[30], "goals_per_wave_step": per[31]}
    # single-launch snapshots: wave start/end (100 MHz realtime), cycles, placement
    snaps = []
    waves = []  # per-wave slots of every snapshot launch (tail study: --stamps-dump)
    slow = np.zeros(STAMP_STRIDE)
    for k in range(args.snapshots):
        for _ in range(args.snapshot_stride - 1):
            one_step()
        nat.check(nat.load().futbol_debug_stamps(venv.ctx.h, buf.ctypes.data, buf.size, 1), venv.ctx.h)  # clear
        one_step()
        torch.cuda.synchronize()
        nat.check(nat.load().futbol_debug_stamps(venv.ctx.h, buf.ctypes.data, buf.size, 0), venv.ctx.h)
        w = buf[:nblk * STAMP_STRIDE].reshape(nblk, STAMP_STRIDE)
        waves.append(w.copy())
        slow += w[int(np.argmax(w[:, 13]))].astype(np.float64)   # phases of this launch's slowest wave
        t0_, t1_, cyc, hw = (w[:, 11].astype(np.float64), w[:, 12].astype(np.float64),
                             w[:, 13].astype(np.float64), w[:, 14])
        place = (hw >> np.uint64(32)) * np.uint64(1 << 12) + ((hw >> np.uint64(4)) & np.uint64(0xFFF))
        _, per_simd = np.unique(place, return_counts=True)
        dur = (t1_ - t0_) / 100.0
        snaps.append({"span_us": (t1_.max() - t0_.min()) / 100.0, "start_spread_us": (t0_.max() - t0_.min()) / 100.0,
                      "wave_us_mean": dur.mean(), "wave_us_p90": float(np.percentile(dur, 90)), "wave_us_max": dur.max(),
                      "wave_cycles_mean": cyc.mean(), "wave_cycles_max": cyc.max(),
                      "simds_used": int(len(per_simd)), "max_waves_per_simd": int(per_simd.max())})
    rep["slowest_wave_phases"] = dict([(STAMP_SLOTS[i], slow[i] / max(len(snaps), 1)) for i in range(11)] +
                                      [(SUB_SLOTS[k], slow[k] / max(len(snaps), 1)) for k in SUB_SLOTS])
    rep["slowest_wave_records"] = slow[15] / max(len(snaps), 1)
    rep["snapshots"] = snaps
    rep["snapshot_mean"] = {k: float(np.mean([x[k] for x in snaps])) for k in snaps[0]} if snaps else None
    if args.stamps_dump:
        np.save(args.stamps_dump, np.stack(waves))
    print(json.dumps(rep, indent=1))
    venv.close()


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) without an external launcher: N child processes of this same script, rank r
    on LOCAL_RANK r (its GPU), rendezvous at 127.0.0.1 on a free port -- what torchrun would set up.
    It runs right after argument parsing, before this process imports the package or touches the GPU
    (the parent only starts and waits for its children; it never initialises HIP and never execs).
    Rank 0's JSON line reaches the caller through the inherited stdout.  Returns 0 when every rank
    succeeded, else the first failing rank's exit status (the other ranks are then terminated, since
    they would wait for it at the next collective)."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            c = procs[r].poll()
            if c is None:
                continue
            alive.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print("bench.py: rank %d exited with status %d; stopping the other ranks" % (r, c),
                      file=sys.stderr, flush=True)
                for q in alive:
                    procs[q].send_signal(signal.SIGTERM)
        time.sleep(0.1)
    return rc


def launcher_selftest(fail_rank):
    """CPU check of the launcher (tests/test_bench_launcher.py): the ranks form a gloo world and
    all-reduce their rank + 1; rank 0 prints {"ranks": world, "sum": ...}.  No GPU, no package."""
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    if rank == fail_rank:
        sys.exit(3)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([float(rank + 1)])
    local = [int(os.environ.get("LOCAL_RANK", "0"))]
    if world > 1:
        dist.all_reduce(t)
        local = [None] * world
        dist.all_gather_object(local, int(os.environ.get("LOCAL_RANK", "0")))
    if rank == 0:
        print(json.dumps({"ranks": world, "sum": float(t.item()), "master_addr": os.environ.get("MASTER_ADDR"),
                          "local_ranks": local}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--kind", default="v1", choices=["v1", "v0", "c1"],
                    help="v1: envs_v1 (C2/C4, --players 5: C5); v0: hard-coded opponent (C3); c1: the C1 CPU line")
    ap.add_argument("--graph", type=int, default=1, help="replay the timed steps from a hipGraph")
    ap.add_argument("--direct", type=int, default=0,
                    help="1: launch the timed steps one by one (pre-generated actions, no hipGraph)")
    ap.add_argument("--groups", type=int, default=1,
                    help="step the B envs as this many independent env groups (B/groups envs each: one "
                         "context, HIP stream and hipGraph per group) that advance asynchronously")
    ap.add_argument("--stagger", type=int, default=0,
                    help="1: spread the envs' episode starts over an episode (slower: every wave then mixes "
                         "contact-heavy and formation phases); 0: all envs in lockstep as DummyVecEnv runs them")
    ap.add_argument("--rollout", type=int, default=0,
                    help="N > 0: step with open-loop rollout launches of up to N steps each (futbol_rollout: the "
                         "synthetic actions do not depend on the observations), instead of one launch per step")
    ap.add_argument("--no-rollout-line", action="store_true",
                    help="skip the open_loop_rollout companion measurement (a child bench.py --rollout 100 run)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=600,
                    help="steps timed per-kernel with HIP events (a multiple of the episode length)")
    ap.add_argument("--snapshots", type=int, default=24, help="--stamps: single-launch wave snapshots")
    ap.add_argument("--snapshot-stride", type=int, default=5, help="--stamps: steps between snapshots")
    ap.add_argument("--stamps-dump", default="",
                    help="--stamps: save every snapshot's per-wave slots [snapshots, waves, 32] to this .npy")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic: load the FUTBOL_STAMPS build and print the per-phase cycle breakdown")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launcher-selftest-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.direct and args.rollout:
        ap.error("--direct launches one futbol_step per step; it cannot be combined with --rollout")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started here (nothing has touched the GPU yet); under torchrun the
        # ranks already exist and WORLD_SIZE is set
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launcher_selftest:
        return launcher_selftest(args.launcher_selftest_fail_rank)
    if args.kind == "c1":  # 1 env on 1 CPU thread, no GPU
        c1 = c1_baseline(args.players)
        print(json.dumps({"metric": "env-steps/sec, 1 env %dv%d envs_v1 step, 1 CPU thread (C1)"
                          % (args.players, args.players), "value": c1["value"], "unit": "env-steps/s",
                          "n_gpus": 0, "steps": c1["steps"], "warmup": 0, "ms_per_step": 1e3 / c1["value"],
                          "higher_is_better": True, "scaling": None, "vs_baseline": None, "dtype": "f64",
                          "data": "synthetic", "config": {"workload": c1["sample"]}, "host": host_cpu(),
                          "episodes": c1["episodes"], "mean_return": c1["mean_return"],
                          "reference_v0_python": REF_V0_PYTHON}), flush=True)
        return
    if args.stamps:
        os.environ.setdefault("FUTBOL_LIB_VARIANT", "stamps")  # (a stamps build of another variant: set it)

    from gym_futbol_amd import FutbolVecEnv
    from gym_futbol_amd import distributed as D
    R = D.init(use_gpu=True)          # one process per GPU; RCCL when world > 1
    rank, world, dev = R.rank, R.world, R.device
    B = args.envs
    n = args.players
    kw = {"number_of_player": n} if args.kind == "v1" else {"random_opp": False}
    venv = FutbolVecEnv(args.kind, B, device=dev, seed=0, env_id_base=R.shard(B), dtype=torch.float32, **kw)
    venv.reset()
    act = venv._act
    stream = torch.cuda.current_stream(dev)
    ALL = 2**64 - 1  # device step counter (advanced by every step launch)

    def one_step():
        venv.random_actions(ALL, seed=1234, out=act)
        venv.step_raw(act)

    def stagger(ve, base):
        """Untimed pre-roll to the steady state of a long-running vector env: the episodes of
        the B envs start at spread-out steps (env with global id g starts at pre-roll step
        (g * 131) mod L, L = the episode length), so any window of steps -- the driver's short
        K as well as whole episodes -- sees every episode phase in the same proportion instead
        of all envs in formation at once.  Same per-env dynamics; only the reset times move."""
        L = ve.episode_steps
        gid = torch.arange(ve.num_envs, device=dev, dtype=torch.int64) + base
        phase = (gid * 131) % L
        a = ve._act
        for t in range(L):
            ve.reset((phase == t).to(torch.uint8))
            ve.random_actions(ALL, seed=1234, out=a)
            ve.step_raw(a)

    if args.stagger:
        stagger(venv, R.shard(B))
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize(dev)

    # per-kernel timing of the dominant kernel (the env step), two ways, over whole episodes
    # (all envs start together, so the per-step cost varies with the episode phase):
    #  (1) HIP events around a hipGraph of `profile_steps` back-to-back step launches with
    #      pre-generated actions (the way the kernel runs in the timed region) -> kernel_ms
    #  (2) events stamped by each dispatch (hipExtLaunchKernelGGL)           -> kernel_ms_dispatch
    acts = torch.empty((args.profile_steps,) + tuple(act.shape), dtype=torch.uint8, device=dev)
    for t in range(args.profile_steps):
        venv.random_actions(10**6 + t, seed=1234, out=acts[t])
    RL = max(0, int(args.rollout))
    rbuf = None
    if RL:  # the rollout launches' output buffers [RL, B, ...] (reused by every launch)
        rbuf = venv.rollout(acts[:min(RL, args.profile_steps)].contiguous())
    kg = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(stream)
    with torch.cuda.stream(s):
        with torch.cuda.graph(kg, stream=s):
            if RL:
                for t0_ in range(0, args.profile_steps, RL):
                    n_ = min(RL, args.profile_steps - t0_)
                    venv.rollout(acts[t0_:t0_ + n_], out=tuple(b[:n_] for b in rbuf))
            else:
                for t in range(args.profile_steps):
                    venv.step_raw(acts[t])
    stream.wait_stream(s)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    kg.replay()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = e0.elapsed_time(e1) / args.profile_steps
    del kg, acts
    venv.kernel_timing(True)
    if RL:
        a_ = venv.random_actions_steps(min(RL, args.profile_steps), ALL, seed=1234)
        for _ in range(max(1, args.profile_steps // RL)):
            venv.rollout(a_, out=tuple(b[:a_.shape[0]] for b in rbuf))
        tot_ms, cnt = venv.kernel_timing(False)
        kernel_ms_dispatch = tot_ms / max(cnt * a_.shape[0], 1)
        del a_
    else:
        for _ in range(args.profile_steps):
            one_step()
        tot_ms, cnt = venv.kernel_timing(False)
        kernel_ms_dispatch = tot_ms / max(cnt, 1)

    if args.stamps:
        return stamps_report(venv, one_step, args)

    # timed loop: hipGraphs of G steps.  The synthetic policy does not look at observations,
    # so one launch before the timed region draws the actions of all K steps ([K, B, 2N] u8 in
    # HBM: the inputs are resident when the timed region starts) and each step kernel of the
    # chunk graphs reads its own step's slice.
    # --groups g > 1: the B envs of this GPU are stepped as g independent groups of B/g envs
    # (their own contexts with env ids base + k*B/g.., so every env's trajectory is the same
    # as in the one-context run), each on its own HIP stream replaying its own graph.  A
    # group's next step waits only for ITS previous step, so the waves of one group's step
    # fill the SIMDs that another group's slowest waves leave idle (EnvPool-style async
    # groups; the per-launch roofline above is measured on the single full-batch launch).
    ngroups = max(1, int(args.groups))
    if B % ngroups or (B // ngroups) % 64:
        raise SystemExit("--groups must split --envs into multiples of 64")
    if ngroups > 1:
        kw_g = dict(kw)
        groups = [FutbolVecEnv(args.kind, B // ngroups, device=dev, seed=0,
                               env_id_base=R.shard(B) + g * (B // ngroups), dtype=torch.float32, **kw_g)
                  for g in range(ngroups)]
        for ge in groups:
            ge.reset()
    else:
        groups = [venv]
    streams = [torch.cuda.Stream(dev) for _ in groups]

    graphs = None
    # graphs of Gs steps each (+ the remainder as a second graph), so that short timed regions
    # (the driver's K = 20) are replayed from a graph too rather than launched step by step
    Gs = min(100, args.steps)

    chunks = [(t0_, min(Gs, args.steps - t0_)) for t0_ in range(0, args.steps, Gs)]

    rbufs = {}

    def capture(ge, s, abuf, t0_, nsteps):
        g_ = torch.cuda.CUDAGraph()
        s.wait_stream(stream)
        with torch.cuda.stream(s):
            if RL and id(ge) not in rbufs:
                rbufs[id(ge)] = ge.rollout(abuf[t0_:t0_ + min(RL, nsteps)].contiguous())
            with torch.cuda.graph(g_, stream=s):
                if RL:  # one open-loop rollout launch per RL steps of the chunk
                    for r0 in range(0, nsteps, RL):
                        n_ = min(RL, nsteps - r0)
                        ge.rollout(abuf[t0_ + r0:t0_ + r0 + n_], out=tuple(b[:n_] for b in rbufs[id(ge)]))
                else:
                    for t in range(nsteps):
                        ge.step_raw(abuf[t0_ + t])
        stream.wait_stream(s)
        return g_

    direct_abuf = None
    if args.direct:  # the timed steps launched one by one from Python, actions pre-generated like the graphs'
        args.graph = 0
        direct_abuf = torch.zeros((args.steps, venv.num_envs, venv.action_dim), dtype=torch.uint8, device=dev)
    if args.graph:
        graphs = []
        for ge, s in zip(groups, streams):
            if ge is not venv:  # warm the group up like the main context
                if args.stagger:
                    stagger(ge, R.shard(B) + groups.index(ge) * (B // ngroups))
                for _ in range(args.warmup + 2 * args.profile_steps):
                    ge.random_actions(ALL, seed=1234, out=ge._act)
                    ge.step_raw(ge._act)
            # zeros (valid noop actions) until the timed region's fill: the untimed warm replay below
            # steps on them, and must not feed uninitialised bytes to the kernel
            abuf = torch.zeros((args.steps, ge.num_envs, ge.action_dim), dtype=torch.uint8, device=dev)
            graphs.append(([capture(ge, s, abuf, t0_, n_) for t0_, n_ in chunks], abuf))
        # one untimed replay of each graph: the first launch of a graph pays its upload
        for (gl, abuf), s in zip(graphs, streams):
            with torch.cuda.stream(s):
                for g_ in gl:
                    g_.replay()
        torch.cuda.synchronize(dev)
    elif ngroups > 1:
        raise SystemExit("--groups needs --graph 1")

    # all envs run their fixed-length episodes in lockstep (DummyVecEnv: one reset at the
    # start, auto-reset every L steps), and a step's cost depends on the episode phase (the
    # first ~75 steps from formation are cheap).  A timed region shorter than an episode is
    # placed in the middle of one by untimed steps, so that it does not sit on the cheap start;
    # K a multiple of L measures whole episodes exactly.
    L = venv.episode_steps
    align = 0
    if not args.stagger and args.steps < L:
        at = (args.warmup + 2 * args.profile_steps + (args.steps if graphs is not None else 0)) % L  # every env's step
        align = ((L - args.steps) // 2 - at) % L
        for ge, s in zip(groups, streams):
            with torch.cuda.stream(s):
                for _ in range(align):
                    ge.random_actions(ALL, seed=1234, out=ge._act)
                    ge.step_raw(ge._act)
            stream.wait_stream(s)

    def all_stats():
        tot = torch.zeros(3, dtype=torch.float64, device=dev)
        for ge in groups:
            tot += ge.episode_stats(clear=False)
        return tot

    stats_buf = torch.zeros(3, dtype=torch.float64, device=dev)
    for ge in groups:
        ge.episode_stats(clear=True)
    fill_ms = None
    if direct_abuf is not None:
        venv.random_actions_steps(args.steps, ALL, seed=1234, out=direct_abuf)
        torch.cuda.synchronize(dev)
    if graphs is not None:  # the synthetic inputs of the K timed steps, fresh draws, into HBM
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record(stream)
        for ge, (gl, abuf), s in zip(groups, graphs, streams):
            s.wait_stream(stream)
            with torch.cuda.stream(s):
                ge.random_actions_steps(args.steps, ALL, seed=1234, out=abuf)
            stream.wait_stream(s)
        f1.record(stream)
        torch.cuda.synchronize(dev)
        fill_ms = f0.elapsed_time(f1) / args.steps
    D.barrier(dev)
    torch.cuda.synchronize(dev)
    dbg = os.environ.get("FUTBOL_BENCH_DEBUG") and (graphs is not None or direct_abuf is not None)
    if dbg:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(streams[0] if graphs is not None else stream)
    t0 = time.perf_counter()
    done_steps = 0
    ci = 0
    while done_steps < args.steps:
        chunk = chunks[ci][1] if graphs is not None else 1
        if graphs is not None:
            for (gl, abuf), s in zip(graphs, streams):
                with torch.cuda.stream(s):
                    gl[ci].replay()
            ci += 1
        elif ngroups > 1:
            for ge, s in zip(groups, streams):
                with torch.cuda.stream(s):
                    for _ in range(chunk):
                        ge.random_actions(ALL, seed=1234, out=ge._act)
                        ge.step_raw(ge._act)
        elif direct_abuf is not None:
            venv.step_raw(direct_abuf[done_steps])
        else:
            for _ in range(chunk):
                one_step()
        prev = done_steps
        done_steps += chunk
        if R.distributed and done_steps // 300 != prev // 300:
            for s in streams:
                stream.wait_stream(s)
            stats_buf.copy_(all_stats())
            D.reduce_episode_stats(stats_buf)  # RCCL over xGMI: [sum return, episodes, env-steps]
    if dbg:
        ev1.record(streams[0] if graphs is not None else stream)
    torch.cuda.synchronize(dev)
    D.barrier(dev)
    elapsed = D.max_over_ranks(time.perf_counter() - t0, dev)
    if dbg:
        print("debug: wall %.1f us, events on the replay stream %.1f us" % (elapsed * 1e6, ev0.elapsed_time(ev1) * 1e3),
              file=sys.stderr, flush=True)
    stats = D.reduce_episode_stats(all_stats().clone()).cpu().numpy()

    total_env_steps = B * args.steps * world
    value = total_env_steps / elapsed
    out_bytes = 4
    per_env = algo_bytes_per_env_step(args.kind, n, out_bytes)
    achieved = per_env * B / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args.kind, n, B)
    ndev = D.distinct_devices(dev)
    ceil = copy_ceiling(dev) if rank == 0 else None
    line = {
        "metric": metric_of(args.kind, n, B), "value": value, "unit": "env-steps/s", "n_gpus": ndev,
        "ranks": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": workload_of(args.kind, n, B, world),
                   "actions": ("synthetic Philox left-team actions of all %d timed steps drawn on the GPU by one "
                               "fill launch before the timed region (resident in HBM, not timed; the fill costs "
                               "action_fill_ms_per_step); the opponent's actions are drawn inside the step kernel"
                               % args.steps) if (graphs is not None or direct_abuf is not None) else
                              "synthetic Philox left-team actions drawn by a fill launch before every step (timed)",
                   "action_fill_ms_per_step": fill_ms,
                   "launch": ("open-loop rollout launches of up to %d steps (futbol_rollout; every step writes its "
                              "obs / reward / done slice)" % RL) if RL else
                             ("one futbol_step launch per step, launched one by one" if direct_abuf is not None else
                              "one futbol_step launch per step, replayed from hipGraphs"),
                   "episode_phases": "staggered" if args.stagger else "lockstep (DummyVecEnv)",
                   "timed_from_episode_step": None if args.stagger else
                   (args.warmup + 2 * args.profile_steps + (args.steps if graphs is not None else 0) + align)
                   % venv.episode_steps,
                   "envs_per_gpu": B, "global_envs": B * world, "parallelism": "dp%d" % world,
                   "obs_dtype": "f32", "hip_graph": bool(graphs is not None), "env_groups": ngroups},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "copy_ceiling_gbs": ceil["gbs"] if ceil else None,
                     "frac_of_copy_ceiling": achieved / ceil["gbs"] if ceil else None,
                     "copy_ceiling": ceil,
                     "kernel": "v1_step_kernel<%d,float>" % n if args.kind == "v1" else "v0_step_kernel<float>",
                     "kernel_ms": kernel_ms, "kernel_ms_dispatch_events": kernel_ms_dispatch,
                     "kernel_timing": ("HIP events around a hipGraph of %d back-to-back step launches"
                                       % args.profile_steps) if not RL else
                                      ("HIP events around a hipGraph of %d steps as rollout launches of %d steps; "
                                       "per step" % (args.profile_steps, RL)),
                     "algo_bytes_per_launch": per_env * B,
                     "algo_bytes_per_env_step": per_env, "traffic_source": traffic_src},
        "episodes": {"finished": float(stats[1]),
                     "mean_return": float(stats[0] / stats[1]) if stats[1] else None},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.kind, n)
    if rank == 0 and world == 1 and not RL and not args.no_rollout_line and args.graph:
        line["open_loop_rollout"] = rollout_companion(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    for ge in groups:
        if ge is not venv:
            ge.close()
    venv.close()
    D.shutdown()


if __name__ == "__main__":
    main()
