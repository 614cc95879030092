"""Copy the judged summaries of a scripts/gpu_profile.sh run from gpurun_out/prof into
profiles/<round>/ (tracked): the rocprofv3 --stats kernel table, per-kernel means of
the SQ counter passes, the bench line printed under the profiler, and the PMC
traffic entry (scripts/pmc_traffic.py).

    python scripts/prof_collect.py --round r01 --tag v1_2v2 [--kind v1 --players 2 --envs 65536]
"""
import argparse
import csv
import json
import os
import shutil
import statistics
import subprocess
import sys


def counter_means(path, key):
    agg = {}
    for r in csv.DictReader(open(path)):
        if key in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prof", default="gpurun_out/prof")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kind", default="v1")
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    dst = os.path.join("profiles", a.round)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(a.prof, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, "%s_kernel_stats.csv" % a.tag))
    key = ("v1_step_kernel<%d," % a.players) if a.kind == "v1" else "v0_step_kernel"
    counters = {}
    for p in ("sq", "sq2"):
        f = os.path.join(a.prof, p, "run_counter_collection.csv")
        if os.path.exists(f):
            counters.update(counter_means(f, key))
    bench_line = None
    for line in open(os.path.join(a.prof, "trace.log")):
        if line.startswith("{\"metric\""):
            bench_line = json.loads(line)
    out = {"kernel": key, "sq_counters_mean_per_launch": counters,
           "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md)",
           "bench_line_under_rocprofv3": bench_line}
    json.dump(out, open(os.path.join(dst, "%s_counters.json" % a.tag), "w"), indent=1)
    subprocess.check_call([sys.executable, os.path.join(os.path.dirname(__file__), "pmc_traffic.py"),
                           "--prof", a.prof, "--round", a.round, "--kind", a.kind,
                           "--players", str(a.players), "--envs", str(a.envs)], stdout=subprocess.DEVNULL)
    print("wrote", dst)


if __name__ == "__main__":
    main()
