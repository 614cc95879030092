"""envs_v1 squares at the full C2 / C5 workload (CPU only): the libm-faithful oracle against (a) the
kernels' arithmetic (portable build: glibc pow restated at the state sites, x*x in the reward) and
(b) x*x at every site (round 3's kernels: the faithful build with orc_v1_set_sq_mask(7)), 65 536 envs x
600 steps for N = 2 and N = 5 (round 4: profiles/r04/v1_sq_divergence.json; tests/sq_divergence.py).
Round 5: (a) for every team size N = 1..10 (profiles/r05/v1_sq_divergence_all.json).

    python scripts/v1_sq_divergence.py [--envs 65536] [--steps 600] [--players 1,2,...] [--masks none,7]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from sq_divergence import divergence  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--steps", type=int, default=600)
ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04", "v1_sq_divergence.json"))
ap.add_argument("--players", default="2,5")
ap.add_argument("--masks", default="none,7", help="none = the portable build (the kernels' arithmetic)")
a = ap.parse_args()
res = []
for n in [int(x) for x in a.players.split(",")]:
    for mask in [None if m == "none" else int(m) for m in a.masks.split(",")]:
        r = divergence(n, a.envs, a.steps, seed=0, nthreads=os.cpu_count() or 8, b_mask=mask)
        print(json.dumps(r), flush=True)
        res.append(r)
with open(a.out, "w") as f:
    json.dump(res, f, indent=1)
