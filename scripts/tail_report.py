"""Summarise a stamps-build tail study (bench.py --stamps --stamps-dump waves.npy): per-phase
cycles of the mean wave and of each launch's slowest wave, launch max vs p90, and what the slowest
waves have in common (solver records m, hits, goals, out-of-bounds, cache/table overflows).

    python scripts/tail_report.py gpurun_out/it/stamps.log gpurun_out/it/waves.npy
"""
import json
import sys

import numpy as np

log, npy = sys.argv[1], sys.argv[2]
s = open(log).read()
d = json.loads(s[s.index("{"):])
print("%-45s %7s %6s %7s" % ("phase", "mean", "share", "slowest"))
for k, v in d["phases"].items():
    print("%-45s %7.0f %6.3f %7.0f" % (k, v["cycles"], v["share"], d["slowest_wave_phases"].get(k, 0)))
print("total mean %.0f" % d["cycles_per_wave_step_total"])
W = np.load(npy).astype(np.float64)[:, :-1] if np.load(npy).shape[1] % 2 else np.load(npy).astype(np.float64)
c = W[:, :, 13]
mid = c.mean(1) > 35000  # mid-episode launches
print("launches %d (mid-episode %d): max %.0f  p99 %.0f  p90 %.0f  mean %.0f" % (
    len(c), mid.sum(), c[mid].max(1).mean(), np.percentile(c[mid], 99, axis=1).mean(),
    np.percentile(c[mid], 90, axis=1).mean(), c[mid].mean()))
names = {15: "m", 26: "hits", 27: "table_ovf", 28: "cache_ovf", 29: "spill", 30: "out", 31: "goal"}
X = W[mid].reshape(-1, W.shape[2])
cx = X[:, 13]
for k, nm in names.items():
    v = X[:, k]
    print("%-10s mean %7.3f  corr %s" % (nm, v.mean(), ("%.3f" % np.corrcoef(v, cx)[0, 1]) if v.std() > 0 else "-"))
for m in range(9):
    f = X[:, 15] == m
    if f.any():
        print("m=%d  frac %.4f  cycles mean %.0f  max %.0f" % (m, f.mean(), cx[f].mean(), cx[f].max()))
g = X[:, 31] > 0
print("goal waves frac %.3f: cycles %.0f vs %.0f" % (g.mean(), cx[g].mean() if g.any() else 0, cx[~g].mean()))
