"""How long is the split solve's critical path per wave, and what would per-component items give?
(CPU, oracle; design study for the N >= 4 solve.)

The split solve runs one item per (env, half) -- per (env, connected component, half) for N <= 3 --
on the wave's lanes; its time is set by the wave's longest item (records x 11 half-applications).
This steps B envs of the oracle (synthetic actions, auto-reset) and, after every step, reads each env's
arbiters of that step (arb_inlist) and computes per 64-env wave:
  whole   = max over envs of the env's record count             (the item length today for N >= 4)
  comp    = max over envs of its largest connected component      (per-component items)
  items   = sum over envs of its components                        (must fit the wave's lanes per half)
Records sharing a dynamic body are connected; segment records belong to their body's component.

  python scripts/solve_chain_sim.py --players 5 --envs 4096 --steps 600
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import O  # noqa: E402


def components(inl, n):
    """inl: [B, P] arbiters in this step's list -> (records [B], largest component's records [B],
    components [B])"""
    B = inl.shape[0]
    nb = 2 * n + 1
    pairs = [(i, j) for i in range(nb) for j in range(i + 1, nb)]
    seg = inl[:, :nb * 12].reshape(B, nb, 12).sum(2)             # segment records per body
    pc = inl[:, nb * 12:nb * 12 + len(pairs)].astype(bool)       # pair hits
    lab = np.tile(np.arange(nb), (B, 1))
    pi = np.array([p[0] for p in pairs])
    rows = np.arange(B)
    for _ in range(nb):  # min-label propagation over the pair edges to a fixed point
        old = lab.copy()
        for q, (i, j) in enumerate(pairs):
            sel = pc[:, q]
            if sel.any():
                m = np.minimum(lab[sel, i], lab[sel, j])
                lab[sel, i] = m
                lab[sel, j] = m
        for _ in range(5):
            lab = lab[rows[:, None], lab]
        if np.array_equal(lab, old):
            break
    rec = np.zeros((B, nb), np.int64)                            # records per component label
    np.add.at(rec, (np.repeat(np.arange(B), nb), lab.ravel()), seg.ravel())
    pl = np.where(pc, lab[:, pi], nb)
    for q in range(len(pairs)):
        hit = pc[:, q]
        rec[hit, pl[hit, q]] += 1
    return rec.sum(1), rec.max(1), (rec > 0).sum(1), rec


def _inorder(lens, A=64):
    """lane w solves items w, w + A, ...: the largest lane sum"""
    if not len(lens):
        return 0
    L = np.zeros(A)
    for i, l in enumerate(lens):
        L[i % A] += l
    return L.max()


def _lpt(lens, A=64):
    """longest item first, each to the least-loaded lane"""
    if not len(lens):
        return 0
    if len(lens) <= A:
        return max(lens)
    import heapq
    h = [0.0] * A
    for l in sorted(lens, reverse=True):
        heapq.heapreplace(h, h[0] + l)
    return max(h)


def _rounds(lens, A=64):
    """the wave runs rounds of A items; each round costs its longest item (the loops are wave-uniform)"""
    return sum(max(lens[i:i + A]) for i in range(0, len(lens), A)) if lens else 0


def strategies(comps_per_env, A=64, spill_k=4):
    """comps_per_env: per env of one wave, the list of its components' record counts.  The wave's solve
    cost in record-units (rounds of A items, each round as long as its longest item):
      whole:     one item per env and half, in env order (today's N >= 4 solve);
      comp:      one item per component and half, in env order;
      comp_sort: the same items, longest first (round 1 = the A longest);
      split:     components for the envs with the most records, whole items for the others, as many
                 envs split (longest first) as keep the items within one round"""
    whole = [sum(c) for c in comps_per_env if c]
    items_whole = [x for x in whole for _ in (0, 1)]
    items_comp = [x for c in comps_per_env for x in c for _ in (0, 1)]
    order = sorted([c for c in comps_per_env if c], key=lambda c: -sum(c))
    items = [sum(c) for c in order for _ in (0, 1)]
    best = _rounds(items_whole, A)
    k = 0
    for k in range(1, len(order) + 1):  # split the k longest envs
        its = [x for c in order[:k] for x in c for _ in (0, 1)] + [sum(c) for c in order[k:] for _ in (0, 1)]
        if len(its) > A:
            break
        best = min(best, max(its))
    def bucket(x):  # long items first by 4 length classes (stable within a class)
        return 0 if x >= 5 else (1 if x >= 3 else (2 if x == 2 else 3))
    items_b = sorted(items_comp, key=bucket)
    rounds_global = (-(-len(items_whole) // A)) * (max(items_whole) if items_whole else 0)  # today's code
    return (_rounds(items_whole, A), _rounds(items_comp, A), _rounds(sorted(items_comp, reverse=True), A), best,
            _rounds(items_b, A), rounds_global, _rounds(sorted(items_whole, reverse=True), A),
            max(items_comp, default=0) if len(items_comp) <= A else rounds_global,  # today's N <= 3 rule
            max(items_comp, default=0) if len(items_comp) <= A else _rounds(sorted(items_whole, reverse=True), A),
            _rounds(sorted([x for c in comps_per_env if c for x in (c if sum(c) > spill_k else [sum(c)])
                            for _ in (0, 1)], reverse=True), A))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=5)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--every", type=int, default=5, help="strategy statistics every this many steps")
    ap.add_argument("--lds-slots", type=int, default=None, help="records past this count spill (default: library)")
    a = ap.parse_args()
    n, B = a.players, a.envs
    ora = O.V1Vec(B, N=n, seed=0, portable=True)
    ora.reset()
    arr = np.ctypeslib.as_array(ora.envs)
    P = (2 * n + 1) * 12 + (2 * n + 1) * (2 * n) // 2
    rng = np.random.default_rng(1234)
    W = B // 64
    whole_w, comp_w, items_w, spill_w = [], [], [], []
    strat = {"whole": [], "comp": [], "comp_sort": [], "split": [], "comp_bucket4": [], "whole_globalm": [],
             "whole_sorted": [], "n23_today": [], "n23_fallback_sorted": [], "spill_envs_split_sorted": []}
    K = a.lds_slots if a.lds_slots is not None else 4
    for t in range(a.steps):
        ora.step(rng.integers(0, 5, (B, 2 * n), dtype=np.int32), nthreads=a.threads)
        inl = arr["arb_inlist"][:, :P].astype(np.int64)
        rec, big, nc, percomp = components(inl, n)
        whole_w.append(rec.reshape(W, 64).max(1))
        comp_w.append(big.reshape(W, 64).max(1))
        items_w.append(nc.reshape(W, 64).sum(1))
        if t % a.every == 0:
            rows = []
            for w in range(W):
                pc_ = percomp[64 * w:64 * w + 64]
                rows.append(strategies([list(x[x > 0]) for x in pc_], spill_k=K))
            for k_, v_ in zip(("whole", "comp", "comp_sort", "split", "comp_bucket4", "whole_globalm", "whole_sorted",
                               "n23_today", "n23_fallback_sorted", "spill_envs_split_sorted"),
                              np.array(rows).T):
                strat[k_].append(v_)
        if a.lds_slots is not None:
            spill_w.append((rec > a.lds_slots).reshape(W, 64).any(1))
    whole_w, comp_w, items_w = np.stack(whole_w), np.stack(comp_w), np.stack(items_w)
    # the launch's slowest wave per step (the step time is the max over waves)
    res = {"N": n, "envs": B, "steps": a.steps,
           "launch_max_whole_records_mean": float(whole_w.max(1).mean()),
           "launch_max_component_records_mean": float(comp_w.max(1).mean()),
           "wave_max_whole_records_mean": float(whole_w.mean()),
           "wave_max_component_records_mean": float(comp_w.mean()),
           "wave_items_mean": float(items_w.mean()), "wave_items_p99": float(np.percentile(items_w, 99)),
           "wave_items_max": int(items_w.max())}
    for k_, v_ in strat.items():
        v_ = np.stack(v_)
        res["strategy_%s_launch_max_mean" % k_] = float(v_.max(1).mean())
        res["strategy_%s_wave_mean" % k_] = float(v_.mean())
    if spill_w:
        res["waves_with_spill_frac"] = float(np.stack(spill_w).mean())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
