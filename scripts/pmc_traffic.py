"""Turn the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_profile.sh into
HBM bytes per launch of the env-step kernel, corrected with the calibration
kernels of scripts/pmc_calib.hip (profiled in the same passes), and append the
entry to profiles/<round>/traffic.json, which bench.py reports as roofline.traffic.

    python scripts/pmc_traffic.py --prof gpurun_out/prof --round r01 [--kind v1 --players 2 --envs 65536]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Correction (MI355X_MICROARCH.md,
HBM section): divide each counter by the ratio counter/true-bytes measured on
the calibration kernel with the same access width -- 8 B/lane loads for the
SoA fp64 state reads, 8 B/lane stores for the state writes (the obs / done
stores are calibrated too and reported, see "calibration").
"""
import argparse
import csv
import json
import os
import statistics


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def find(d, key):
    hits = [k for k in d if key in k]
    if len(hits) != 1:
        raise KeyError("%s: %d matching kernels in %s" % (key, len(hits), list(d)[:8]))
    return statistics.mean(d[hits[0]]), hits[0], len(d[hits[0]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prof", default="gpurun_out/prof")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--kind", default="v1")
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--calib-bytes", type=int, default=512 << 20)
    a = ap.parse_args()
    fetch = per_kernel(os.path.join(a.prof, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.prof, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    cfetch = per_kernel(os.path.join(a.prof, "calib_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    cwrite = per_kernel(os.path.join(a.prof, "calib_write", "run_counter_collection.csv"), "WRITE_SIZE")
    nb = a.calib_bytes
    calib = {
        "rd_f64_fetch_ratio": find(cfetch, "rd_f64(")[0] / nb,
        "wr_f64_write_ratio": find(cwrite, "wr_f64(")[0] / nb,
        "wr_aos20_write_ratio": find(cwrite, "wr_aos20")[0] / (nb // 80 * 80),
        "wr_u8_write_ratio": find(cwrite, "wr_u8")[0] / nb,
    }
    try:  # 16 B/lane (the envs_v1 body state since round 3: (x, y) pairs)
        calib["rd_f64x2_fetch_ratio"] = find(cfetch, "rd_f64x2(")[0] / nb
        calib["wr_f64x2_write_ratio"] = find(cwrite, "wr_f64x2(")[0] / nb
    except Exception:
        pass
    key = ("v1_step_kernel<%d," % a.players) if a.kind == "v1" else "v0_step_kernel"
    f, kname, nf = find(fetch, key)
    w, _, nw = find(write, key)
    # the dominant access width: 16 B/lane (the envs_v1 body pairs, the v0 row pairs)
    wide = "rd_f64x2_fetch_ratio" in calib  # every state array since round 3 (v1 bodies, v0 rows)
    rd = f / calib["rd_f64x2_fetch_ratio" if wide else "rd_f64_fetch_ratio"]
    wr = w / calib["wr_f64x2_write_ratio" if wide else "wr_f64_write_ratio"]
    entry = {"kind": a.kind, "players": a.players, "envs": a.envs, "kernel": kname,
             "launches": [nf, nw], "fetch_size_bytes_raw": f, "write_size_bytes_raw": w,
             "calibration": calib, "read_bytes_corrected": rd, "write_bytes_corrected": wr,
             "hbm_bytes_per_launch": rd + wr}
    out = os.path.join("profiles", a.round, "traffic.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    entries = []
    if os.path.exists(out):
        entries = [e for e in json.load(open(out))
                   if not (e["kind"] == a.kind and e.get("players") == a.players and e["envs"] == a.envs)]
    entries.append(entry)
    json.dump(entries, open(out, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
