"""Summarise a gpurun_out/<dir> of bench / stamps logs (CPU-side helper)."""
import json, sys, os, glob
d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "bench*.log"))):
    for l in open(f):
        if l.startswith("{"):
            j = json.loads(l)
            print("%-12s %.3f G env-steps/s  kernel %.2f us  frac %.3f" % (os.path.basename(f), j["value"] / 1e9,
                  j["roofline"]["kernel_ms"] * 1e3, j["roofline"]["frac"]))
p = os.path.join(d, "stamps.log")
if os.path.exists(p):
    s = open(p).read(); j = json.loads(s[s.index("{"):])
    print("stamps mean total %.0f" % j["cycles_per_wave_step_total"])
    for k, v in j["phases"].items():
        print("  %-40s %8.0f %5.3f   slowest %8.0f" % (k, v["cycles"], v["share"], j["slowest_wave_phases"][k]))
    print("  records mean %.2f slowest %.2f" % (j["solver_records_per_wave_step"], j["slowest_wave_records"]))
    print("  ", {k: round(v, 1) for k, v in j["snapshot_mean"].items()})
