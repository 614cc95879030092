"""Summarise the bench lines of a gpu_steps.sh output directory (one log per step):
step name, env-steps/s (G), step-kernel µs, roofline fraction; pytest summary lines as they are.

  python scripts/bench_lines.py gpurun_out/c9
"""
import glob
import json
import os
import sys


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "*.log")), key=os.path.getmtime):
        name = os.path.basename(f)[:-4]
        for line in open(f, errors="replace"):
            if line.startswith("{"):
                try:
                    x = json.loads(line)
                except ValueError:
                    continue
                r = x.get("roofline") or {}
                if "value" in x and "kernel_ms" in r:
                    print("%-14s %8.4f G  %8.2f us  frac %.4f" % (name, x["value"] / 1e9, r["kernel_ms"] * 1e3,
                                                                r.get("frac", 0.0)))
            elif " passed" in line or " failed" in line or "error" in line.lower()[:40]:
                print("%-14s %s" % (name, line.strip()))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
