"""Build the MI355X (gfx950) kernels + C ABI into gym_futbol_amd/libfutbol_amd.so.

    python gym-futbol_amd/build.py [--force] [-j N]

Each csrc/*.hip translation unit is compiled by hipcc in parallel (one TU per
team size for the envs_v1 kernels), then linked into one shared library that
exports exactly the C ABI of include/futbol.h.  -ffp-contract=off: the env
math must round exactly like the reference's (no FMA contraction).
"""
import argparse
import glob
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# A/B experiments: FUTBOL_CSRC=<other source tree> FUTBOL_BUILD_VARIANT=<name> builds
# gym_futbol_amd/libfutbol_amd_<name>.so, loaded with FUTBOL_LIB_VARIANT=<name>
CSRC = os.environ.get("FUTBOL_CSRC", os.path.join(HERE, "csrc"))
VARIANT = os.environ.get("FUTBOL_BUILD_VARIANT", "")  # "stamps": diagnostic build with -DFUTBOL_STAMPS
OBJ = os.path.join(HERE, "build", "obj" + ("_" + VARIANT if VARIANT else ""))
LIB = os.path.join(HERE, "gym_futbol_amd", "libfutbol_amd%s.so" % ("_" + VARIANT if VARIANT else ""))
ARCH = os.environ.get("FUTBOL_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
          "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include")]
# SimplifyCFG folds an if/else whose arms cost up to this many instructions into selects: the
# default (4) leaves the fp64 arms of the action / contact code as divergent branches (~40 cycles
# each on a wave64); 20 measured best for the 2v2 step (-1.5% step time).  Only for the N <= 3
# instances: the 5v5 float instance built this way (~500 VGPRs, spills) corrupted its step
# counter on the GPU (tests/test_gpu_api.py episode lengths), so N >= 5 keeps the default.
PHI = os.environ.get("FUTBOL_PHI_FOLD", "20")
PHI_SOURCES = {"futbol_v1_n1_e64.hip": PHI, "futbol_v1_n2_e64.hip": PHI, "futbol_v1_n3_e64.hip": PHI,
               "futbol_v0.hip": os.environ.get("FUTBOL_PHI_FOLD_V0", "50")}  # v0: 50 measured best (-1.9%)
# diagnostic variants: FUTBOL_PHI_EXTRA="futbol_v1_n5_e64.hip ..." builds those TUs with the threshold too
for _src in os.environ.get("FUTBOL_PHI_EXTRA", "").split():
    PHI_SOURCES[_src] = PHI


def _phi_flags(src):
    t = PHI_SOURCES.get(os.path.basename(src))
    return [] if t is None else ["-mllvm", "-two-entry-phi-node-folding-threshold=" + t,
                                 "-mllvm", "-phi-node-folding-threshold=" + t]


# Machine scheduler of the envs_v1 step kernels: "max-memory-clause" measured 2v2 21.62 -> 21.48 us,
# 5v5 51.25 -> 50.5 us against LLVM's default (max-occupancy; the kernels run at one wave per SIMD
# either way), bit-identical results; the v0 kernel was neutral and keeps the default.
SCHED = os.environ.get("FUTBOL_SCHED", "max-memory-clause")


# Only the instances without scratch spills (N <= 5): the N = 9 double-output step instance
# (512 VGPRs, ~300 spilled VGPRs, 1.3 KB of scratch per lane) computed wrong velocities on the GPU
# with this strategy and right ones with LLVM's default scheduler or at -O1, from the same source
# (round 3, scripts/diag_n9.py; -verify-machineinstrs reports nothing) -- a code-generation fault
# at the register limit, like the phi-folding one of round 2 ("compiler").
# N = 3 is left out too: its rollout instances (f32 default field, f64 runtime geometry) diverged from
# the oracle at step 19 of tests/test_gpu_instances.py with this strategy and the phi-folding
# threshold together (either one alone: correct)
SCHED_SOURCES = {"futbol_v1_n%d_e64.hip" % n for n in (1, 2, 4, 5)}


# extra flags for the large instances (N = 6..10: 512 VGPRs with spills), e.g. FUTBOL_BIG_FLAGS=-O1
BIG_SOURCES = {"futbol_v1_n%d_e64.hip" % n for n in (6, 7, 8, 9, 10)}
BIG_FLAGS = os.environ.get("FUTBOL_BIG_FLAGS", "").split()


def _big_flags(src):
    return BIG_FLAGS if os.path.basename(src) in BIG_SOURCES else []


# diagnostic variants: extra flags for single TUs, FUTBOL_TU_FLAGS="<tu.hip>:<flags>;<tu.hip>:<flags>"
# (e.g. the round-3 failing configurations, scripts/gpu_fault_r04.sh)
TU_FLAGS = {}
for _ent in os.environ.get("FUTBOL_TU_FLAGS", "").split(";"):
    if ":" in _ent:
        _tu, _fl = _ent.split(":", 1)
        TU_FLAGS[_tu.strip()] = _fl.split()


def _tu_flags(src):
    return TU_FLAGS.get(os.path.basename(src), [])


def _sched_flags(src):
    b = os.path.basename(src)
    if not SCHED or b not in SCHED_SOURCES:
        return []
    return ["-mllvm", "-amdgpu-sched-strategy=" + SCHED]
# A/B of compiler options: FUTBOL_EXTRA_CFLAGS="..." (with a FUTBOL_BUILD_VARIANT name)
CFLAGS += os.environ.get("FUTBOL_EXTRA_CFLAGS", "").split()
# Diagnostic defines, selected explicitly: a variant named exactly "stamps" / "crumbs" / "bounds", or a
# "_"-separated word with a "+" prefix (e.g. FUTBOL_BUILD_VARIANT=kx6_+bounds), so that a plain word of an
# A/B variant's name (e.g. "no_stamps") never turns a diagnostic on
_DIAG_WORDS = ("stamps", "crumbs", "bounds")
_VWORDS = {VARIANT} & set(_DIAG_WORDS) | {w[1:] for w in VARIANT.split("_") if w.startswith("+")}
_unknown = _VWORDS - set(_DIAG_WORDS)
if _unknown:
    raise SystemExit("FUTBOL_BUILD_VARIANT=%s: unknown diagnostic word(s) %s" % (VARIANT, sorted(_unknown)))
if "stamps" in _VWORDS:
    CFLAGS.append("-DFUTBOL_STAMPS")
if "crumbs" in _VWORDS:  # diagnostic: per-wave phase markers in host-coherent memory
    CFLAGS.append("-DFUTBOL_CRUMBS")
if "bounds" in _VWORDS:  # diagnostic: index checks that flag and clamp instead of faulting
    CFLAGS.append("-DFUTBOL_BOUNDS")


def _deps():
    return (glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(CSRC, "*.h")) +
            [os.path.join(ROOT, "include", "futbol.h"), __file__])


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


# Code-generation gate ("compiler"): after compiling a TU, its code object is
# scanned for register copies placed before a join block's exec restore (scripts/isa_exec_check.py),
# the pattern behind round 3's wrong-result / illegal-address instances, and (round 5) for loaded or
# computed values that are only copied into registers nobody reads (scripts/isa_liveness.py), the
# pattern behind round 4's two wrong-result builds.  A TU with a finding is
# recompiled with the next of these register-allocation / scheduling variants (each changes where the
# allocator splits live ranges) until none is found; the build fails if every variant has findings.
# The variant used is recorded in the object's stamp.  FUTBOL_ISA_GATE=0 skips the gate.
# The first fallback switches LLVM's pre-RA exec-mask optimization (SIOptimizeExecMaskingPreRA) off: with
# it, the copies of the N = 7 segment-candidate loop's exit landed before the restore.  (Off for every TU,
# the kernels measured 1-2% slower: 2v2 22.66 vs 22.42 us, v0 22.92 vs 22.45 us, 5v5 52.8 vs 52.3 us.)
NO_PRE_RA = ["-mllvm", "-amdgpu-opt-exec-mask-pre-ra=false"]
GATE_VARIANTS = [[], NO_PRE_RA, ["-mllvm", "-split-spill-mode=size"], ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
                 NO_PRE_RA + ["-mllvm", "-split-spill-mode=size"], NO_PRE_RA + ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
                 ["-mllvm", "-split-spill-mode=size", "-mllvm", "-amdgpu-sched-strategy=max-ilp"]]
GATE = os.environ.get("FUTBOL_ISA_GATE", "1") != "0"
# the lane-aware liveness check (scripts/isa_liveness.py, round 5): FUTBOL_LIVENESS_GATE=0 skips it
LIVENESS_GATE = os.environ.get("FUTBOL_LIVENESS_GATE", "1") != "0"


def _isa_findings(obj):
    """both static checks of a compiled TU: register copies before an exec restore (isa_exec_check) and
    values that are only copied to registers nobody reads (isa_liveness: lane-aware liveness, run in a
    child process so that the TUs' checks run in parallel)"""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import isa_exec_check
    found = isa_exec_check.check_object(obj, ARCH)
    if LIVENESS_GATE:
        # --all: computed values as well as loaded ones (round 6: with relaxed long branches in the CFG the
        # shipped objects have no finding of either kind, so both gate)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "isa_liveness.py"), "--json", "--all",
                            "--arch=" + ARCH, obj], capture_output=True, text=True)
        if r.returncode not in (0, 1):
            raise RuntimeError("isa_liveness failed on %s:\n%s" % (obj, r.stderr[-4000:]))
        for ln in r.stdout.splitlines():
            found += [(k, a, ["lost value: " + t]) for k, a, t in json.loads(ln)["findings"]]
    return found


def _compile(src, force):
    """One TU.  Its full command line is stamped next to the object (<obj>.cmd): a build with other
    flags (the env-var knobs above) recompiles instead of reusing an object built differently."""
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    base = [HIPCC] + CFLAGS + _phi_flags(src) + _sched_flags(src) + _big_flags(src) + _tu_flags(src)
    stamp = obj + ".cmd"
    try:
        with open(stamp) as f:
            same = f.read().split("\n#gate")[0] == "\n".join(base)
    except OSError:
        same = False
    if not (force or not same or _stale(obj, [src] + _deps())):
        return obj
    log = []
    for k, extra in enumerate(GATE_VARIANTS if GATE else [[]]):
        cmd = base + extra + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr[-8000:]))
        found = _isa_findings(obj) if GATE else []
        log.append("%s: %d finding(s)%s" % (" ".join(extra) or "default", len(found),
                                            "".join("\n#   %s @ %s: %s" % (f[0][:60], f[1], "; ".join(f[2][:3]))
                                                    for f in found[:4])))
        if not found:
            with open(stamp, "w") as f:
                f.write("\n".join(base) + "\n#gate variant %d: %s\n#" % (k, " ".join(extra) or "default") +
                        "\n#".join(log))
            if k:
                print("isa gate: %s built with %s" % (os.path.basename(src), " ".join(extra)), flush=True)
            return obj
    os.remove(obj)
    raise RuntimeError("isa gate: every variant of %s has code-generation findings:\n%s"
                       % (src, "\n".join(log)))


# A/B variants of a few TUs: FUTBOL_VARIANT_TUS="futbol_v1_n2_e64.hip futbol_v1_n5_e64.hip" compiles only
# those with the variant's flags and links the product's objects (build/obj) for the others
VARIANT_TUS = set(os.environ.get("FUTBOL_VARIANT_TUS", "").split())
PRODUCT_OBJ = os.path.join(HERE, "build", "obj")


def build(force=False, jobs=None, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    jobs = jobs or min(8, os.cpu_count() or 4)

    def one(src):
        if VARIANT and VARIANT_TUS and os.path.basename(src) not in VARIANT_TUS:
            obj = os.path.join(PRODUCT_OBJ, os.path.basename(src) + ".o")
            if not os.path.exists(obj):
                raise RuntimeError("FUTBOL_VARIANT_TUS: build the product first (%s missing)" % obj)
            # the product object must be current with the product sources, or the A/B would link stale code
            psrc = os.path.join(HERE, "csrc", os.path.basename(src))
            pdeps = (glob.glob(os.path.join(HERE, "csrc", "*.hpp")) + glob.glob(os.path.join(HERE, "csrc", "*.h")) +
                     [os.path.join(ROOT, "include", "futbol.h")])
            if _stale(obj, [psrc] + pdeps):
                raise RuntimeError("FUTBOL_VARIANT_TUS: %s is older than the product sources; rebuild the product" % obj)
            return obj
        return _compile(src, force)
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(one, srcs))
    if force or _stale(LIB, objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s" % r.stderr[-8000:])
        if verbose:
            print("built", LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    try:
        build(a.force, a.j)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
