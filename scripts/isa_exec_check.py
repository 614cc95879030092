"""Static check of the built gfx950 code objects for one miscompilation pattern (DESIGN.md section 6,
"compiler"): register copies placed at the start of a join block BEFORE its exec-mask restore.

A divergent `if` is lowered to `s_and_saveexec_b64 sX, ...` / `s_cbranch_execz JOIN` / body / `JOIN:
s_or_b64 exec, exec, sX`.  Any vector instruction between the JOIN label and the restore executes with
the body's lanes only -- with NO lane when the execz branch was taken.  A register-allocator copy of
a value that is live in every lane (a live-range split: `v_accvgpr_write aN, vM`, `v_mov`, a scratch
spill) placed there leaves the destination stale in the other lanes, and whatever later reads it back
gets garbage.  Found in round 4 in the N = 9 step instances built with max-memory-clause scheduling
and 8 preloaded cache entries: the per-lane address of an arbiter-cache array copied into a144:a145
at the join of the invalid-action atomic's `if`, and read back 1 600 instructions later.

usage: python scripts/isa_exec_check.py <object.o | code-object.elf> ...   (exit 1 on findings)
       check_object(path) -> [(kernel, join_address, [instructions])]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
COPY = re.compile(r"(v_accvgpr_write|v_accvgpr_read|v_accvgpr_mov|v_mov_b32|v_mov_b64|scratch_store|scratch_load|"
                  r"buffer_store|buffer_load)")
RESTORE = re.compile(r"s_or_b64 exec, exec, s\[\d+:\d+\]")
LINE = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):")
FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:")


def code_objects(path, tmp, arch="gfx950"):
    """the `arch` code object(s) of a HIP object file (its .hip_fatbin bundle, unbundled into the
    directory tmp), or the path itself if it is already an AMDGPU ELF."""
    out = subprocess.run([LLVM + "/llvm-readelf", "-h", path], capture_output=True, text=True).stdout
    if "AMDGPU" in out:
        return [path]
    secs = subprocess.run([LLVM + "/llvm-readelf", "-S", path], capture_output=True, text=True).stdout
    if ".hip_fatbin" not in secs:
        return []  # host code only
    fb = os.path.join(tmp, "fatbin")
    subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, path, os.path.join(tmp, "x.o")],
                   check=True, capture_output=True)
    co = os.path.join(tmp, arch + ".elf")
    subprocess.run([LLVM + "/clang-offload-bundler", "--type=o", "--input=" + fb,
                    "--targets=hipv4-amdgcn-amd-amdhsa--" + arch, "--output=" + co, "--unbundle"],
                   check=True, capture_output=True)
    return [co]


def disassemble(path, arch="gfx950"):
    """llvm-objdump -d listing(s) of the code object(s) of `path`"""
    with tempfile.TemporaryDirectory(prefix="isa_") as tmp:
        return [subprocess.run([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                               text=True, check=True).stdout for co in code_objects(path, tmp, arch)]


def long_branch(ins, i):
    """A relaxed long branch ending at ins[i] (past the SOPP branches' 16-bit range, big kernels):
    s_getpc_b64 s[x:x+1]; s_add_u32 sx, sx, lo; s_addc_u32 sx+1, sx+1, hi; s_setpc_b64 s[x:x+1] jumps to
    (address of s_getpc) + 4 + (hi:lo).  ins: [(address, text)].  Returns (target, relaxed_execz): the
    second is True when the sequence is the taken side of a relaxed s_cbranch_execz (an s_cbranch_execnz
    right before it skips over it).  None when ins[i] is not such a sequence."""
    m = re.match(r"^s_setpc_b64 s\[(\d+):(\d+)\]$", ins[i][1])
    if not m or i < 3:
        return None
    x = int(m.group(1))
    (ga, gt), ad, ac = ins[i - 3], ins[i - 2][1], ins[i - 1][1]
    ma = re.match(r"^s_add_u32 s(\d+), s(\d+), (0x[0-9a-f]+|-?\d+)$", ad)
    mc = re.match(r"^s_addc_u32 s(\d+), s(\d+), (0x[0-9a-f]+|-?\d+)$", ac)
    if gt != "s_getpc_b64 s[%d:%d]" % (x, x + 1) or not (ma and mc):
        return None
    if not (int(ma.group(1)) == x == int(ma.group(2)) and int(mc.group(1)) == x + 1 == int(mc.group(2))):
        return None
    off = ((int(mc.group(3), 0) & 0xffffffff) << 32) | (int(ma.group(3), 0) & 0xffffffff)
    if off >= 1 << 63:
        off -= 1 << 64
    execz = False
    if i >= 4 and ins[i - 4][1].startswith("s_cbranch_execnz"):
        o = int(ins[i - 4][1].split()[1])
        execz = ins[i - 4][0] + 4 + 4 * (o - 65536 if o >= 32768 else o) == ins[i][0] + 4
    return ga + 4 + off, execz


def scan(disasm):
    """findings of one llvm-objdump -d listing"""
    cur = None
    ins = []  # (addr, kernel, text)
    for ln in disasm.splitlines():
        m = FUNC.match(ln)
        if m:
            cur = m.group(2)
            continue
        m = LINE.match(ln)
        if m and cur:
            ins.append((int(m.group(2), 16), cur, m.group(1)))
    index = {a: i for i, (a, _, _) in enumerate(ins)}
    starts, execz = set(), set()
    pairs = [(a, re.sub(r"\s+", " ", t)) for a, _, t in ins]
    for i, (a, k, t) in enumerate(ins):
        if t.startswith("s_setpc_b64"):
            # a relaxed long branch: a block start, and the join of a skipped branch when it is the taken
            # side of a relaxed s_cbranch_execz (kernels past 128 KB of code: N >= 8)
            lb = long_branch(pairs, i)
            if lb is not None:
                starts.add(lb[0])
                if lb[1]:
                    execz.add(lb[0])
            continue
        if t.startswith(("s_cbranch", "s_branch")):
            # SOPP branch: target = address + 4 + 4 * simm16
            off = int(t.split()[1])
            tgt = a + 4 + 4 * (off - 65536 if off >= 32768 else off)
            starts.add(tgt)
            if t.startswith("s_cbranch_execz"):
                execz.add(tgt)
    found = []
    # blocks entered with a possibly partial / empty exec mask: execz-branch targets (the join of a
    # skipped branch) and the fallthrough of a loop's backward s_cbranch_execnz (the loop exit: every
    # lane has left the loop, exec = 0 until the exit's restore)
    for a, k, t in ins:
        if t.startswith("s_cbranch_execnz"):
            off = int(t.split()[1])
            if off >= 32768:  # backward branch: a loop
                execz.add(a + 4)
                starts.add(a + 4)
    for tgt in sorted(execz):
        i = index.get(tgt)
        if i is None:
            continue
        pre = []
        for a, k, t in ins[i:i + 64]:
            if a != tgt and a in starts:
                break
            if RESTORE.match(t):
                c = [p for p in pre if COPY.match(p)]
                if c:
                    found.append((k, hex(tgt), c))
                break
            dst = t.split(",")[0]
            if "exec" in dst or "saveexec" in t or t.startswith(("s_cbranch", "s_branch", "s_endpgm")):
                break
            pre.append(re.sub(r"\s+", " ", t))
    return found


def check_object(path, arch="gfx950"):
    found = []
    for dis in disassemble(path, arch):
        found += scan(dis)
    return found


if __name__ == "__main__":
    bad = 0
    for p in sys.argv[1:]:
        f = check_object(p)
        print("%-40s %d finding(s)" % (os.path.basename(p), len(f)))
        for k, a, c in f:
            print("   %s @ %s: %s" % (k[:70], a, "; ".join(c[:4])))
        bad += len(f)
    sys.exit(1 if bad else 0)
