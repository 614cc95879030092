"""Register liveness over a gfx950 kernel's ISA (llvm-objdump listing): a second static check of the
code objects next to scripts/isa_exec_check.py ("compiler").

It finds values that the register allocator moved around but that never reach a real use: a load
or an arithmetic result whose register is read only by copies (v_mov, v_accvgpr_*) whose own
destinations then die.  LLVM removes dead code before register allocation and only copies live values,
so such a value is the trace of a copy that went to the wrong register -- the register the later
instruction reads still holds an older value.  The round-4 "kx6" build (6 spill records in registers
for 5v5) is the case that motivated it: staging glibc's pow tables into LDS, the register allocator
assembled the 16-byte chunk a[222:225] from a scratch reload and AGPR copies, but copied the chunk's
second dword into a255 -- never read -- and left a223 holding the PREVIOUS chunk's second dword, so the
ds_write_b128 wrote a wrong high word into every lane's third kPowLog chunk (one 5v5 env in 96 got a
wrong glibc square at step 5; tests/test_gpu_instances.py).

The same check finds the round-4 "latec" build's fault (N = 10, three of four step instances diverged at
step 58): after the solve's v pass, the bodies' velocity rows are read back from LDS (ds_read_b128) and
seven of the 21 are only copied into AGPRs that are never read, so the stored velocities are stale.

Analysis: basic blocks and edges from the SOPP branches (s_branch / s_cbranch_* targets, fallthrough),
plus "lane parking" edges (exec_regions): where exec is narrowed (s_and_saveexec, an ELSE, a loop
latch's s_andn2 exec) the removed lanes resume where the saved mask is OR-ed / moved back into exec, so
their registers must survive the code in between -- without these edges, the ELSE block's writes
would look like kills of the THEN block's phi values.  Per-instruction defs / uses of v / a registers
(32-bit granularity, tuples v[a:b] expanded); liveness to a fixed point twice: plain, and "strong"
(faint variables: a copy's source is live only where its destination is).  Conservative where the
encoding is partial: DPP / SDWA / op_sel / d16 / v_writelane / MAC-style tied destinations count as
use + def.  The product build's objects have no finding; the kx6 and latec builds' failing objects do
(DESIGN.md section 6).

The gate (gym-futbol_amd/build.py) runs with `--all`: LOADED values (global / LDS loads; a scratch reload
is a copy) and computed ones.  A result that is only copied and lost cannot be dead code -- LLVM deletes
unused values before register allocation -- and all three round-4 wrong builds (kx6, latec, the N = 6
batched-squares build) are loads of this kind.  Relaxed long branches (s_getpc / s_add / s_addc /
s_setpc, emitted in kernels past 128 KB of code) are CFG edges (isa_exec_check.long_branch): until round
6 they were not, and the N = 9 / 10 objects showed 33 / 14 "arithmetic copied and lost" results -- the
out-of-bounds restart's new positions, computed in a cold block at the kernel's end that returns by a
long branch -- which were false findings (every leaf is bit-exact on the GPU,
tests/test_gpu_v1_parity.py test_out_of_bounds_every_pick); with the edges there are none, and computed
values gate too.

usage: python scripts/isa_liveness.py [--json] [--all] [--arch=gfx950] <object.o | code-object> ...   (exit 1 on findings)
       (without --all: loaded values only)
       check_object(path, arch) -> [(kernel, address, instruction [pattern])]
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_exec_check as X  # noqa: E402  (code-object extraction, disassembly)

LINE = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):")
FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:")
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?![0-9]))")
# instructions whose register operands are all read (no v / a destination)
NO_DEF = re.compile(r"^(global_store|flat_store|scratch_store|buffer_store|ds_write|ds_store|ds_add_u|ds_sub_u|"
                    r"ds_min|ds_max|ds_and_b|ds_or_b|ds_xor_b|ds_inc_u|ds_dec_u|ds_cmpst_b|ds_gws|exp |"
                    r"s_|v_cmp_|v_cmpx_|v_readlane|v_readfirstlane)")
# destination also read (tied / partial writes): use + def
TIED = re.compile(r"^(v_mac_|v_fmac_|v_pk_fmac|v_dot2c|v_writelane|v_mfma|v_smfmac|v_swap)")
PARTIAL = re.compile(r"(_sdwa\b|_dpp\b|\bop_sel:\[\d,\d,\d,1\]|d16)")
COPY = re.compile(r"^(v_mov_b32|v_mov_b64|v_accvgpr_write|v_accvgpr_read|v_accvgpr_mov|v_pk_mov_b32|scratch_load|"
                  r"buffer_load_dword\b)")


def regs(tok):
    out = []
    for m in REG.finditer(tok):
        k = m.group(1)
        if m.group(4) is not None:
            out.append((k, int(m.group(4))))
        else:
            out += [(k, i) for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    return out


def defs_uses(text):
    """(defs, uses) of v / a registers of one instruction"""
    mn = text.split()[0]
    rest = text[len(mn):].strip()
    ops = [o.strip() for o in rest.split(",")] if rest else []
    if mn.startswith("global_load_lds") or (mn.startswith("buffer_load") and re.search(r"\blds\b", rest)):
        return [], [r for o in ops for r in regs(o)]  # LDS-DMA: the data goes to LDS, no register written
    if NO_DEF.match(mn + " "):
        d = []
        u = [r for o in ops for r in regs(o)]
        if mn.startswith(("ds_", "global_atomic", "flat_atomic", "buffer_atomic")) and "rtn" in mn:
            d = regs(ops[0])
        return d, u
    if mn.startswith(("global_atomic", "flat_atomic", "buffer_atomic", "scratch_atomic")):
        # returning form (sc0 / glc): first operand is the destination
        if re.search(r"\b(sc0|glc)\b", rest):
            return regs(ops[0]), [r for o in ops[1:] for r in regs(o)]
        return [], [r for o in ops for r in regs(o)]
    if mn == "s_swappc_b64":
        # a call (a device function, e.g. glibc_pow2_full_call): its arguments are v0-v31 under the AMDGPU
        # calling convention; counted as read (conservative: nothing the caller passes looks lost)
        return [], [("v", r) for r in range(32)]
    if not ops:
        return [], []
    d = regs(ops[0])
    u = [r for o in ops[1:] for r in regs(o)]
    if TIED.match(mn) or PARTIAL.search(text):
        u = u + d
    return d, u


def parse(disasm):
    """{kernel: [(addr, text)]}"""
    fns, cur = {}, None
    for ln in disasm.splitlines():
        m = FUNC.match(ln)
        if m:
            cur = m.group(2)
            fns[cur] = []
            continue
        m = LINE.match(ln)
        if m and cur:
            fns[cur].append((int(m.group(2), 16), re.sub(r"\s+", " ", m.group(1))))
    return fns


SREG = re.compile(r"\bs(?:\[(\d+):(\d+)\]|(\d+)(?![0-9]))")
VOP3B = re.compile(r"^(v_\w+_co_\w+|v_div_scale|v_mad_u64_u32|v_mad_i64_i32|v_addc_|v_subb_|v_subbrev_)")


def _sregs(tok):
    out = []
    for m in SREG.finditer(tok):
        if m.group(3) is not None:
            out.append(int(m.group(3)))
        else:
            out += list(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _pair(tok):
    r = _sregs(tok)
    return tuple(r) if len(r) == 2 else None


def exec_regions(ins, succ):
    """Lane parking: where exec is narrowed, the removed lanes wait and resume where exec is widened
    again; on the scalar CFG of the listing that is an extra edge (park point -> resume point) -- the
    parked lanes' registers must survive whatever the wave executes in between (the other branch of an
    if / else, later loop iterations).  The saved masks are followed through s_mov, SGPR spill lanes
    (v_writelane / v_readlane) by a forward data-flow over the CFG; every mask gets the id of the
    instruction that created it.  Returns the extra edges [(i, j)]: after instruction i -> before j."""
    n = len(ins)
    preds = [[] for _ in range(n)]
    for i in range(n):
        for j in succ[i]:
            preds[j].append(i)
    # per point: {("s", reg) | ("l", vgpr, lane): (mask_id, half)}; None = not yet visited
    IN = [None] * n
    IN[0] = {}
    opens = {}   # mask id -> set of park points (instruction indices)
    resumes = []  # (resume instruction, mask id)
    work = [0]
    inq = {0}

    def transfer(i, st):
        t = ins[i][1]
        mn = t.split()[0]
        ops = [o.strip() for o in t[len(mn):].split(",")]
        st = dict(st)

        def get(pr):
            if pr is None:
                return None
            a, b = st.get(("s", pr[0])), st.get(("s", pr[1]))
            if a and b and a[0] == b[0] and a[1] == 0 and b[1] == 1:
                return a[0]
            return None

        def put(pr, mid):
            if pr is None:
                return
            for h, r in enumerate(pr):
                if mid is None:
                    st.pop(("s", r), None)
                else:
                    st[("s", r)] = (mid, h)
        if mn in ("s_and_saveexec_b64", "s_or_saveexec_b64", "s_andn2_saveexec_b64", "s_xor_saveexec_b64",
                  "s_orn2_saveexec_b64", "s_andn1_saveexec_b64"):
            d, src = _pair(ops[0]), _pair(ops[1]) if len(ops) > 1 else None
            if ops[1] == "-1":  # whole-wave mode: exec = all lanes
                put(d, None)
                return st
            old = get(src)
            if old is not None and mn != "s_and_saveexec_b64":  # ELSE: the parked lanes resume here
                resumes.append((i, old))
            put(d, i)
            opens.setdefault(i, set()).add(i)
            return st
        if mn == "s_xor_b64" and len(ops) == 3 and ops[1] == "exec" and _pair(ops[0]) is not None:
            put(_pair(ops[0]), get(_pair(ops[2])))  # the IF's mask complemented for its ELSE: same region
            return st
        if mn in ("s_or_b64", "s_mov_b64", "s_and_b64", "s_andn2_b64", "s_xor_b64") and ops[0] == "exec":
            src = _pair(ops[-1])
            mid = get(src)
            if mn in ("s_or_b64", "s_mov_b64", "s_xor_b64") and mid is not None:
                resumes.append((i, mid))   # END_CF / restore / ELSE of the older form
            elif mn == "s_andn2_b64" and mid is not None:
                opens.setdefault(mid, set()).add(i)  # loop latch: the lanes in the mask park here
            return st
        if mn == "s_mov_b64" and len(ops) == 2:
            d = _pair(ops[0])
            if ops[1] == "exec":
                put(d, i)
                opens.setdefault(i, set()).add(i)
            elif ops[1] == "0":
                put(d, i)   # a loop's break mask starts empty
                opens.setdefault(i, set()).add(i)
            else:
                put(d, get(_pair(ops[1])))
            return st
        if mn == "s_or_b64" and len(ops) == 3 and _pair(ops[0]) is not None and _pair(ops[0]) in (_pair(ops[1]), _pair(ops[2])):
            other = ops[1] if _pair(ops[0]) == _pair(ops[2]) else ops[2]
            mid = get(_pair(ops[0]))
            if mid is not None:  # a loop break accumulating lanes into the mask
                opens.setdefault(mid, set()).add(i)
                if other != "exec" and _pair(other) is not None:
                    pass
                return st
        if mn == "v_writelane_b32":
            r = _sregs(ops[1])
            v = regs(ops[0])
            if r and v:
                key = ("l", v[0], ops[2])
                val = st.get(("s", r[0]))
                if val is None:
                    st.pop(key, None)
                else:
                    st[key] = val
            return st
        if mn == "v_readlane_b32":
            r = _sregs(ops[0])
            v = regs(ops[1])
            if r and v:
                val = st.get(("l", v[0], ops[2]))
                if val is None:
                    st.pop(("s", r[0]), None)
                else:
                    st[("s", r[0])] = val
            return st
        if mn == "s_mov_b32" and len(ops) == 2:
            r, q = _sregs(ops[0]), _sregs(ops[1])
            if r:
                val = st.get(("s", q[0])) if q else None
                if val is None:
                    st.pop(("s", r[0]), None)
                else:
                    st[("s", r[0])] = val
            return st
        # any other SGPR write kills what it overwrites
        killed = []
        if ops and ops[0]:
            if not NO_DEF.match(mn + " ") or mn.startswith(("s_", "v_cmp", "v_readfirstlane")):
                killed += _sregs(ops[0])
        if VOP3B.match(mn) and len(ops) > 1:
            killed += _sregs(ops[1])
        if mn.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_setprio",
                          "s_sleep", "s_barrier", "s_endpgm", "s_store", "s_dcache", "s_trap")):
            killed = []
        for r in killed:
            st.pop(("s", r), None)
        return st
    OUT = [None] * n
    while work:
        i = work.pop()
        inq.discard(i)
        o = transfer(i, IN[i])
        if OUT[i] == o:
            continue
        OUT[i] = o
        for j in succ[i]:
            if IN[j] is None:
                nw = dict(o)
            else:
                nw = {k: v for k, v in IN[j].items() if o.get(k) == v}
            if nw != IN[j]:
                IN[j] = nw
                if j not in inq:
                    inq.add(j)
                    work.append(j)
    edges = set()
    for j, mid in resumes:
        for i in opens.get(mid, ()):
            if i != j:
                edges.add((i, j))
    return sorted(edges)


def long_branch_target(ins, i):
    """target address of the relaxed long branch ending at ins[i] (isa_exec_check.long_branch), or None"""
    lb = X.long_branch(ins, i)
    return None if lb is None else lb[0]


def _cfg(ins, lanes=True):
    n = len(ins)
    idx = {a: i for i, (a, _) in enumerate(ins)}
    succ = [[] for _ in range(n)]
    rets = set()
    for i, (a, t) in enumerate(ins):
        mn = t.split()[0]
        if mn == "s_setpc_b64":
            # a relaxed long branch (kernels past 128 KB of code): without this edge every value that
            # flows through one looks dead -- the source of the non-gating "arithmetic copied and lost"
            # findings of round 5 (N = 9 / 10: the out-of-bounds restart block sits at the end of the
            # kernel and returns to the main body by a long branch)
            tgt = long_branch_target(ins, i)
            if tgt is not None and tgt in idx:
                succ[i].append(idx[tgt])
            else:
                rets.add(i)  # a device function's return: every register counts as live out
            continue
        if mn.startswith(("s_branch", "s_cbranch")):
            off = int(t.split()[1])
            tgt = a + 4 + 4 * (off - 65536 if off >= 32768 else off)
            if tgt in idx:
                succ[i].append(idx[tgt])
            if mn.startswith("s_cbranch") and i + 1 < n:
                succ[i].append(i + 1)
        elif mn in ("s_endpgm", "s_trap"):
            pass
        elif i + 1 < n:
            succ[i].append(i + 1)
    if lanes:
        for i, j in exec_regions(ins, succ):
            if j not in succ[i]:
                succ[i].append(j)
    leader = [False] * n
    if n:
        leader[0] = True
    for i in range(n):
        if len(succ[i]) != 1 or succ[i][0] != i + 1:
            if i + 1 < n:
                leader[i + 1] = True
        for s in succ[i]:
            if s != i + 1:
                leader[s] = True
    starts = [i for i in range(n) if leader[i]]
    bend = {}
    for k, s in enumerate(starts):
        bend[s] = (starts[k + 1] if k + 1 < len(starts) else n) - 1
    _cfg.rets = {s for s in starts if bend[s] in rets}
    return starts, bend, {s: list(succ[bend[s]]) for s in starts}


def _bit(r):
    return 1 << ((0 if r[0] == "v" else 512) + r[1])


def liveness(ins, strong=False, lanes=True):
    """live-after bit sets per instruction.  strong: a copy's source is live only where the copy's
    destination is (faint-variable analysis: values that reach no real use through copies are dead)"""
    n = len(ins)
    starts, bend, bsucc = _cfg(ins, lanes)
    du = [defs_uses(t) for _, t in ins]
    dmask = [sum(_bit(r) for r in set(d)) for d, _ in du]
    umask = [sum(_bit(r) for r in set(u)) for _, u in du]
    iscopy = [bool(COPY.match(t)) and not t.startswith("scratch_load") and len(du[i][0]) == len(du[i][1]) and
              not (dmask[i] & umask[i]) for i, (_, t) in enumerate(ins)]
    pairs = [list(zip(du[i][0], du[i][1])) if iscopy[i] else None for i in range(n)]

    def step(i, live):
        if strong and iscopy[i]:
            add = 0
            for d, u in pairs[i]:
                if live & _bit(d):
                    add |= _bit(u)
            return (live & ~dmask[i]) | add
        return (live & ~dmask[i]) | umask[i]
    rets = _cfg.rets
    ALL = (1 << 1024) - 1
    live_in = {s: 0 for s in starts}
    changed = True
    while changed:
        changed = False
        for s in reversed(starts):
            live = ALL if s in rets else 0
            for t in bsucc[s]:
                live |= live_in[t]
            for i in range(bend[s], s - 1, -1):
                live = step(i, live)
            if live != live_in[s]:
                live_in[s] = live
                changed = True
    after = [0] * n
    for s in starts:
        live = ALL if s in rets else 0
        for t in bsucc[s]:
            live |= live_in[t]
        for i in range(bend[s], s - 1, -1):
            after[i] = live
            live = step(i, live)
    return after, dmask, umask, du


def dead_writes(ins):
    """indices of instructions all of whose v / a destinations are dead right after them (diagnostic)"""
    after, dmask, umask, _ = liveness(ins)
    return [i for i in range(len(ins)) if dmask[i] and not (dmask[i] & after[i]) and not (dmask[i] & umask[i])]


# results the check does not judge: copies themselves, SGPR-spill lane writes (the compiler's own
# save / restore machinery for SGPRs, read back with v_readlane)
NOT_PRODUCERS = re.compile(r"^(v_writelane|v_readlane|v_readfirstlane)")


LOADS = re.compile(r"^(global_load|flat_load|scratch_load|buffer_load|ds_read|ds_load)")


def suspects(ins, loads_only=True):
    """Instructions (not copies) with a destination register whose value reaches no real use -- only
    copies whose own destinations then die -- on the lane-aware CFG: [(index, pattern)], pattern one
    character per destination register: L = used, c = copied but lost, . = never read.  A loaded or
    computed value that the register allocator copied somewhere and then never used is the trace of a
    copy to the wrong register (the kx6 pow-table chunk, the latec solver rows)."""
    strong, _, _, du = liveness(ins, strong=True)
    weak, _, _, _ = liveness(ins)
    out = []
    for i, (_, t) in enumerate(ins):
        rs = du[i][0]
        if not rs or NOT_PRODUCERS.match(t):
            continue
        if loads_only:
            if not LOADS.match(t) or t.startswith("scratch_load"):
                continue
        elif COPY.match(t):
            continue
        live = [bool(strong[i] & _bit(r)) for r in rs]
        read = [bool(weak[i] & _bit(r)) for r in rs]
        lost = any((not l) and w for l, w in zip(live, read))
        if lost and not LOADS.match(t) and any(live):
            # a computed multi-register value whose used part is live: a 64-bit operation of which only one
            # half is needed (v_lshrrev_b64 for a 32-bit result) moved as a pair -- the other half's copy is
            # dead by construction, not a misplaced copy.  Loads are judged per register (the kx6 / N = 6
            # faults: one dword of a 16-byte load lost while the others are used)
            lost = False
        if lost:
            out.append((i, "".join("L" if l else ("c" if w else ".") for l, w in zip(live, read))))
    return out


def scan(disasm, loads_only=True):
    found = []
    for k, ins in parse(disasm).items():
        for i, pat in suspects(ins, loads_only):
            found.append((k, hex(ins[i][0]), "%s   [%s]" % (ins[i][1], pat)))
    return found


def check_object(path, arch="gfx950", loads_only=True):
    found = []
    for dis in X.disassemble(path, arch):
        found += scan(dis, loads_only)
    return found


if __name__ == "__main__":
    import json
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    arch = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--arch=")), "gfx950")
    bad = 0
    for p in args:
        f = check_object(p, arch, loads_only="--all" not in sys.argv)
        if "--json" in sys.argv:
            print(json.dumps({"object": p, "findings": f}))
        else:
            print("%-40s %d finding(s)" % (os.path.basename(p), len(f)))
            for k, a, t in f[:20]:
                print("   %s @ %s: %s" % (k[:70], a, t))
        bad += len(f)
    sys.exit(1 if bad else 0)
