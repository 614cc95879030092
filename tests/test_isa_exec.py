"""Static check of the shipped gfx950 code ("compiler"): no register copy or spill
placed at the start of a divergent branch's join block BEFORE the exec restore, where it runs with the
branch's lanes only (none, when the branch was skipped) and leaves stale values for the other lanes.
That pattern was the cause of round 3's wrong-result / illegal-address instances
(scripts/isa_exec_check.py).  Scans the objects the library was linked from (CPU only: llvm-objdump)."""
import glob
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
OBJS = sorted(glob.glob(os.path.join(ROOT, "gym-futbol_amd", "build", "obj", "futbol_*.hip.o")))


@pytest.mark.skipif(not OBJS or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="no built objects / ROCm LLVM tools")
def test_no_copies_before_exec_restore():
    import isa_exec_check as I
    found = []
    for o in OBJS:
        found += [(os.path.basename(o),) + f for f in I.check_object(o)]
    assert not found, "\n".join("%s %s @ %s: %s" % (o, k[:60], a, "; ".join(c[:3])) for o, k, a, c in found)


def test_checker_finds_the_pattern():
    """The checker itself, on a hand-written listing of the round-4 finding (join of the atomic's
    one-lane `if`, an AGPR copy before `s_or_b64 exec, exec`)."""
    import isa_exec_check as I
    dis = "\n".join([
        "0000000000001000 <_Z1kv>:",
        "\ts_and_saveexec_b64 s[4:5], vcc   // 000000001000: BE84206A",
        "\ts_cbranch_execz 2                 // 000000001004: BF880002",
        "\tv_mov_b64_e32 v[4:5], s[2:3]      // 000000001008: 7E087002",
        "\tglobal_atomic_add_x2 v2, v[4:5], s[2:3]   // 00000000100C: DD888000",
        "\tv_accvgpr_write_b32 a144, v232    // 000000001010: D3D94090",
        "\ts_or_b64 exec, exec, s[0:1]       // 000000001014: 87FE007E",
        "\ts_endpgm                          // 000000001018: BF810000",
    ])
    f = I.scan(dis)
    assert len(f) == 1 and f[0][1] == hex(0x1010) and "a144" in f[0][2][0]
    clean = dis.replace("\tv_accvgpr_write_b32 a144, v232    // 000000001010: D3D94090\n", "")
    assert I.scan(clean) == []


# ---- round 5: lane-aware liveness (scripts/isa_liveness.py), the second gate check
def _kernel(lines, base=0x1000):
    """a hand-written llvm-objdump listing: one kernel, 4-byte instructions from `base`"""
    out = ["%016x <_Z1kv>:" % base]
    for k, t in enumerate(lines):
        out.append("\t%-40s // %012X: 00000000" % (t, base + 4 * k))
    return "\n".join(out)


@pytest.mark.skipif(not OBJS or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="no built objects / ROCm LLVM tools")
def test_no_lost_loads_in_shipped_objects():
    """No loaded or computed value of the shipped kernels is only copied into registers nobody reads (the
    round-4 kx6 / latec / N = 6 faults).  One child process per object, as the build
    gate runs it (--all: computed values too, since round 6)."""
    import json
    import subprocess
    from concurrent.futures import ThreadPoolExecutor
    tool = os.path.join(ROOT, "scripts", "isa_liveness.py")

    def one(o):
        r = subprocess.run([sys.executable, tool, "--json", "--all", o], capture_output=True, text=True)
        assert r.returncode in (0, 1), r.stderr[-2000:]
        return [(os.path.basename(o),) + tuple(f) for f in json.loads(r.stdout.splitlines()[0])["findings"]]
    with ThreadPoolExecutor(min(8, os.cpu_count() or 4)) as ex:
        found = [f for fs in ex.map(one, [o for o in OBJS if "_v1_n" in o or "_v0" in o]) for f in fs]
    assert not found, "\n".join("%s %s @ %s: %s" % (o, k[:60], a, t) for o, k, a, t in found)


def test_liveness_finds_a_lost_load_component():
    """The kx6 fault in miniature: a 16-byte load staged into a[0:3] for a ds_write_b128, but its second
    dword copied into a5 (never read) -- a1 keeps its old value.  The correct listing passes."""
    import isa_liveness as L
    good = ["global_load_dwordx4 v[0:3], v10, s[0:1]", "s_waitcnt vmcnt(0)",
            "v_accvgpr_write_b32 a0, v0", "v_accvgpr_write_b32 a1, v1", "v_accvgpr_write_b32 a2, v2",
            "v_accvgpr_write_b32 a3, v3", "ds_write_b128 v10, a[0:3] offset:18432", "s_endpgm"]
    assert L.scan(_kernel(good)) == []
    bad = list(good)
    bad[3] = "v_accvgpr_write_b32 a5, v1"
    f = L.scan(_kernel(bad))
    assert len(f) == 1 and f[0][1] == hex(0x1000) and f[0][2].endswith("[LcLL]"), f


def test_liveness_keeps_phi_values_of_both_branches():
    """An if / else whose arms write the same register (a phi): on the wave's linear code the ELSE arm
    runs after the THEN arm, but only for the other lanes -- the lane-parking edges keep the THEN arm's
    value live, so the loaded value it copies is not reported.  Without them it would be."""
    import isa_liveness as L
    lst = ["global_load_dwordx2 v[0:1], v10, s[0:1]", "s_waitcnt vmcnt(0)",
           "s_and_saveexec_b64 s[2:3], vcc", "s_xor_b64 s[2:3], exec, s[2:3]",
           "v_mov_b32_e32 v4, v0",                                   # THEN: x = lo
           "s_or_saveexec_b64 s[2:3], s[2:3]", "s_xor_b64 exec, exec, s[2:3]",
           "v_mov_b32_e32 v4, v1",                                   # ELSE: x = hi
           "s_or_b64 exec, exec, s[2:3]",
           "global_store_dword v[8:9], v4, off", "s_endpgm"]
    assert L.scan(_kernel(lst)) == []
    ins = L.parse(_kernel(lst))["_Z1kv"]
    strong, _, _, _ = L.liveness(ins, strong=True, lanes=False)
    assert not strong[0] & L._bit(("v", 0)), "the scalar CFG alone loses the THEN arm's value"


def test_exec_scanner_limits_are_measured():
    """Why the exec-restore scanner is not anchored on every restore: inside a divergent
    region, copies of values live through the region are normal (phi copies, spill traffic) -- a
    fallthrough join's split copy cannot be told from them in the listing.  Measured on the shipped
    2v2 object: ~3 000 such copies, so that anchoring cannot gate; the liveness
    check above is the second gate instead.  Here: the scanner still finds its pattern at an execz
    join, and a join reached by fallthrough is outside what it claims to check."""
    import isa_exec_check as I
    at_join = ["s_and_saveexec_b64 s[4:5], vcc", "s_cbranch_execz 1", "v_add_u32_e32 v1, v1, v2",
               "v_accvgpr_write_b32 a144, v232", "s_or_b64 exec, exec, s[4:5]", "s_endpgm"]
    assert len(I.scan(_kernel(at_join))) == 1
    fallthrough = [t for t in at_join if not t.startswith("s_cbranch")]
    assert I.scan(_kernel(fallthrough)) == []


def _long_jump(from_index, to_index, sreg=98, base=0x1000):
    """the four instructions of a relaxed long branch placed at index from_index (its s_getpc) to index
    to_index: s_getpc_b64; s_add_u32 lo; s_addc_u32 hi; s_setpc_b64 (LLVM's branch relaxation)"""
    off = (base + 4 * to_index) - (base + 4 * from_index + 4)
    lo, hi = off & 0xffffffff, (off >> 32) & 0xffffffff
    s = "s[%d:%d]" % (sreg, sreg + 1)
    return ["s_getpc_b64 " + s, "s_add_u32 s%d, s%d, 0x%x" % (sreg, sreg, lo),
            "s_addc_u32 s%d, s%d, %s" % (sreg + 1, sreg + 1, "-1" if hi == 0xffffffff else "0x%x" % hi),
            "s_setpc_b64 " + s]


def test_liveness_follows_relaxed_long_branches():
    """Round 6: kernels past 128 KB of code (N >= 8) leave a cold block at the end and return from it by a
    relaxed long branch (s_getpc / s_add / s_addc / s_setpc).  The liveness CFG follows it: a value computed
    in the cold block and used after the jump back is live.  Without that edge the N = 9 / 10 objects
    showed 33 / 14 "arithmetic copied and lost" results (the out-of-bounds restart's new positions) --
    false findings, since every leaf of that switch is bit-exact on the GPU (test_gpu_v1_parity.py
    test_out_of_bounds_every_pick)."""
    import isa_liveness as L
    # 0: branch to the cold block; 1-2: main body after the return point (index 1 uses a4)
    main = ["s_branch 3", "global_store_dword v[8:9], v4, off", "s_endpgm"]
    # 3..: cold block: computes v[2:3], copies to a4, jumps back to index 1
    cold = ["global_load_dwordx2 v[2:3], v10, s[0:1]", "s_waitcnt vmcnt(0)", "v_accvgpr_write_b32 a4, v2",
            "v_accvgpr_read_b32 v4, a4"]
    lst = main + cold + _long_jump(len(main) + len(cold), 1)
    assert L.scan(_kernel(lst)) == [], "the value reaches the store through the long branch"
    # without the jump back (the cold block ending the program) the same value is lost -- the finding the
    # long branch's edge removes (an undecodable s_setpc is a function return: everything live, no finding)
    broken = main + cold + ["s_endpgm"]
    assert len(L.scan(_kernel(broken))) == 1


def test_exec_scanner_checks_relaxed_execz_joins():
    """A relaxed s_cbranch_execz (s_cbranch_execnz over a long branch): the long branch's target is a join
    entered with exec = 0 when taken, so a copy placed there before the exec restore is the round-3 fault
    pattern -- the scanner must see it."""
    import isa_exec_check as I
    head = ["s_and_saveexec_b64 s[4:5], vcc", "s_cbranch_execnz 4"]
    jump_at = len(head)
    body = ["v_add_u32_e32 v1, v1, v2", "s_endpgm"]
    join = ["v_accvgpr_write_b32 a144, v232", "s_or_b64 exec, exec, s[4:5]", "s_endpgm"]
    join_at = jump_at + 4 + len(body)
    lst = head + _long_jump(jump_at, join_at) + body + join
    f = I.scan(_kernel(lst))
    assert len(f) == 1 and f[0][1] == hex(0x1000 + 4 * join_at), f
    assert I.scan(_kernel(lst[:join_at] + join[1:])) == []


def test_liveness_partial_use_of_computed_pairs():
    """--all judges computed values whole: a 64-bit shift whose high half is unused but moved with the pair
    (v_mov_b64) is not a finding, a computed pair lost entirely is -- and a load is judged per register."""
    import isa_liveness as L
    part = ["v_lshrrev_b64 v[6:7], v2, v[8:9]", "v_mov_b64_e32 v[10:11], v[6:7]",
            "global_store_dword v[20:21], v10, off", "s_endpgm"]
    assert L.scan(_kernel(part), loads_only=False) == []
    whole = ["v_add_f64 v[6:7], v[2:3], v[4:5]", "v_mov_b64_e32 v[10:11], v[6:7]", "s_endpgm"]
    f = L.scan(_kernel(whole), loads_only=False)
    assert len(f) == 1 and f[0][2].endswith("[cc]"), f
    load = ["global_load_dwordx2 v[6:7], v2, s[0:1]", "s_waitcnt vmcnt(0)", "v_mov_b64_e32 v[10:11], v[6:7]",
            "global_store_dword v[20:21], v10, off", "s_endpgm"]
    f = L.scan(_kernel(load))
    assert len(f) == 1 and f[0][2].endswith("[Lc]"), f


def test_liveness_models_calls_and_returns():
    """A device function's return (s_setpc_b64 of its return address, not a decodable long branch) leaves every
    register live -- its result in v[0:1] is not lost -- and a call (s_swappc_b64) reads the argument registers
    v0-v31, so the value the caller passes is not lost either (round 6: glibc_pow2_full_call)."""
    import isa_liveness as L
    callee = ["v_mul_f64 v[2:3], v[0:1], v[0:1]", "v_mov_b64_e32 v[0:1], v[2:3]", "s_setpc_b64 s[30:31]"]
    assert L.scan(_kernel(callee), loads_only=False) == []
    caller = ["global_load_dwordx2 v[6:7], v10, s[0:1]", "s_waitcnt vmcnt(0)", "v_mov_b64_e32 v[0:1], v[6:7]",
              "s_swappc_b64 s[30:31], s[16:17]", "global_store_dwordx2 v[20:21], v[0:1], off", "s_endpgm"]
    assert L.scan(_kernel(caller)) == []
