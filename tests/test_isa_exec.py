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
