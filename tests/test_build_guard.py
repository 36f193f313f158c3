"""The build's guard against callable device functions whose long branches go through s[30:31], the
return address (safestakeoperator_amd/build.py long_branch_clobbers; DESIGN.md §4 "A toolchain
hazard"): the disassembly scanner on listings shaped like llvm-objdump's, and the built objects."""
import glob
import os

import pytest

from safestakeoperator_amd import build

LISTING = """
0000000000001000 <_ZN3ssb10rc_k_chainERNS_3jacINS_3fp2EEEPKhPKm>:
	s_waitcnt vmcnt(0) expcnt(0) lgkmcnt(0)                    // 000000001000: BF8C0000
	s_getpc_b64 s[30:31]                                       // 000000001004: BE9E1C00
	s_add_u32 s30, s30, 0x57b10                                // 000000001008: 801EFF1E 00057B10
	s_setpc_b64 s[30:31]                                       // 000000001010: BE801D1E
	s_setpc_b64 s[30:31]                                       // 000000001014: BE801D1E

0000000000002000 <_ZN3ssb7jac_dblINS_3fp2EEEvRNS_3jacIT_EERKS4_>:
	s_getpc_b64 s[16:17]                                       // 000000002000: BE901C00
	s_swappc_b64 s[30:31], s[16:17]                            // 000000002004: BE9E1E10
	s_setpc_b64 s[30:31]                                       // 000000002008: BE801D1E

0000000000003000 <_ZN3ssb1k14k_miller_finalEv>:
	s_getpc_b64 s[30:31]                                       // 000000003000: BE9E1C00
	s_setpc_b64 s[30:31]                                       // 000000003004: BE801D1E
"""


def test_scanner_flags_return_address_long_branches_only():
    got = build.scan_disassembly(LISTING.splitlines(True), {"_ZN3ssb1k14k_miller_finalEv"})
    # the callable function's long branch through s[30:31] is flagged; a call sequence (s_getpc on
    # another pair, s_swappc writing s[30:31]) and a kernel's s[30:31] are not
    assert got == {"_ZN3ssb10rc_k_chainERNS_3jacINS_3fp2EEEPKhPKm": 1}


def test_built_objects_have_no_return_address_long_branches():
    objs = sorted(glob.glob(os.path.join(build.OBJDIR, "*.o")))
    if not objs or not os.path.exists(os.path.join(build.LLVM, "llvm-objdump")):
        pytest.skip("no built objects / no llvm-objdump")
    assert build.long_branch_clobbers(objs) == {}
