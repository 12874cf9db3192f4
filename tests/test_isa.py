"""Static checks of the built gfx950 code (CPU): no SCC value the compiler keeps live across the
sort networks' compare-exchange asm (the missing-clobber bug that sorted some key sets with an
inverted network stage), and the DPP / permlane-swap wait states (scripts/check_isa.py)."""
import glob
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import check_isa  # noqa: E402

OBJS = sorted(glob.glob(os.path.join(ROOT, "br-archive_amd", "build", "*.o")))


@pytest.mark.skipif(not OBJS, reason="library not built (python __graft_entry__.py)")
@pytest.mark.parametrize("obj", OBJS, ids=[os.path.basename(p) for p in OBJS])
def test_machine_code_checks(obj):
    findings = check_isa.check(obj)
    assert not findings, "\n".join(findings[:10])


def test_checker_flags_a_live_scc_across_the_xnor(tmp_path):
    """The checker itself: an s_cselect fed by the compare-exchange string's xnor is reported."""
    s = tmp_path / "k.s"
    s.write_text("k:\n\ts_cmp_eq_u32 s4, 0\n\t;;#ASMSTART\n\tv_sub_co_u32 v0, vcc, v1, v2\n\ts_xnor_b64 vcc, vcc, s[6:7]\n"
                 "\tv_cndmask_b32 v1, v1, v2, vcc\n\t;;#ASMEND\n\ts_cselect_b32 s8, s9, 0xaaaaaaaa\n\ts_endpgm\n")
    assert len(check_isa.check(str(s))) == 1
