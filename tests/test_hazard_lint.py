"""tools/hazard_lint.py on small assembly snippets (the build runs it on the compiled kernel)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import hazard_lint as H  # noqa: E402


def run(body):
    return H.lint(body.strip().splitlines())


def test_spill_restore_before_saddr_load_is_flagged():
    bad = run("""
        v_readlane_b32 s8, v59, 12
        v_readlane_b32 s9, v59, 13
        ;;#ASMSTART
        global_load_dword v13, v11, s[8:9]
        s_waitcnt vmcnt(0)
        ;;#ASMEND
    """)
    assert len(bad) == 1 and bad[0][5] == 0


def test_padding_or_salu_source_is_clean():
    assert not run("""
        v_readlane_b32 s9, v59, 13
        s_nop 4
        ;;#ASMSTART
        global_load_dword v13, v11, s[8:9]
        ;;#ASMEND
    """)
    assert not run("""
        s_add_u32 s8, s6, s2
        s_addc_u32 s9, s7, s3
        ;;#ASMSTART
        global_load_dword v13, v11, s[8:9]
        ;;#ASMEND
    """)


def test_lane_select_and_m0():
    assert run("""
        v_readfirstlane_b32 s8, v1
        ;;#ASMSTART
        v_readlane_b32 s0, v9, s8
        ;;#ASMEND
    """)
    assert not run("""
        s_lshl_b32 s8, s12, 8
        ;;#ASMSTART
        v_readlane_b32 s0, v9, s8
        ;;#ASMEND
    """)
    assert run("""
        s_add_i32 m0, s11, s10
        ;;#ASMSTART
        global_load_lds_dword v[6:7], off
        ;;#ASMEND
    """)
    assert not run("""
        s_add_i32 m0, s11, s10
        ;;#ASMSTART
        s_nop 0
        global_load_lds_dword v[6:7], off
        ;;#ASMEND
    """)


def test_branch_predecessor_is_checked():
    """a consumer at a branch target is checked against the writes on the branch's
    path too, not only the fall-through (here the fall-through is clean, the branch path is not)."""
    bad = run("""
        v_readfirstlane_b32 s8, v1
        s_cbranch_scc1 .LBB0_7
        s_add_u32 s8, s6, s2
        s_addc_u32 s9, s7, s3
    .LBB0_7:
        ;;#ASMSTART
        global_load_dword v13, v11, s[8:9]
        ;;#ASMEND
    """)
    assert len(bad) == 1 and bad[0][4] == "v_readfirstlane_b32"
    assert not run("""
        v_readfirstlane_b32 s8, v1
        s_nop 4
        s_cbranch_scc1 .LBB0_7
        s_add_u32 s8, s6, s2
    .LBB0_7:
        ;;#ASMSTART
        global_load_dword v13, v11, s[8:9]
        ;;#ASMEND
    """)


def test_asm_loop_back_edge_is_checked():
    """The walk loop's head ("1:") is also reached from its own back edge ("s_cbranch_scc0 1b")."""
    bad = run("""
        s_mov_b32 s8, 0
        ;;#ASMSTART
    1:
        v_readlane_b32 s0, v9, s8
        v_readfirstlane_b32 s8, v2
        s_cbranch_scc0 1b
        ;;#ASMEND
    """)
    assert len(bad) == 1 and bad[0][4] == "v_readfirstlane_b32"
