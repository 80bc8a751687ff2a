"""scripts/check_isa.py's queue-value guard on synthetic disassembly: the value a
vs_queue_issue atomic returns may be read only by the v_readfirstlane behind its vmcnt wait, on
every control-flow path; a copy before the wait (what a register-allocator split would emit) fails."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import check_isa as C  # noqa: E402

HEAD = "0000000000001000 <_Zkern>:\n"


def body(*lines):
    out, addr = [HEAD], 0x1000
    for ln in lines:
        out.append(f"\t{ln:60s}// {addr:012X}: 00000000\n")
        addr += 4
    return "".join(out)


ISSUE = ("s_mov_b64 s[6:7], exec", "s_mov_b64 exec, 1", "global_atomic_add v7, v2, v3, s[4:5] sc0",
         "s_mov_b64 exec, s[6:7]")


def test_clean_consumer_passes():
    b = body(*ISSUE, "global_store_dwordx4 v1, v[8:11], s[0:1]", "s_waitcnt vmcnt(1)",
             "v_readfirstlane_b32 s9, v7", "s_endpgm")
    assert C.queue_value_hazards(b) == (1, [])


def test_copy_before_the_wait_is_flagged():
    b = body(*ISSUE, "v_mov_b32_e32 v40, v7", "s_waitcnt vmcnt(1)", "v_readfirstlane_b32 s9, v40", "s_endpgm")
    n, issues = C.queue_value_hazards(b)
    assert n == 1 and issues and "v_mov_b32_e32 v40, v7" in issues[0]


def test_readfirstlane_without_wait_is_flagged():
    b = body(*ISSUE, "v_readfirstlane_b32 s9, v7", "s_endpgm")
    assert "no vmcnt wait" in C.queue_value_hazards(b)[1][0]


def test_branch_paths_are_followed():
    # path 1 (branch taken) reads v7 early; the fall-through path is clean
    b = body(*ISSUE, "s_cbranch_scc1 2 <_Zkern+0x20>", "s_waitcnt vmcnt(0)", "v_readfirstlane_b32 s9, v7",
             "s_endpgm", "v_add_u32_e32 v1, v7, v1", "s_endpgm")
    # instruction 4 (0x1010) branches to +0x20 = the v_add reading v7
    n, issues = C.queue_value_hazards(b)
    assert n == 1 and any("v_add_u32_e32" in m for m in issues), issues


def test_non_queue_atomics_are_ignored():
    b = body("global_atomic_add v2, v0, v1, s[0:1] sc0", "v_cmp_eq_u32_e32 vcc, s2, v2", "s_endpgm")
    assert C.queue_value_hazards(b) == (0, [])
