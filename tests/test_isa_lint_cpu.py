"""ISA hazard lint of the shipped library (no GPU needed).

The production LDS-DMA statements (``common.h`` ``glds16_asm_s`` / ``glds16_asm_sa``) read a 64-bit
base from SGPRs that a VALU often writes just before them (``v_readfirstlane_b32``, or a
``v_readlane_b32`` restoring a spilled SGPR).  A VMEM instruction reading such an SGPR needs 5 wait
states, which hipcc never inserts inside an asm string; with fewer, some waves of some launches load
from a stale base with no fault.  ``tools/isa_lint.py`` disassembles every gfx950 code object of
``libeegfusion.so`` and walks back from each VMEM instruction; this test requires zero findings.
"""
from pathlib import Path

import pytest

from tools import isa_lint

LIB = Path(__file__).resolve().parents[1] / "eeg-multimodal_amd" / "eegfusion" / "libeegfusion.so"


def _inst(addr, text):
    mnem, _, rest = text.partition(" ")
    ops = [o.strip().split()[0] for o in rest.split(",") if o.strip()]
    return isa_lint.Inst(addr, mnem, ops, text)


def _prog(*texts):
    return [_inst(4 * k, t) for k, t in enumerate(texts)]


def test_lint_flags_readfirstlane_two_states_before_dma():
    """The exact round-3 pattern: 2 wait states between the VALU write and the DMA base read."""
    f = isa_lint.lint_function("k", _prog(
        "v_readfirstlane_b32 s1, v7", "v_readfirstlane_b32 s0, v6", "s_mov_b32 m0, s3", "s_nop 0",
        "global_load_lds_dwordx4 v1, s[0:1]"))
    assert [(x.kind, x.states) for x in f] == [("valu_sgpr_vmem", 2)]


def test_lint_counts_nops_and_accepts_five_states():
    ok = isa_lint.lint_function("k", _prog(
        "v_readfirstlane_b32 s0, v6", "s_mov_b32 m0, s3", "s_nop 3", "global_load_lds_dwordx4 v1, s[0:1]"))
    assert ok == []
    short = isa_lint.lint_function("k", _prog(
        "v_readlane_b32 s61, v242, 2", "s_mov_b32 m0, s3", "s_nop 2", "global_load_lds_dwordx4 v1, s[60:61]"))
    assert [(x.kind, x.states) for x in short] == [("valu_sgpr_vmem", 4)]


def test_lint_m0_and_carry_and_branch_predecessors():
    m0 = isa_lint.lint_function("k", _prog("s_mov_b32 m0, s3", "global_load_lds_dwordx4 v1, off"))
    assert [x.kind for x in m0] == ["salu_m0_lds_dma"]
    # a carry-out SGPR of v_mad_u64_u32 read as buffer soffset
    carry = isa_lint.lint_function("k", _prog(
        "v_mad_u64_u32 v[4:5], s[8:9], v3, s0, v[0:1]", "buffer_load_dword v1, v2, s[4:7], s8 offen"))
    assert [x.kind for x in carry] == ["valu_sgpr_vmem"]
    # the writer sits before a branch that jumps straight to the load (target = function start + 0x10)
    br = [_inst(0, "v_readfirstlane_b32 s0, v6"), _inst(4, "s_branch 2 <k+0x10>"),
          _inst(8, "s_nop 7"), _inst(12, "s_nop 7"), _inst(16, "global_load_dword v1, v2, s[0:1]")]
    assert [(x.kind, x.states) for x in isa_lint.lint_function("k", br)] == [("valu_sgpr_vmem", 1)]


def test_lint_flags_sign_extended_low_word_of_an_address():
    """r4o: ``hi << 32 | readfirstlane(lo)`` (an ``int``) compiled to a sign-extend + OR; bit 31 of the
    address set the whole high word and the weight-gradient GEMM faulted the GPU."""
    bad = isa_lint.lint_function("k", _prog(
        "s_add_u32 s54, s52, s70", "s_bfe_i64 s[54:55], s[54:55], 0x200000", "s_or_b64 s[56:57], s[54:55], s[44:45]"))
    assert [x.kind for x in bad] == ["sext_low_word"]
    # the same extract feeding something else (a sign-extended int64 index) is not the pattern
    ok = isa_lint.lint_function("k", _prog(
        "s_bfe_i64 s[4:5], s[4:5], 0x200000", "s_lshl_b64 s[4:5], s[4:5], 1", "s_add_u32 s0, s0, s4"))
    assert ok == []


def _bias_issue():
    return [f"global_load_dwordx4 v[{4 * j}:{4 * j + 3}], v[40:41], off" + (f" offset:{64 * j}" if j else "")
            for j in range(8)]


_WAIT = ["s_cmp_eq_u32 s4, 0", "s_cbranch_scc1 1 <k+0x0>", "s_waitcnt vmcnt(8)"]


def test_lint_flags_a_copy_of_in_flight_bias_registers():
    """gemm4r's split bias load: a copy of a destination register between the issue statement and its
    counted wait reads data still being loaded (the first build of the split did that on one side of a
    branch); MFMAs and other registers in between are fine."""
    ok = isa_lint.lint_async("k", _prog(*_bias_issue(), "v_mfma_f32_16x16x32_bf16 a[0:3], v[48:51], v[52:55], a[0:3]",
                                        *_WAIT, "v_mov_b64_e32 v[60:61], v[4:5]"))
    assert ok == []
    bad = isa_lint.lint_async("k", _prog(*_bias_issue(), "v_mov_b64_e32 v[60:61], v[4:5]", *_WAIT))
    assert [x.kind for x in bad] == ["async_load_touch"]
    # load_bias8 (issue + wait in one statement) is not a split load
    assert isa_lint.async_issue_blocks(_prog(*_bias_issue(), "s_waitcnt vmcnt(0)", "v_mov_b32 v60, v4")) == []


def test_lint_flags_an_accumulator_read_inside_the_mfma_latency():
    """An asm MFMA is opaque to hipcc's hazard recognizer: a register-allocator copy of its accumulator
    one state later read stale values (the first split-bias build of gemm4r)."""
    mfma = "v_mfma_f32_16x16x32_bf16 a[8:11], v[96:99], v[248:251], a[8:11]"
    bad = isa_lint.lint_mfma_d("k", _prog(mfma, "s_nop 0", "v_accvgpr_read_b32 v33, a11"))
    assert [(x.kind, x.states) for x in bad] == [("mfma_d_read", 1)]
    ok = isa_lint.lint_mfma_d("k", _prog(mfma, "s_nop 7", "s_nop 7", "v_accvgpr_read_b32 v33, a11"))
    assert ok == []
    other = isa_lint.lint_mfma_d("k", _prog(mfma, "v_accvgpr_read_b32 v33, a12"))     # not the MFMA's D
    assert other == []


def test_lint_flags_a_fresh_vgpr_source_of_an_mfma():
    """hipcc rebuilt the ones operand of the weight-gradient row-sum MFMA (an asm statement) with v_mov
    right before it: the MFMA read a half-written operand (NaN bias gradients)."""
    bad = isa_lint.lint_mfma_src("k", _prog("v_mov_b32_e32 v153, v150",
                                            "v_mfma_f32_16x16x32_bf16 v[78:81], v[150:153], v[34:37], v[78:81]"))
    assert [x.kind for x in bad] == ["mfma_src_write"]
    ok = isa_lint.lint_mfma_src("k", _prog("v_mov_b32_e32 v153, v150", "s_nop 2",
                                           "v_mfma_f32_16x16x32_bf16 v[78:81], v[150:153], v[34:37], v[78:81]"))
    assert ok == []
    # a VGPR accumulator read by VALU inside the result latency
    d = isa_lint.lint_mfma_d("k", _prog("v_mfma_f32_16x16x32_bf16 v[78:81], v[150:153], v[34:37], v[78:81]",
                                        "v_mov_b32_e32 v0, v78"))
    assert [x.kind for x in d] == ["mfma_d_read"]


@pytest.mark.skipif(not LIB.exists(), reason="libeegfusion.so not built (run __graft_entry__.build())")
def test_shipped_library_has_no_vmem_sgpr_hazards():
    findings, counts = isa_lint.lint(LIB)
    assert counts["lds_dma"] > 1000, counts          # the production GEMM / attention DMA rings are present
    assert findings == [], "\n".join(
        f"{f.kind}: {f.func} @0x{f.addr:x} '{f.inst}' {f.states} states after '{f.writer}'" for f in findings[:20])
