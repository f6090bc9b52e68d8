#!/usr/bin/env python3
"""ISA hazard lint over the gfx950 code objects inside ``libeegfusion.so``.

hipcc pads wait states around its own instructions but nothing inside an ``asm`` string, so a
hazard between compiler code and an asm statement (or inside one) is invisible until a kernel
returns wrong values on some waves of some launches (cdna_hip_programming.md "What hipcc does not
do", item 2).  This lint reads the shipped library, not the sources:

1. the ``.hip_fatbin`` section is split into its clang offload bundles (one per ``csrc/*.hip``
   translation unit) and every ``gfx950`` code object is disassembled with ``llvm-objdump``;
2. every vector-memory instruction (``global_*``, ``buffer_*``, ``scratch_*``, ``flat_*``) is walked
   backwards through straight-line code and branch predecessors, counting wait states (one per
   instruction, N + 1 for ``s_nop N``), and checked against the two hazards that touch LDS-DMA:

   * ``valu_sgpr_vmem`` — a VALU instruction writes an SGPR (``v_readfirstlane_b32``,
     ``v_readlane_b32`` restoring a spilled SGPR, a ``v_cmp`` / carry-out destination) that the VMEM
     instruction reads as address base, descriptor or soffset: 5 wait states required;
   * ``salu_m0_lds_dma`` — ``s_mov_b32 m0`` ahead of an LDS-DMA load (``*_lds_*`` / ``... lds``),
     which reads M0 as its LDS destination: 1 wait state required.

3. one source-level bug class that shows in the ISA: ``sext_low_word`` — ``s_bfe_i64 d, s, 0x200000``
   (sign-extend bits 0..31) whose result is ``s_or_b64``-ed within the next two instructions, i.e. a
   64-bit address rebuilt as ``hi << 32 | lo`` from a signed low word (``__builtin_amdgcn_readfirstlane``
   returns ``int``): bit 31 of the address then sets bits 32..63, an illegal address on roughly half
   of all buffers (r4o: a GPU memory-access fault in the weight-gradient GEMM).

4. ``async_load_touch`` — gemm4r issues its bias quads in one asm statement (``issue_bias8``: eight
   ``global_load_dwordx4`` at offsets 0 .. 448 with no wait) and retires them in a later one
   (``wait_vm_bias8``: ``s_cmp_eq_u32`` / ``s_cbranch_scc1`` / ``s_waitcnt vmcnt(8)``).  hipcc does not
   know the destination VGPRs are still being written, so every control-flow path from the issue to
   that wait is walked and any instruction naming a destination register is reported (a copy placed
   there reads in-flight data: the first build of the split did exactly that on one side of a branch).

5. ``mfma_d_read`` — an instruction that reads or writes an MFMA's destination (AGPRs or VGPRs; an
   MFMA taking it as srcC excepted) sooner after it than hipcc pads its own MFMAs (16x16x32 bf16: 8
   wait states, 16x16x4 f32: 10).  hipcc pads its own MFMAs, but the K-loops' MFMAs
   are asm statements, and the register allocator may place an accumulator copy right after one (it
   did when a 32-VGPR value was kept live across the last K-tile: wrong epilogue values).

6. ``mfma_src_write`` — a VALU write of a VGPR that an MFMA reads as srcA / srcB fewer than 2 wait states
   before it (hipcc rebuilt a constant operand of an asm MFMA with ``v_mov`` right before it).

usage: python tools/isa_lint.py [path/to/libeegfusion.so] [--all]
Exit status 1 when any hazard is found.  ``tests/test_isa_lint_cpu.py`` runs it on the built library.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile
from collections import Counter, defaultdict
from dataclasses import dataclass
from pathlib import Path

LLVM_BIN = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib" / "llvm" / "bin"
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
ARCH = "gfx950"

REQUIRED = {"valu_sgpr_vmem": 5, "salu_m0_lds_dma": 1}
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
SEXT32 = "0x200000"          # s_bfe_i64 operand: offset 0, width 32

# VALU mnemonics whose second operand is an SGPR destination (carry-out / scale flag)
_SDST1 = re.compile(r"^v_(add_co|sub_co|subrev_co|addc_co|subb_co|subbrev_co)_u32|^v_mad_(u64_u32|i64_i32)|"
                    r"^v_div_scale_f(32|64)")
_VMEM = re.compile(r"^(global|buffer|scratch|flat|tbuffer)_")
_LINE = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>")
_SREG = re.compile(r"^s\[(\d+):(\d+)\]$|^s(\d+)$")
_NAMED = {"vcc": ("vcc_lo", "vcc_hi"), "vcc_lo": ("vcc_lo",), "vcc_hi": ("vcc_hi",), "m0": ("m0",),
          "exec": ("exec_lo", "exec_hi"), "exec_lo": ("exec_lo",), "exec_hi": ("exec_hi",)}


@dataclass
class Inst:
    addr: int
    mnem: str
    ops: list
    text: str


@dataclass
class Finding:
    kind: str
    func: str
    addr: int
    inst: str
    writer: str
    states: int


def bundles(so: Path) -> list[bytes]:
    """gfx950 code objects of every offload bundle in the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as td:
        fb = Path(td) / "fatbin"
        subprocess.run([str(LLVM_BIN / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", str(so),
                        str(Path(td) / "stripped")], check=True, capture_output=True)
        data = fb.read_bytes()
    out, pos = [], 0
    while True:
        start = data.find(BUNDLE_MAGIC, pos)
        if start < 0:
            break
        n = struct.unpack_from("<Q", data, start + 24)[0]
        p = start + 32
        end = start + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            end = max(end, start + off + size)
            if triple.endswith(ARCH) and size:
                out.append(data[start + off:start + off + size])
        pos = max(end, start + len(BUNDLE_MAGIC))
    return out


def disassemble(code: bytes) -> dict[str, list[Inst]]:
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(code)
        f.flush()
        txt = subprocess.run([str(LLVM_BIN / "llvm-objdump"), "-d", "--no-show-raw-insn", f"--mcpu={ARCH}",
                              f.name], check=True, capture_output=True, text=True).stdout
    funcs: dict[str, list[Inst]] = {}
    cur = None
    for line in txt.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = funcs.setdefault(m.group(2), [])
            continue
        m = _LINE.match(line)
        if m and cur is not None:
            mnem, rest, addr = m.group(1), m.group(2).strip(), int(m.group(3), 16)
            ops = [o.strip().split()[0] for o in rest.split(",") if o.strip()] if rest else []
            text = f"{mnem} {rest}".strip()
            if mnem.startswith(("s_branch", "s_cbranch")):
                # the branch target sits in objdump's trailing comment ("// addr: enc <func+0x..>"); keep it
                # in the text, or no branch edge is ever followed
                t = _TARGET.search(line)
                if t:
                    text += f" <{t.group(1)}+0x{t.group(2)}>"
            cur.append(Inst(addr, mnem, ops, text))
    return funcs


def sregs(op: str) -> tuple:
    m = _SREG.match(op)
    if m:
        if m.group(3) is not None:
            return (f"s{m.group(3)}",)
        return tuple(f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1))
    return _NAMED.get(op, ())


def valu_sgpr_writes(ins: Inst) -> set:
    if not ins.mnem.startswith("v_") or not ins.ops:
        return set()
    w = set(sregs(ins.ops[0]))
    if len(ins.ops) > 1 and _SDST1.match(ins.mnem):
        w |= set(sregs(ins.ops[1]))
    if ins.mnem.startswith("v_cmpx"):
        w |= {"exec_lo", "exec_hi"}
    return w


def is_lds_dma(ins: Inst) -> bool:
    return bool(_VMEM.match(ins.mnem)) and ("_lds_" in ins.mnem or re.search(r"\blds\b", ins.text) is not None)


def vmem_sgpr_reads(ins: Inst) -> set:
    r = set()
    for op in ins.ops[1:] if not ins.mnem.startswith(("global_store", "buffer_store", "scratch_store", "flat_store",
                                                       "global_atomic", "buffer_atomic")) else ins.ops:
        r |= set(sregs(op))
    if is_lds_dma(ins):
        r.add("m0")
    return r


def states(ins: Inst) -> int:
    if ins.mnem == "s_nop":
        return int(ins.ops[0], 0) + 1 if ins.ops else 1
    return 1


def lint_function(name: str, insts: list[Inst]) -> list[Finding]:
    by_addr = {ins.addr: k for k, ins in enumerate(insts)}
    preds = defaultdict(list)               # index of a branch target -> indices of branches to it
    for k, ins in enumerate(insts):
        if ins.mnem.startswith(("s_branch", "s_cbranch")):
            m = _TARGET.search(ins.text)
            if m and insts:
                tgt = insts[0].addr + int(m.group(2), 16)
                if tgt in by_addr:
                    preds[by_addr[tgt]].append(k)
    out: list[Finding] = []
    for k, ins in enumerate(insts):
        if ins.mnem == "s_bfe_i64" and len(ins.ops) == 3 and ins.ops[2] == SEXT32:
            dst = set(sregs(ins.ops[0]))
            for p in insts[k + 1:k + 3]:
                if p.mnem == "s_or_b64" and dst & set().union(*(sregs(o) for o in p.ops[1:])):
                    out.append(Finding("sext_low_word", name, ins.addr, ins.text, p.text, 0))
                    break
        if not _VMEM.match(ins.mnem):
            continue
        reads = vmem_sgpr_reads(ins)
        if not reads:
            continue
        found = {}

        def walk(j: int, acc: int, seen: frozenset):
            # j: index of the instruction just before the point reached; acc: wait states between
            while j >= 0 and acc < REQUIRED["valu_sgpr_vmem"]:
                for b in preds.get(j + 1, ()):   # insts[j + 1] is a branch target: its branches too
                    if b != j and b not in seen:
                        walk(b - 1, acc + 1, seen | {b})
                p = insts[j]
                if p.mnem in ("s_branch", "s_endpgm", "s_setpc_b64"):
                    return                       # no fall-through from above an unconditional branch
                if valu_sgpr_writes(p) & reads:
                    found.setdefault("valu_sgpr_vmem", (acc, p.text))
                    return
                if is_lds_dma(ins) and p.mnem.startswith("s_") and p.ops and p.ops[0] == "m0" and \
                        acc < REQUIRED["salu_m0_lds_dma"]:
                    found.setdefault("salu_m0_lds_dma", (acc, p.text))
                acc += states(p)
                j -= 1

        walk(k - 1, 0, frozenset())
        for kind, (acc, wtext) in found.items():
            out.append(Finding(kind, name, ins.addr, ins.text, wtext, acc))
    return out


def vregs(text: str) -> set:
    out = set()
    for m in _VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def async_issue_blocks(insts: list[Inst]) -> list[tuple[int, set]]:
    """(index after the block, destination VGPRs) of every issue-only bias load block."""
    out = []
    for k in range(len(insts) - 8):
        blk = insts[k:k + 8]
        if not all(i.mnem == "global_load_dwordx4" for i in blk):
            continue
        if k > 0 and insts[k - 1].mnem == "global_load_dwordx4":
            continue
        offs = [int(m.group(1)) if (m := re.search(r"offset:(\d+)", i.text)) else 0 for i in blk]
        if offs != [64 * j for j in range(8)] or len({i.ops[1] for i in blk}) != 1:
            continue
        nxt = insts[k + 8]
        if nxt.mnem == "s_waitcnt" and "vmcnt" in nxt.text:
            continue                                # load_bias8: retired in the same statement
        out.append((k + 8, set().union(*(vregs(i.ops[0]) for i in blk))))
    return out


def lint_async(name: str, insts: list[Inst]) -> list[Finding]:
    by_addr = {ins.addr: k for k, ins in enumerate(insts)}
    out = []
    for start, dst in async_issue_blocks(insts):
        seen, stack, touches = set(), [start], []
        while stack:
            j = stack.pop()
            while j < len(insts) and j not in seen:
                seen.add(j)
                ins = insts[j]
                if ins.mnem == "s_cmp_eq_u32" and j + 2 < len(insts) and insts[j + 1].mnem == "s_cbranch_scc1" and \
                        insts[j + 2].mnem == "s_waitcnt" and "vmcnt" in insts[j + 2].text:
                    break                           # wait_vm_bias8: retired on this path
                if ins.mnem in ("s_endpgm", "s_setpc_b64"):
                    break
                if vregs(ins.text) & dst:
                    touches.append(ins)
                if ins.mnem.startswith(("s_branch", "s_cbranch")):
                    m = _TARGET.search(ins.text)
                    if m:
                        tgt = insts[0].addr + int(m.group(2), 16)
                        if tgt in by_addr:
                            stack.append(by_addr[tgt])
                    if ins.mnem == "s_branch":
                        break
                j += 1
        for t in touches[:1]:
            out.append(Finding("async_load_touch", name, insts[start - 8].addr, insts[start - 8].text, t.text, len(touches)))
    return out


_AREG = re.compile(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b")


def aregs(op: str) -> set:
    out = set()
    for m in _AREG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def lint_mfma_d(name: str, insts: list[Inst]) -> list[Finding]:
    """Any instruction but an MFMA taking it whole as srcC that reads or writes an MFMA's destination
    (AGPRs or VGPRs) within its result latency (straight-line look-ahead)."""
    out = []
    for k, ins in enumerate(insts):
        if not ins.mnem.startswith("v_mfma") or not ins.ops:
            continue
        d = ins.ops[0]
        dst = ("a", aregs(d)) if d.startswith("a") else ("v", vregs(d))
        if not dst[1]:
            continue
        # the result latency in wait states, as hipcc pads its own MFMAs on gfx950 (16x16x32 bf16: 8,
        # 16x16x4 f32: 10; 32x32 shapes taken as 16)
        need = 16 if "32x32" in ins.mnem else 8 if "16x16x32" in ins.mnem else 10 if "16x16x4" in ins.mnem else 12
        acc, j = 0, k + 1
        while j < len(insts) and acc < need:
            p = insts[j]
            if p.mnem in ("s_branch", "s_endpgm", "s_setpc_b64") or p.mnem.startswith("s_cbranch"):
                break
            rd = aregs if dst[0] == "a" else vregs
            if p.mnem.startswith("v_mfma"):
                # MFMA -> MFMA through srcC is interlocked (the accumulate chains; hipcc pads its own
                # other cases); through srcA / srcB it is a hazard
                if len(p.ops) > 2 and (rd(p.ops[1]) | rd(p.ops[2])) & dst[1]:
                    out.append(Finding("mfma_d_read", name, p.addr, p.text, ins.text, acc))
                    break
                acc += 1
                j += 1
                continue
            regs = rd(p.text)
            if regs & dst[1]:
                out.append(Finding("mfma_d_read", name, p.addr, p.text, ins.text, acc))
                break
            acc += states(p)
            j += 1
    return out


def lint_mfma_src(name: str, insts: list[Inst]) -> list[Finding]:
    """A VALU / VMEM / LDS write of a VGPR that the next MFMA reads as srcA / srcB within 2 wait states
    (hipcc pads its own MFMAs; an asm MFMA's operands it does not)."""
    out = []
    for k, ins in enumerate(insts):
        if not ins.mnem.startswith("v_mfma") or len(ins.ops) < 3:
            continue
        src = vregs(ins.ops[1]) | vregs(ins.ops[2])
        acc, j = 0, k - 1
        while j >= 0 and acc < 2:
            p = insts[j]
            if p.mnem in ("s_branch", "s_endpgm", "s_setpc_b64") or p.mnem.startswith("s_cbranch"):
                break
            if p.mnem.startswith("v_") and not p.mnem.startswith("v_mfma") and p.ops and vregs(p.ops[0]) & src:
                out.append(Finding("mfma_src_write", name, ins.addr, ins.text, p.text, acc))
                break
            acc += states(p)
            j -= 1
    return out


def lint(so: Path) -> tuple[list[Finding], Counter]:
    findings, vmem = [], Counter()
    for code in bundles(so):
        for name, insts in disassemble(code).items():
            findings += lint_function(name, insts)
            findings += lint_async(name, insts)
            findings += lint_mfma_d(name, insts)
            findings += lint_mfma_src(name, insts)
            vmem["async_issue"] += len(async_issue_blocks(insts))
            vmem["lds_dma"] += sum(is_lds_dma(i) for i in insts)
            vmem["vmem"] += sum(bool(_VMEM.match(i.mnem)) for i in insts)
    return findings, vmem


def main(argv: list[str]) -> int:
    args = [a for a in argv if not a.startswith("--")]
    so = Path(args[0]) if args else Path(__file__).resolve().parents[1] / "eeg-multimodal_amd" / "eegfusion" / \
        "libeegfusion.so"
    findings, vmem = lint(so)
    print(f"{so}: {vmem['vmem']} VMEM instructions ({vmem['lds_dma']} LDS-DMA, {vmem['async_issue']} split bias "
          f"loads), {len(findings)} hazards")
    per = Counter((f.kind, f.func) for f in findings)
    for (kind, func), n in per.most_common():
        print(f"  {n:5d}  {kind:16s} {func}")
    for f in findings if "--all" in argv else findings[:10]:
        print(f"  {f.kind}: {f.func} @0x{f.addr:x}: '{f.inst}' {f.states} state(s) after '{f.writer}'")
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
