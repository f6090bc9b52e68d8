#!/usr/bin/env python3
"""Issue budget of a deferred GEMM epilogue, from the persistent kernels' own ISA (the VERDICT r5 probe of
the "hide the epilogue in the next tile's K-loop" design).

usage: python tools/epi_budget.py <gemm_big.s> [K]
  <gemm_big.s>: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S csrc/gemm_big.hip
  K: the contraction length of the shape (768: QKV / out-projection / FFN1; default)

For every gemm4r instantiation it reads
  * the steady-state K-loop (the loop whose body holds one K-tile pair, 128 MFMAs per wave) and prices
    its non-MFMA instructions in issue cycles (MI355X_MICROARCH.md, per-instruction constants: a
    v_mfma_f32_16x16x32_bf16 holds the SIMD's vector issue for 8 of its 16 cycles; transcendental VALU 8,
    other VALU / LDS / VMEM / SALU 4, s_nop n 4 (n + 1); waits and barriers 0);
  * the epilogue (from the three s_nop 7 that close the K-loop to the next tile's first MFMA), priced the
    same way;
and prints, per 256 x 256 tile and wave, the MFMA-gap issue cycles the K-loop leaves free (16 - 8 - its own
overhead per MFMA, times K / 32 x 64 MFMAs) against the epilogue's issue cycles: the fraction of the
epilogue a deferred schedule could hide at best, before any register cost.
"""
import re
import sys

TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_")


def cost(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return 8
    if op.startswith(("s_waitcnt", "s_barrier", "s_setprio", "s_sched")):
        return 0
    if op == "s_nop":
        return 4 * (int(ins.split()[1], 0) + 1)
    if TRANS.match(op):
        return 8
    return 4


def body(lines, name):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^\S+:", l) and name in l and not l.startswith("."):
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"{name} not found")


def instrs(block):
    return [x.strip() for x in block if x.startswith("\t") and not x.strip().startswith((".", ";"))]


def main():
    path = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    lines = open(path).read().splitlines()
    names = sorted({m.group(1) for l in lines for m in [re.match(r"^(_Z\S*gemm4r_kernel\S*):", l)] if m})
    mf_per_tile = (K // 32) * 64
    print(f"K = {K}: {mf_per_tile} MFMAs per wave and 256 x 256 tile\n")
    print("| kernel | K-loop overhead cyc/MFMA | free gap cyc per tile | epilogue instrs | epilogue issue cyc "
          "| transcendental | hideable at best |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for nm in names:
        b = body(lines, nm)
        lab = {m.group(1): i for i, l in enumerate(b) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
        loop = None
        for i, l in enumerate(b):
            m = re.match(r"^\s+s_c?branch\w*\s+(\.LBB\w+)", l)
            if m and m.group(1) in lab and lab[m.group(1)] < i:
                ins = instrs(b[lab[m.group(1)]:i + 1])
                if sum(x.startswith("v_mfma") for x in ins) == 128:
                    loop = ins
                    break
        ins = instrs(b)
        mk = [i for i in range(len(ins) - 2) if all(ins[i + d].startswith("s_nop 7") for d in range(3))]
        if loop is None or not mk:
            continue
        j = mk[0] + 3
        while j < len(ins) and not ins[j].startswith(("v_mfma", "s_endpgm")):
            j += 1
        epi = ins[mk[0] + 3:j]
        over = sum(cost(x) for x in loop if not x.startswith("v_mfma")) / 128.0
        free = max(0.0, 16 - 8 - over) * mf_per_tile
        ecyc = sum(cost(x) for x in epi)
        ntr = sum(1 for x in epi if TRANS.match(x.split()[0]))
        short = re.sub(r"^_ZN12_GLOBAL__N_113", "", nm)
        print(f"| `{short}` | {over:.2f} | {free:.0f} | {len(epi)} | {ecyc} | {ntr} | {min(1.0, free / ecyc):.2f} |")


if __name__ == "__main__":
    main()
