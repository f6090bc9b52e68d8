#!/usr/bin/env python3
"""Per-class instruction counts of one kernel in a hipcc --cuda-device-only -S listing.

usage: python tools/isa_classes.py <file.s> <kernel-name-substring> [--loop]
Classes: MFMA, transcendental VALU (exp/log/rcp/rsq/sqrt), 64-bit integer multiply (v_mad_u64_u32,
the Philox rounds), 32-bit integer multiply-high/low, bit ops (bitop3/xor/and/or/shifts/bfe/perm/
alignbit), f32 VALU arithmetic (add/mul/fma/max/min), conversions / packs (cvt, pk), lane exchange
(DPP / permlane / bpermute / readlane), LDS, global / buffer memory, scalar, waits / barriers /
nops.  Static counts over the kernel body (the steady-state loop dominates both kernels), so they
rank instruction classes, not cycles."""
import re
import sys
from collections import Counter

CLASSES = [
    ("mfma", r"^v_mfma"),
    ("transcendental", r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_"),
    ("mul_u64 (Philox)", r"^v_mad_u64_u32|^v_mad_i64_i32"),
    ("mul_u32", r"^v_mul_(hi|lo)_[ui]32|^v_mul_u32_u24|^v_mad_u32_u24|^v_mul_hi_u32_u24"),
    ("bitops", r"^v_(bitop3|xor|and|or|not|lshl|lshr|ashr|bfe|bfi|perm|alignbit|alignbyte|lshl_or|and_or|or3|xad|xor3|lshl_add|add_lshl)"),
    ("int add/sub/cmp/sel", r"^v_(add|sub|subrev)_(u32|i32|co_u32|nc_u32|co_ci_u32|i16|u16)|^v_cmp|^v_cndmask|^v_min_u32|^v_max_u32|^v_sad|^v_pk_(add|sub|min|max)_u16|^v_pk_(add|sub)_i16|^v_mad_u32"),
    ("f32 arith", r"^v_(add|sub|mul|fma|fmac|max|min|max3|min3|med3|mac|ldexp|fmamk|fmaak)_f32|^v_pk_(fma|mul|add)_f32|^v_dot2"),
    ("convert/pack", r"^v_cvt|^v_pk_|^v_pack"),
    ("lane xchg", r"^v_(mov_b32_dpp|permlane|readlane|readfirstlane|writelane)|^ds_(bpermute|permute|swizzle)|_dpp"),
    ("vgpr mov", r"^v_(mov|accvgpr)"),
    ("lds", r"^ds_"),
    ("global/buffer", r"^(global|buffer|flat|scratch)_"),
    ("scalar", r"^s_(?!waitcnt|barrier|nop|setprio|sleep|cbranch|branch|endpgm)"),
    ("wait/barrier/nop/prio", r"^s_(waitcnt|barrier|nop|setprio|sleep)"),
    ("branch", r"^s_(cbranch|branch|endpgm)"),
]


def body(lines, name):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^\S+:\s*(;.*)?$", l) and name in l and not l.startswith("."):
            start = i
        elif start is not None and (l.startswith(".Lfunc_end") or l.strip() == "s_endpgm"):
            return lines[start:i + 1]
    raise SystemExit(f"kernel {name!r} not found")


def classify(insts):
    c = Counter()
    for ins in insts:
        for cls, pat in CLASSES:
            if re.match(pat, ins):
                c[cls] += 1
                break
        else:
            c["other:" + ins.split("_")[0]] += 1
    return c


def main():
    f, name = sys.argv[1], sys.argv[2]
    lines = open(f).read().splitlines()
    b = body(lines, name)
    insts = [l.strip().split()[0] for l in b if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    c = classify(insts)
    mf = c.get("mfma", 0) or 1
    print(f"{name}: {len(insts)} instructions, {c.get('mfma', 0)} MFMA")
    print(f"| class | count | per MFMA |\n|---|---:|---:|")
    for k, v in c.most_common():
        print(f"| {k} | {v} | {v / mf:.2f} |")


if __name__ == "__main__":
    main()
