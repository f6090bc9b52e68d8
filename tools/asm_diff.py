#!/usr/bin/env python3
"""Per-kernel instruction diff of two hipcc --cuda-device-only -S listings.

usage: python tools/asm_diff.py <old.s> <new.s> [kernel-substring]
Prints the kernels whose instruction streams differ (with old / new instruction counts): a
source refactor meant to be codegen-neutral should print none."""
import re
import sys


def kernels(path):
    d, cur = {}, None
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            d[cur] = []
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
        elif cur and line.startswith("\t") and not line.startswith("\t."):
            d[cur].append(line.split(";")[0].strip())
    return d


def main(argv):
    a, b = kernels(argv[0]), kernels(argv[1])
    filt = argv[2] if len(argv) > 2 else ""
    diff = 0
    for k in sorted(set(a) | set(b)):
        if filt not in k:
            continue
        if k not in a or k not in b:
            print("only in", "new" if k in b else "old", k)
            diff += 1
        elif a[k] != b[k]:
            print(f"DIFF {k}: {len(a[k])} -> {len(b[k])}")
            diff += 1
    print(f"{len(a)} / {len(b)} kernels, {diff} differ")


if __name__ == "__main__":
    main(sys.argv[1:])
