#!/usr/bin/env python3
"""Waits, scratch traffic and stores inside the MFMA stretches of one kernel in a hipcc -S listing.

usage: python tools/kloop_waits.py <file.s> <kernel-substring>
A 'K-loop' instruction is one with an MFMA within W instructions on both sides (the unrolled
K-tiles are dense MFMA streams; the epilogue and out-of-line blocks are not).  A compiler wait
there (vmcnt, or a scratch reload) would stall on the in-flight LDS-DMA of the asm staging."""
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from asm_diff import kernels  # noqa: E402

W = 24


def main(path, sub):
    for k, L in kernels(path).items():
        if sub not in k:
            continue
        mf = [i for i, l in enumerate(L) if l.startswith("v_mfma")]
        inner = set()
        j = 0
        for i in range(len(L)):
            while j < len(mf) and mf[j] < i - W:
                j += 1
            if j < len(mf) and mf[j] <= i + W and any(i - W <= m < i for m in mf[j:j + 64]) and \
                    any(i < m <= i + W for m in mf[j:j + 64]):
                inner.add(i)
        cnt = {}
        for i in sorted(inner):
            l = L[i]
            for key, pat in (("vmcnt", r"^s_waitcnt.*vmcnt"), ("scratch", r"^scratch_"),
                             ("store", r"^global_store"), ("lgkm", r"^s_waitcnt lgkmcnt"),
                             ("readlane", r"^v_readlane"), ("writelane", r"^v_writelane")):
                if re.match(pat, l):
                    cnt.setdefault(key, []).append(l)
        print(k[:80], len(L), "instr", len(mf), "mfma")
        for key, v in cnt.items():
            print(f"  {key:9s} {len(v):4d}  e.g. {sorted(set(v))[:4]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
