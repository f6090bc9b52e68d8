"""List the s_waitcnt vmcnt instructions of one kernel in a hipcc --save-temps .s file, each with the
two instructions that follow it (finds compiler-inserted drains in glds-pipelined loops).
Usage: python tools/vmw.py <file.s> <mangled kernel name>"""
import sys

s = open(sys.argv[1]).read()
n = sys.argv[2]
i = s.index(n + ': ;')
j = s.index('.Lfunc_end', i)
L = s[i:j].split('\n')
for k, l in enumerate(L):
    if 's_waitcnt vmcnt' in l:
        nxt = [x.strip() for x in L[k + 1:k + 4] if x.strip() and not x.strip().startswith(';')]
        print(k, l.strip(), '|', ' / '.join(nxt[:2])[:120])
