#!/bin/bash
# Interleaved A/B of GEMM library builds on selected tools/gemm_bench.py shapes (one process per
# build and round; the in-tree library is "cur").
# usage (on the box, repo root): bash tools/ab_gemm.sh <tag> <rounds> "<lib names under ab/ or cur>" <shape>...
set -o pipefail
TAG=$1 ROUNDS=$2 LIBS=$3; shift 3
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for r in $(seq 1 $ROUNDS); do
  for v in $LIBS; do
    # cur = the in-tree library; NAME=VALUE = the in-tree library under that environment variable; else ab/lib<v>.so
    # <lib>@NAME=VALUE: ab/lib<lib>.so under that environment variable
    lib=""; envs=""
    case $v in cur) ;; *@*) lib=ab/lib${v%%@*}.so; envs=${v#*@} ;; *=*) envs=$v ;; *) lib=ab/lib$v.so ;; esac
    echo "== $v $r" >> $O/${TAG}_gemm_ab.log
    env EEGF_LIB=$lib $envs timeout -k 10 200 python -u tools/gemm_bench.py "$@" >> $O/${TAG}_gemm_ab.log 2>&1 || exit 1
  done
done
python3 - "$O/${TAG}_gemm_ab.log" <<'PY'
import re, sys, collections
cur, res = None, collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"== (\S+) \d+", line)
    if m: cur = m.group(1); continue
    m = re.match(r"(\S+)\s+M=.*eegf\s+([\d.]+) us", line)
    if m: res[(m.group(1), cur)].append(float(m.group(2)))
shapes = sorted({s for s, _ in res}); libs = sorted({l for _, l in res})
print("shape".ljust(20) + "".join(l.rjust(12) for l in libs) + "   (median us)")
for s in shapes:
    print(s.ljust(20) + "".join(f"{sorted(res[(s, l)])[len(res[(s, l)]) // 2]:12.1f}" for l in libs))
PY
