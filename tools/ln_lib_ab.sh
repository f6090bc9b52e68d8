#!/bin/bash
# LayerNorm A/B of ab/libbase.so against the in-tree library: tools/ln_bench.py alternating, then the step.
# usage (on the box, repo root): bash tools/ln_lib_ab.sh <tag>
set -o pipefail
TAG=${1:-lnab}; O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=ab/libbase.so
    echo "== $v $r" >> $O/${TAG}_ln.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/ln_bench.py >> $O/${TAG}_ln.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/${TAG}_ln.log | grep "==\|rpw 16\|rpw 32"
