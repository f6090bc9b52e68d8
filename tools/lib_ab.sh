#!/bin/bash
# A/B of two builds of libeegfusion.so on the GPU box: ab/libbase.so (a reference build of an older
# tree, made with `git worktree` + eegfusion.build) against the in-tree library, interleaved so clock
# and box drift hit both.  usage (on the box, repo root): bash tools/lib_ab.sh <tag> [bench|gemm|attn]...
set -o pipefail
TAG=${1:-ab}
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {   # run <label> <lib or ""> <cmd...>
  local label=$1 lib=$2; shift 2
  echo "== $label" >> $O/${TAG}_ab.log
  EEGF_LIB=$lib timeout -k 10 240 "$@" >> $O/${TAG}_ab.log 2>&1
}
for s in "${@:2}"; do
  for rep in 1 2; do
    case $s in
      bench) run "base bench $rep" ab/libbase.so python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 || exit 1
             run "new bench $rep" "" python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 || exit 1 ;;
      gemm) run "base gemm $rep" ab/libbase.so python -u tools/gemm_bench.py || exit 1
            run "new gemm $rep" "" python -u tools/gemm_bench.py || exit 1 ;;
      attn) run "base attn $rep" ab/libbase.so python -u tools/attn_bench.py || exit 1
            run "new attn $rep" "" python -u tools/attn_bench.py || exit 1 ;;
    esac
  done
done
echo "[lib_ab] done"
