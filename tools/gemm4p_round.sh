#!/bin/bash
# persistent-GEMM session: kernel tests, interleaved A/B per shape, bench with the key off / on
# usage (on the box): bash tools/gemm4p_round.sh <tag>
set -o pipefail
TAG=${1:-r3}
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k persistent --timeout 120 --timeout-method thread > $O/${TAG}_p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/gemm4p_ab.py > $O/${TAG}_p_ab.log 2>&1 || { echo "ab failed"; exit 1; }
for v in 0 2 1; do
  EEGF_GEMM4P=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > $O/${TAG}_p_bench$v.json 2> $O/${TAG}_p_bench$v.err || { echo "bench $v failed"; exit 1; }
  echo "bench $v done"
done
