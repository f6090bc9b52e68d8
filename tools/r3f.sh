#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $O/r3f_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/r3f_gpu_tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/gemm4p_ab.py > $O/r3f_p_ab.log 2>&1 || { echo "ab failed"; exit 1; }
for v in 0 2 1; do
  EEGF_GEMM4P=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > $O/r3f_p_bench$v.json 2> $O/r3f_p_bench$v.err || { echo "bench $v failed"; exit 1; }
  echo "bench $v done"
done
