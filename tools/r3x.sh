#!/bin/bash
# widened (permlane16-swap, 16-B) persistent-GEMM epilogue stores: GEMM tests, persistent-vs-default bit
# identity + timing, interleaved step A/B against the HEAD build (ab/libprev.so)
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_production_gpu.py -q --timeout 200 --timeout-method thread > $O/r3x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r3x_tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/gemm4p_ab.py > $O/r3x_p_ab.log 2>&1 || exit 1
for rep in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=ab/libprev.so
    echo "== $v bench $rep" >> $O/r3x_ab.log
    EEGF_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 >> $O/r3x_ab.log 2>&1 || exit 1
  done
done
echo done
