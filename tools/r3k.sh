#!/bin/bash
# attention forward rewrite: attention tests, then interleaved attn_bench base (ab/libbase.so) / new
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dropout_parity_gpu.py tests/test_determinism_gpu.py -q -k "attention or dropout or determin" --timeout 120 --timeout-method thread > $O/r3k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r3k_tests.log; [ $rc -le 1 ] || exit 1
for rep in 1 2 3; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=ab/libbase.so
    echo "== $v attn $rep" >> $O/r3k_ab.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/attn_bench.py 0 0.1 --nobits >> $O/r3k_ab.log 2>&1 || exit 1
  done
done
echo done
