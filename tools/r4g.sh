#!/bin/bash
# 32-bit-call Philox in the L = 256 attention kernels vs HEAD's (ab/libprevat.so)
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_dropout_parity_gpu.py -x -q -k "attn or attention or dropout" --timeout 120 --timeout-method thread > $O/r4g_tests.log 2>&1 || { tail -5 $O/r4g_tests.log; exit 1; }
tail -1 $O/r4g_tests.log
for rep in 1 2 3; do
  for v in new prevat; do
    lib=""; [ $v != new ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $O/r4g_attn.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/attn_bench.py --nobits >> $O/r4g_attn.log 2>&1 || exit 1
  done
done
echo done
