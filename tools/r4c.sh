#!/bin/bash
# weight-gradient K-loop ceilings: in-tree vs the EEGF_W_PROBE builds (ab/libwp1..3.so)
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in new wp1 wp2 wp3; do
    lib=""; [ $v != new ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $O/r4c_wprobe.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/gemm_bench.py qkv_wgrad ffn1_wgrad ffn2_wgrad ao_wgrad >> $O/r4c_wprobe.log 2>&1 || exit 1
  done
done
echo done
