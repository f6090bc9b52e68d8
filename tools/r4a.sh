#!/bin/bash
# persistent-GEMM epilogue store cache policy: default vs nt vs sc1 vs sc0 sc1 (ab/libpol*.so)
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in new pol1 pol2 pol3; do
    lib=""; [ $v != new ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $O/r4a_pol.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/gemm_bench.py ffn1_fwd ffn1_fwd_gelu_d qkv_fwd ffn1_dgrad_acc >> $O/r4a_pol.log 2>&1 || exit 1
  done
done
echo done
