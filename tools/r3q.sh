#!/bin/bash
# persistent-GEMM epilogue anatomy: normal vs no stores (exp1) vs no GELU VALU (exp2)
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in new exp1 exp2; do
    lib=""; [ $v != new ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $O/r3q_exp.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/gemm_bench.py ffn1_fwd ffn1_fwd_gelu_d ffn1_fwd_nogelu >> $O/r3q_exp.log 2>&1 || exit 1
  done
done
echo done
