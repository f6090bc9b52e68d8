#!/bin/bash
# packed softmax fma/add in the L = 256 attention forward vs HEAD (ab/libprevat.so): 8 alternating
# processes, 100 launches each
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for rep in 1 2 3 4 5 6 7 8; do
  for v in new prevat; do
    lib=""; [ $v != new ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $O/r4h_attn2.log
    EEGF_LIB=$lib timeout -k 10 120 python -u -c "import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import attn_bench as t; t.main(p=0.1, iters=100, use_bits=False)" >> $O/r4h_attn2.log 2>&1 || exit 1
  done
done
echo done
