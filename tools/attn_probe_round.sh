#!/bin/bash
# attention-backward probe variants (ab/libabp*.so, EEGF_AB_PROBE) against the in-tree build, interleaved
set -o pipefail
O=gpurun_out; mkdir -p $O; L=$O/${1:-abp}_attn_probe.log; : > $L
for rep in 1 2; do
  for v in base abp1 abp2 abp4 abp8; do
    lib=""; [ $v != base ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $L
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/attn_bench.py --nobits >> $L 2>&1 || exit 1
  done
done
grep -E "^==|attn_bwd|attn_fwd" $L
