#!/bin/bash
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
for v in base new; do
  lib=""; [ $v = base ] && lib=ab/libbase.so
  echo "== $v" >> $O/r3v_cos.log
  EEGF_LIB=$lib timeout -k 10 300 python -u tools/cos_probe.py 0.1 1,2,3,4,5,6,7,8 >> $O/r3v_cos.log 2>&1 || exit 1
done
echo done
