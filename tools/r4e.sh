#!/bin/bash
# whole-128-B-line epilogue stores (in-tree) vs the half-line form (ab/libhalf.so)
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "persistent or gemm_big or epilogue" --timeout 120 --timeout-method thread > $O/r4e_tests.log 2>&1 || { tail -5 $O/r4e_tests.log; exit 1; }
tail -1 $O/r4e_tests.log
for rep in 1 2; do
  for v in new half; do
    lib=""; [ $v != new ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $O/r4e_gemm.log
    EEGF_LIB=$lib timeout -k 10 120 python -u tools/gemm_bench.py qkv_fwd ao_fwd ffn1_fwd ffn1_fwd_gelu_d ffn2_fwd >> $O/r4e_gemm.log 2>&1 || exit 1
  done
done
for rep in 1 2 3; do
  for v in new half; do
    lib=""; [ $v != new ] && lib=ab/lib$v.so
    echo "== $v $rep" >> $O/r4e_bench.log
    EEGF_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 >> $O/r4e_bench.log 2>&1 || exit 1
  done
done
echo done
