#!/bin/bash
# beta-batched epilogue: GEMM tests, dgrad A/B (base = HEAD build in ab/libbase.so), step A/B
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 --timeout-method thread > $O/r3i_gemm_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/r3i_gemm_tests.log; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=ab/libbase.so
    echo "== $v gemm $rep" >> $O/r3i_ab.log
    EEGF_LIB=$lib timeout -k 10 200 python -u tools/gemm_bench.py ffn1_dgrad qkv_dgrad ao_dgrad ffn1_dgrad_acc qkv_dgrad_acc ao_dgrad_acc ffn2_dgrad_mulaux >> $O/r3i_ab.log 2>&1 || exit 1
  done
done
for rep in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=ab/libbase.so
    echo "== $v bench $rep" >> $O/r3i_ab.log
    EEGF_LIB=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 >> $O/r3i_ab.log 2>&1 || exit 1
  done
done
echo done
