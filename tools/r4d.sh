#!/bin/bash
# weight-gradient L2 prefetch (eegf_tune key 13 / EEGF_WGRAD_PF = distance beyond the LDS ring)
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "prefetch_bitwise and 3072" --timeout 60 --timeout-method thread > $O/r4d_tests1.log 2>&1 || { tail -3 $O/r4d_tests1.log; exit 1; }
EEGF_WGRAD_PF=6 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > $O/r4d_tests.log 2>&1 || { tail -3 $O/r4d_tests.log; exit 1; }
tail -1 $O/r4d_tests.log
for rep in 1 2; do
  for d in 0 2 4 8 12; do
    echo "== pf $d $rep" >> $O/r4d_pf.log
    EEGF_WGRAD_PF=$d timeout -k 10 120 python -u tools/gemm_bench.py qkv_wgrad ffn1_wgrad ffn2_wgrad ao_wgrad >> $O/r4d_pf.log 2>&1 || exit 1
  done
done
echo done
