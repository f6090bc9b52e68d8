#!/bin/bash
# non-temporal persistent-GEMM epilogue stores (eegf_tune key 12) on the whole step
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -k persistent --timeout 120 --timeout-method thread > $O/r4b_tests.log 2>&1; rc=$?; tail -1 $O/r4b_tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 500 python -u tools/step_ab.py --key 12 --values 0,1 --rounds 7 > $O/r4b_step_ab.log 2>&1 || { echo "step ab failed"; exit 1; }
echo done
