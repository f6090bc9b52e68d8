#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_production_gpu.py -q --timeout 120 --timeout-method thread > $O/r3w_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/r3w_tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/gemm4p_ab.py > $O/r3w_p_ab.log 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 400 python -u tools/step_ab.py --key 11 --values 2,3,1,0 > $O/r3w_step_ab.log 2>&1 || { echo "step ab failed"; exit 1; }
echo done
