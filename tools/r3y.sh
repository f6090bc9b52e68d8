#!/bin/bash
# persistent-GEMM routing (eegf_tune key 11) on the whole step: 2 (won set), 3 (+ aux product), 1 (every eligible)
set -o pipefail
O=gpurun_out; mkdir -p $O; export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/step_ab.py --key 11 --values 2,3,1 --rounds 7 > $O/r3y_step_ab.log 2>&1 || { echo "step ab failed"; exit 1; }
echo done
