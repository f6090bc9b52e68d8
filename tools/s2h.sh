cd $GRAFT_REPO_ROOT
O=gpurun_out
EEGF_GEMM8=4 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/s2h_gemm8_tests.log 2>&1 || exit 1
EEGF_GEMM_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread >> $O/s2h_gemm8_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/gemm_bench.py --ab --variants=0,2,4,5 > $O/s2h_gemm_ab.log 2>&1 || exit 1
echo done
