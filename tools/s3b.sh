cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "acs or 4wave" > $O/s3b_tests.log 2>&1 || exit 1
echo done
