cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $O/s2d_attn_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/attn_bench.py 0 0.1 > $O/s2d_attn.log 2>&1 || exit 1
echo done
