cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "4wave" > $O/s2t_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/gemm_bench.py --ab --variants=0,4,8 sq4k sq8k ffn2_fwd qkv_fwd ffn1_fwd_nogelu ffn1_fwd ao_fwd > $O/s2t_gb.log 2>&1 || exit 1
echo done
