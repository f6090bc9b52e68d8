cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "4wave" > $O/s2x_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/gemm_bench.py --ab --variants=4,8 sq4k ffn2_fwd qkv_fwd ffn1_fwd_nogelu qkv_dgrad ffn1_dgrad ffn1_wgrad qkv_wgrad > $O/s2x_gb.log 2>&1 || exit 1
echo done
