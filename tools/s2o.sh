cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/s2o_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/gemm_bench.py --ab --variants=0,4,6 ffn1_fwd ffn1_fwd_nogelu qkv_fwd ao_fwd ffn2_fwd ffn2_dgrad_dgelu ffn2_dgrad_plain ffn1_dgrad qkv_dgrad ao_dgrad > $O/s2o_gb.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gemm_bench.py qkv_wgrad ffn1_wgrad ffn2_wgrad ao_wgrad >> $O/s2o_gb.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_bench.py 0.1 > $O/s2o_attn.log 2>&1 || exit 1
echo done
