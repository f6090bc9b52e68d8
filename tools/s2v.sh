cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "4wave" > $O/s2v_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/gemm_bench.py --ab --variants=0,4,8 qkv_wgrad ffn1_wgrad ffn2_wgrad ao_wgrad qkv_dgrad ffn1_dgrad ffn2_dgrad_plain ffn2_dgrad_dgelu ao_dgrad > $O/s2v_gb.log 2>&1 || exit 1
echo done
