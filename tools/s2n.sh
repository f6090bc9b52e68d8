cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "persistent or big" > $O/s2n_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_bench.py --ab --variants=4,6 ffn1_fwd ffn1_fwd_nogelu qkv_fwd ao_fwd ffn2_fwd ffn2_dgrad_dgelu ffn2_dgrad_plain ffn1_dgrad qkv_dgrad ao_dgrad > $O/s2n_gb.log 2>&1 || exit 1
echo done
