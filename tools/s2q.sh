cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u tools/gemm_bench.py --ab --variants=0,1,4 qkv_wgrad ffn1_wgrad ffn2_wgrad ao_wgrad sq4k sq8k ffn2_fwd > $O/s2q_gb.log 2>&1 || exit 1
echo done
