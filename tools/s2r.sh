cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u tools/gemm_bench.py --ab --variants=4,7,0 sq4k ffn2_fwd qkv_fwd ffn1_fwd_nogelu qkv_dgrad ffn1_wgrad > $O/s2r_gb.log 2>&1 || exit 1
echo done
