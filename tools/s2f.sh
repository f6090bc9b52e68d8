cd $GRAFT_REPO_ROOT
O=gpurun_out
for m in 3 0; do EEGF_ATTN256=$m timeout -k 10 120 python -u tools/attn_bench.py 0.1 >> $O/s2f_attn.log 2>&1 || exit 1; done
echo done
