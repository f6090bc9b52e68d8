cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/gemm_bench.py $GEMMS > gpurun_out/gb.log 2>&1 || exit 1
echo done
