cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/s2g_gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/attn_bench.py 0 0.1 > $O/s2g_attn.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/s2g_bench.json 2> $O/s2g_bench.err || exit 1
echo done
